"""Producer-side batching: the reference's ``ProducerClient.produce`` with the
messages of many calls sent to the engine as ONE batch.

The reference sends one message per RPC and one Raft entry per message:
``ProducerClientImpl.produce(topic, message)`` picks a partition with ``RoundRobinSelector``
(``mq-common/src/main/java/partition/selector/RoundRobinSelector.java:17-31``:
``Math.abs(counter.getAndIncrement()) % partitions.size()``, one counter per topic) and calls
``PartitionClient.sendMessage`` (``PartitionClient.java:39-45``: a ``MessageAppendRequest`` holding
that single message). ``ProducerClient`` here keeps the call, the partition choice and the errors
("Topic not found: <topic>") but queues the request; the queue goes to the broker's batched
append processor (``PartitionBroker.process_append``, one ``rmq_append``) when it holds
``batch_records`` messages, when the oldest queued message is ``linger_s`` old at the next call,
or on ``flush()`` / ``close()``. Each call gets a ``ProduceResult`` that resolves with the
request's ``MessageAppendResponse`` (success only once committed, as in the reference).
"""
from __future__ import annotations

import time

from .state_machine import MessageAppendRequest, MessageAppendResponse, PartitionBroker


class ProduceResult:
    """The response of one produce call, known after the batch holding it was applied."""

    def __init__(self, topic: str, partition_id: int):
        self.topic = topic
        self.partition_id = partition_id
        self.response: MessageAppendResponse | None = None

    def done(self) -> bool:
        return self.response is not None

    def isSuccess(self) -> bool:
        return self.response is not None and self.response.isSuccess()

    def getErrorMsg(self):
        return None if self.response is None else self.response.getErrorMsg()


def _java_abs_mod(counter: int, n: int) -> int:
    """Math.abs(int) % n with Java int wrap-around (abs(MIN_VALUE) stays negative)."""
    c = ((counter + (1 << 31)) % (1 << 32)) - (1 << 31)
    a = c if c >= 0 else (c if c == -(1 << 31) else -c)
    r = abs(a) % n
    return r if a >= 0 else -r


class ProducerClient:
    """``ProducerClient.produce(topic, message)`` over a ``PartitionBroker``, batched."""

    def __init__(self, broker: PartitionBroker, partitions_per_topic: dict[str, int], *,
                 batch_records: int = 65536, linger_s: float | None = None):
        self.broker = broker
        self.partitions = dict(partitions_per_topic)
        self.batch_records = int(batch_records)
        self.linger_s = linger_s
        self.counters: dict[str, int] = {}  # RoundRobinSelector.topicCounters
        self.queue: list[tuple[MessageAppendRequest, ProduceResult]] = []
        self.oldest = 0.0
        self.batches = 0

    def select_partition(self, topic: str) -> int:
        n = self.partitions[topic]
        c = self.counters.get(topic, 0)
        self.counters[topic] = c + 1
        idx = _java_abs_mod(c, n)
        if idx < 0:  # the reference's List.get(negative) throws here
            raise IndexError(f"RoundRobinSelector index {idx} for topic {topic}")
        return idx

    def produce(self, topic: str, message) -> ProduceResult:
        n = self.partitions.get(topic)
        if n is None:
            raise RuntimeError(f"Topic not found: {topic}")
        if n == 0:
            raise RuntimeError(f"No partitions found for topic: {topic}")
        pid = self.select_partition(topic)
        res = ProduceResult(topic, pid)
        if not self.queue:
            self.oldest = time.monotonic()
        self.queue.append((MessageAppendRequest([message], topic, pid), res))
        if len(self.queue) >= self.batch_records or (
                self.linger_s is not None and time.monotonic() - self.oldest >= self.linger_s):
            self.flush()
        return res

    def flush(self) -> list[ProduceResult]:
        """Send the queued requests as one engine batch; returns their results."""
        if not self.queue:
            return []
        q, self.queue = self.queue, []
        resp = self.broker.process_append([r for r, _ in q])
        self.batches += 1
        for (_, res), rsp in zip(q, resp):
            res.response = rsp
        return [res for _, res in q]

    def close(self) -> None:
        self.flush()
