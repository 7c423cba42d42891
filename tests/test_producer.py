"""Producer-side batching (ripplemq_amd/producer.py) against the reference model.

The sample producer's stream (sample-producer/src/main/java/org/example/Main.java:31-37: produce
10k messages to one topic through ProducerClient.produce, RoundRobinSelector choosing the
partition) goes through the batching client: every partition's log must hold exactly what
tests/refmodel.py's one-message-per-request broker holds, in the same order, and the number of
engine batches is the number of flushes. CPU: the oracle's handle; GPU: the HIP engine.
"""
import numpy as np
import pytest

from refmodel import Broker
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.producer import ProducerClient, _java_abs_mod
from ripplemq_amd.state_machine import MessageBatchReadRequest, PartitionBroker, PartitionDirectory

TOPIC = "topic1"


def _flow(make_engine, P=3, n=10_000, batch=1000):
    d = PartitionDirectory({TOPIC: P, "other": 2}, max_consumers=2)
    cfg = EngineConfig(num_partitions=len(d), replication_factor=3, segment_bytes=1 << 21, index_interval=1024,
                       max_consumers=2, max_batch_records=4096)
    ref = Broker(TOPIC, P)
    g = np.random.default_rng(0x52495050)
    msgs = [bytes(g.integers(0, 256, 100, dtype=np.uint8)) for _ in range(n)]
    with make_engine(cfg) as eng:
        b = PartitionBroker(d, eng, messages_as_str=False)
        prod = ProducerClient(b, {TOPIC: P, "other": 2}, batch_records=batch)
        results = [prod.produce(TOPIC, m) for m in msgs]
        prod.close()
        assert prod.batches == -(-n // batch)
        assert all(r.isSuccess() for r in results)
        for k, m in enumerate(msgs):  # RoundRobinSelector: abs(counter++) % n
            assert results[k].partition_id == k % P
            ref.produce(k % P, m)
        for p in range(P):
            got = b.state_machine(f"{TOPIC}-{p}").handleBatchRead(MessageBatchReadRequest("c", n, TOPIC, p))
            assert got.getOffset() == 0 and got.getMessages() == ref.sms[p].messages
        with pytest.raises(RuntimeError, match="Topic not found: nope"):
            prod.produce("nope", b"x")


def test_producer_batching_oracle_handle(oracle_mod):
    _flow(oracle_mod.OracleEngine)


def test_round_robin_counter_wraps_like_java():
    assert [_java_abs_mod(c, 3) for c in range(5)] == [0, 1, 2, 0, 1]
    assert _java_abs_mod((1 << 31) - 1, 7) == ((1 << 31) - 1) % 7
    assert _java_abs_mod(1 << 31, 7) == -((1 << 31) % 7)  # Math.abs(MIN_VALUE) % 7 < 0 in Java
    assert _java_abs_mod((1 << 31) + 1, 7) == ((1 << 31) - 1) % 7


@pytest.mark.gpu
def test_producer_batching_gpu():
    from ripplemq_amd.engine import Engine
    _flow(Engine)
