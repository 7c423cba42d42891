"""Reference-shaped partition interface over the engine (host glue, no data-path compute).

Mirrors the broker side of anshmehtamm/ripplemq for the hot path, with the reference's names,
argument meaning and error behaviour, so a broker (or a test) written against the reference reads
the same here:

* request / response records: ``mq-common/src/main/java/request/partition/*.java``
  (``MessageAppendRequest(messages, topicName, partitionId)``, ``getGroupId() == topic-partition``,
  ``MessageBatchReadRequest(consumerId, maxMessages, topicName, partitionId)``,
  ``ConsumerOffsetUpdateRequest(consumerId, offset, topicName, partitionId)``,
  ``MessageBatchReadResponse{messages, offset}``, ``*Response{success, errorMsg}``);
* ``PartitionStateMachine`` — ``handleMessageAppendRequest`` / ``handleConsumerOffsetUpdateRequest``
  / ``handleBatchRead`` / ``getConsumerOffset`` / ``onLeaderStart``
  (``mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:64-126``);
* ``PartitionBroker.process_*`` — the three request processors
  (``mq-broker/src/main/java/metadata/raft/request/processor/{MessageAppend,MessageBatchRead,
  ConsumerOffsetUpdate}RequestProcessor.java``), except that the append processor gathers many
  requests into ONE engine batch (the point of the engine) and, unlike the reference, stops after
  answering "Not leader" (the reference replies and then applies anyway).

The partition directory is the reference's ``groupId -> PartitionRaftServer`` map
(``PartitionManager.java:196-198``) reduced to ``groupId -> dense pidx``; consumer ids are interned
to dense ids per directory (the engine's consumer-offset table is dense,
``include/ripplemq_engine.h`` rmq_config.max_consumers).

Every data-path operation is one C-ABI call on the engine handle (``ripplemq_amd.engine.Engine``).
The handle is injected so the host logic can be unit-tested on CPU against the oracle's handle
(tests only); production constructs ``Engine``, which fails loudly without the HIP library.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _abi as A
from .engine import Engine, EngineConfig, EngineError, parse_records

NOT_LEADER = "Not leader"
COMMIT_PENDING = "Commit pending"


# ---- request / response records (mq-common/src/main/java/request/partition/)
@dataclass
class MessageAppendRequest:
    messages: list
    topicName: str
    partitionId: int

    def getMessages(self):
        return self.messages

    def getGroupId(self) -> str:
        return f"{self.topicName}-{self.partitionId}"


@dataclass
class MessageAppendResponse:
    success: bool = False
    errorMsg: str | None = None

    def isSuccess(self) -> bool:
        return self.success

    def getErrorMsg(self):
        return self.errorMsg


@dataclass
class ConsumerOffsetUpdateRequest:
    consumerId: str
    offset: int
    topicName: str
    partitionId: int

    def getConsumerId(self) -> str:
        return self.consumerId

    def getOffset(self) -> int:
        return self.offset

    def getGroupId(self) -> str:
        return f"{self.topicName}-{self.partitionId}"


@dataclass
class ConsumerOffsetUpdateResponse:
    success: bool = False
    errorMsg: str | None = None
    ticket: int = 0  # COMMIT_PENDING: the engine's offset ticket (PartitionBroker.offset_update_done)

    def isSuccess(self) -> bool:
        return self.success

    def getErrorMsg(self):
        return self.errorMsg


@dataclass
class MessageBatchReadRequest:
    consumerId: str
    maxMessages: int
    topicName: str
    partitionId: int

    def getConsumerId(self) -> str:
        return self.consumerId

    def getMaxMessages(self) -> int:
        return self.maxMessages

    def getGroupId(self) -> str:
        return f"{self.topicName}-{self.partitionId}"


@dataclass
class MessageBatchReadResponse:
    messages: list = field(default_factory=list)
    offset: int = 0

    def getMessages(self):
        return self.messages

    def getOffset(self) -> int:
        return self.offset


def _encode(m) -> bytes:
    """Messages are Java Strings in the reference; bytes pass through, str is UTF-8."""
    return m if isinstance(m, (bytes, bytearray)) else str(m).encode("utf-8")


def _decode(b: bytes, as_str: bool):
    return b.decode("utf-8") if as_str else b


class PartitionDirectory:
    """groupId ("topic-partitionId") -> dense partition index, consumerId -> dense consumer id."""

    def __init__(self, topics: dict[str, int] | None = None, max_consumers: int = 64):
        self.group_to_pidx: dict[str, int] = {}
        self.pidx_to_group: list[str] = []
        self.consumers: dict[str, int] = {}
        self.max_consumers = max_consumers
        for topic, n in (topics or {}).items():
            for pid in range(n):
                self.add(f"{topic}-{pid}")

    def add(self, group_id: str) -> int:
        if group_id not in self.group_to_pidx:
            self.group_to_pidx[group_id] = len(self.pidx_to_group)
            self.pidx_to_group.append(group_id)
        return self.group_to_pidx[group_id]

    def pidx(self, group_id: str) -> int | None:
        return self.group_to_pidx.get(group_id)

    def consumer(self, consumer_id: str) -> int:
        c = self.consumers.get(consumer_id)
        if c is None:
            if len(self.consumers) >= self.max_consumers:
                raise EngineError(A.RMQ_EINVAL, f"consumer table full ({self.max_consumers})")
            c = self.consumers[consumer_id] = len(self.consumers)
        return c

    def __len__(self) -> int:
        return len(self.pidx_to_group)


class PartitionBroker:
    """The broker's partition processors over one engine handle (one GPU's partitions)."""

    def __init__(self, directory: PartitionDirectory, engine=None, *, replication_factor: int = 1,
                 segment_bytes: int = 1 << 22, index_interval: int = 4096, device: int = 0,
                 messages_as_str: bool = True, durable=None):
        """durable: a ``ripplemq_amd.tier.DurableLog`` over this engine, or None. With it, a read
        below a ring's retained start is served from the segment files (the reference never
        evicts, PartitionStateMachine.java:26) instead of failing with RMQ_EOFFSET."""
        self.dir = directory
        self.durable = durable
        if engine is None:
            cfg = EngineConfig(num_partitions=len(directory), replication_factor=replication_factor,
                               segment_bytes=segment_bytes, index_interval=index_interval,
                               max_consumers=directory.max_consumers, device=device)
            engine = Engine(cfg)
        self.engine = engine
        self.as_str = messages_as_str
        self._sms: dict[str, PartitionStateMachine] = {}

    def close(self) -> None:
        self.engine.close()

    # ---- MessageAppendRequestProcessor.handleRequest, batched
    def process_append(self, requests: list[MessageAppendRequest]) -> list[MessageAppendResponse]:
        """Apply every request's messages in request order as ONE engine batch.

        As in the reference, a request succeeds only once its entries are committed and applied
        (the PartitionClosure runs after BallotBox commit, MessageAppendRequestProcessor.java:39-48):
        a request whose records all got offsets below the partition's commit index answers success;
        one whose records are appended but not yet committed (followers on other ranks have not
        acknowledged) answers "Commit pending". A request for a partition this broker does not
        lead answers "Not leader"; one whose partition had no room for this batch (FORMAT.md §3)
        answers RMQ_ENOSPC; an unknown groupId answers "Unknown partition" (the reference
        dereferences null there)."""
        pidx, msgs, owner = [], [], []
        out = [MessageAppendResponse() for _ in requests]
        for r, req in enumerate(requests):
            p = self.dir.pidx(req.getGroupId())
            if p is None:
                out[r].errorMsg = "Unknown partition"
                continue
            for m in req.getMessages():
                pidx.append(p)
                msgs.append(_encode(m))
                owner.append(r)
        if not msgs:
            for r, req in enumerate(requests):
                if out[r].errorMsg is None:
                    out[r].success = True  # an empty message list applies trivially
            return out
        lens = np.fromiter((len(m) for m in msgs), np.uint32, len(msgs))
        payload = np.frombuffer(b"".join(msgs), np.uint8) if lens.sum() else np.zeros(0, np.uint8)
        pidx = np.asarray(pidx, np.uint32)
        try:
            offs, _ = self.engine.append(pidx, lens, payload)
        except EngineError as e:  # whole-batch rejections (invalid payload ranges)
            for r in set(owner):
                out[r].errorMsg = A.STATUS_NAMES.get(e.status, str(e.status))
            return out
        owner = np.asarray(owner)
        rejected = offs == np.uint64(A.RMQ_OFFSET_NONE)
        commit = self.engine.commit_snapshot()
        pending = ~rejected & (offs >= commit[pidx])
        leads = {p: bool(self.engine.state(p)["is_leader"]) for p in set(pidx[rejected].tolist())}
        bad, wait = {}, set(owner[pending].tolist())
        for k in np.flatnonzero(rejected).tolist():
            bad.setdefault(int(owner[k]), NOT_LEADER if not leads[int(pidx[k])] else A.STATUS_NAMES[A.RMQ_ENOSPC])
        for r in range(len(requests)):
            if out[r].errorMsg is not None:
                continue
            if r in bad:
                out[r].errorMsg = bad[r]
            elif r in wait:
                out[r].errorMsg = COMMIT_PENDING
            else:
                out[r].success = True
        return out

    # ---- ConsumerOffsetUpdateRequestProcessor.handleRequest, batched
    def process_consumer_offset_update(self, requests: list[ConsumerOffsetUpdateRequest]
                                       ) -> list[ConsumerOffsetUpdateResponse]:
        out = [ConsumerOffsetUpdateResponse() for _ in requests]
        idx, p, c, o = [], [], [], []
        for r, req in enumerate(requests):
            pi = self.dir.pidx(req.getGroupId())
            if pi is None:
                out[r].errorMsg = "Unknown partition"
                continue
            idx.append(r)
            p.append(pi)
            c.append(self.dir.consumer(req.getConsumerId()))
            o.append(int(req.getOffset()))
        if idx:
            _, status = self.engine.commit_consumer_offset(np.asarray(p, np.uint32), np.asarray(c, np.uint32),
                                                           np.asarray(o, np.uint64))
            # the reference answers from the Raft closure, once the update is committed
            # (ConsumerOffsetUpdateRequestProcessor.java:40-49,60): success only when the rows are on a
            # quorum (rmq_poll_commit of the call's offset ticket), else COMMIT_PENDING with the ticket
            ticket = self.engine.last_offset_ticket
            done = self.offset_update_done(ticket) if ticket else A.RMQ_OK
            for r, s in zip(idx, status.tolist()):
                if s != A.RMQ_OK:
                    out[r].errorMsg = NOT_LEADER if s == A.RMQ_ENOTLEADER else A.STATUS_NAMES.get(s, str(s))
                elif done == A.RMQ_OK:
                    out[r].success = True
                elif done == A.RMQ_PENDING:
                    out[r].errorMsg = COMMIT_PENDING
                    out[r].ticket = ticket
                else:
                    out[r].errorMsg = NOT_LEADER
        return out

    def offset_update_done(self, ticket: int) -> int:
        """A pending consumer-offset update: RMQ_OK once committed on a quorum (the reference's
        closure then answers success), RMQ_PENDING, or RMQ_ENOTLEADER (failed by a leader change)."""
        return self.engine.poll_offsets(ticket)

    # ---- MessageBatchReadRequestProcessor.handleRequest, batched
    def process_batch_read(self, requests: list[MessageBatchReadRequest]) -> list:
        """One MessageBatchReadResponse per request, or the string "Not leader" as the reference
        sends it (``rpcCtx.sendResponse("Not leader")``)."""
        out: list = [None] * len(requests)
        idx, p, c, mx = [], [], [], []
        for r, req in enumerate(requests):
            pi = self.dir.pidx(req.getGroupId())
            if pi is None:
                out[r] = "Unknown partition"
                continue
            idx.append(r)
            p.append(pi)
            c.append(self.dir.consumer(req.getConsumerId()))
            mx.append(max(int(req.getMaxMessages()), 0))
        if idx:
            _, res, buf, _ = self.engine.fetch(np.asarray(p, np.uint32), np.asarray(c, np.uint32),
                                               np.asarray(mx, np.uint32))
            spilled = False
            for k, r in enumerate(idx):
                st = int(res["status"][k])
                if st == A.RMQ_ENOTLEADER:
                    out[r] = NOT_LEADER
                    continue
                if st == A.RMQ_EOFFSET and self.durable is not None:
                    # below the ring: [off, min(off + max, hw)) from the segment files, after a
                    # spill has made everything committed durable
                    if not spilled:
                        self.durable.spill()
                        spilled = True
                    # (the row's start_offset is the first retained offset there: the consumer's
                    # own offset comes from the table)
                    off = int(self.engine.consumer_offsets(p[k])[c[k]])
                    hw = int(self.engine.state(p[k])["high_watermark"])
                    recs = self.durable.read(p[k], off, min(mx[k], hw - off))
                    out[r] = MessageBatchReadResponse([_decode(b, self.as_str) for _, _, b in recs], off)
                    continue
                if st != A.RMQ_OK:
                    raise EngineError(st, f"fetch {requests[r].getGroupId()}")
                pos, nb = int(res["out_pos"][k]), int(res["bytes"][k])
                recs = parse_records(buf[pos:pos + nb])
                out[r] = MessageBatchReadResponse([_decode(b, self.as_str) for _, _, b in recs],
                                                  int(res["start_offset"][k]))
        return out

    def getConsumerOffset(self, group_id: str, consumer_id: str) -> int:
        p = self.dir.pidx(group_id)
        c = self.dir.consumers.get(consumer_id)
        if p is None or c is None:
            return 0  # consumerOffsets.getOrDefault(consumerId, 0L)
        return int(self.engine.consumer_offsets(p)[c])

    # ---- PartitionStateMachine.onLeaderStart -> engine leadership (term bookkeeping)
    def onLeaderStart(self, group_id: str, term: int) -> None:
        self.engine.become_leader(self.dir.pidx(group_id), int(term))

    def state_machine(self, group_id: str) -> "PartitionStateMachine":
        sm = self._sms.get(group_id)
        if sm is None:
            if self.dir.pidx(group_id) is None:
                raise KeyError(group_id)
            sm = self._sms[group_id] = PartitionStateMachine(group_id, self)
        return sm


class PartitionStateMachine:
    """Per-partition facade with the reference's method names (PartitionStateMachine.java)."""

    def __init__(self, groupId: str, broker: PartitionBroker):
        self.groupId = groupId
        self.broker = broker

    def handleMessageAppendRequest(self, request: MessageAppendRequest) -> MessageAppendResponse:
        return self.broker.process_append([request])[0]

    def handleConsumerOffsetUpdateRequest(self, request: ConsumerOffsetUpdateRequest) -> ConsumerOffsetUpdateResponse:
        return self.broker.process_consumer_offset_update([request])[0]

    def handleBatchRead(self, request: MessageBatchReadRequest):
        return self.broker.process_batch_read([request])[0]

    def getConsumerOffset(self, consumerId: str) -> int:
        return self.broker.getConsumerOffset(self.groupId, consumerId)

    def onLeaderStart(self, term: int) -> None:
        self.broker.onLeaderStart(self.groupId, term)
