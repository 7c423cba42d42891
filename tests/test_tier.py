"""Durable segment files and replay (ripplemq_amd/tier.py).

The reference never evicts (PartitionStateMachine.java:26: every message stays in `messages`), so
a consumer reading from offset 0 long after its records left the engine's rings must still get
them: the broker serves such reads from the segment files the tier spilled. Checked against
tests/refmodel.py (the literal restatement of the reference state machine). Replay rebuilds a
fresh engine from the files and the tier checks every offset and the ring bytes of the retained
window against the files. The CPU test injects the oracle's handle (host logic only); the GPU test
runs the same flow on the HIP engine.
"""
import numpy as np
import pytest

from refmodel import Broker
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.state_machine import (ConsumerOffsetUpdateRequest, MessageAppendRequest, MessageBatchReadRequest,
                                        PartitionBroker, PartitionDirectory)
from ripplemq_amd.tier import DurableLog, replay

TOPIC = "topic1"
P = 4


def _flow(make_engine, tmp_path, seg_file_bytes):
    d = PartitionDirectory({TOPIC: P}, max_consumers=4)
    cursor = d.consumer("__durable_tier")
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 14, index_interval=256,
                       max_consumers=4, max_batch_records=4096)
    ref = Broker(TOPIC, P)
    g = np.random.default_rng(31)
    with make_engine(cfg) as eng:
        tier = DurableLog(eng, str(tmp_path), range(P), cursor, segment_file_bytes=seg_file_bytes)
        b = PartitionBroker(d, eng, messages_as_str=False, durable=tier)
        for rnd in range(40):
            reqs = []
            for i in range(int(g.integers(20, 60))):
                pid = int(g.integers(0, P))
                reqs.append(MessageAppendRequest([bytes(g.integers(0, 256, int(g.integers(0, 300)), dtype=np.uint8))],
                                                 TOPIC, pid))
            assert all(r.isSuccess() for r in b.process_append(reqs))
            for r in reqs:
                ref.produce(r.partitionId, r.messages[0])
            if rnd % 3 == 2:
                tier.spill()
        starts = [eng.state(p)["log_start_offset"] for p in range(P)]
        assert min(starts) > 0, "rings never evicted: the tier is not exercised"
        # a consumer from offset 0: read max 10 then commit, until drained (ConsumerClientImpl.java:61-117)
        for p in range(P):
            sm = b.state_machine(f"{TOPIC}-{p}")
            while True:
                got = sm.handleBatchRead(MessageBatchReadRequest("late-consumer", 10, TOPIC, p))
                want, off = ref.sms[p].handle_batch_read("late-consumer", 10)
                assert got.getOffset() == off and got.getMessages() == want, f"partition {p} offset {off}"
                if not want:
                    break
                assert sm.handleConsumerOffsetUpdateRequest(
                    ConsumerOffsetUpdateRequest("late-consumer", off + len(want), TOPIC, p)).isSuccess()
                ref.sms[p].handle_consumer_offset_update_request("late-consumer", off + len(want))
        tier.spill()
        ends = [tier.end(p) for p in range(P)]
        assert ends == [len(ref.sms[p].messages) for p in range(P)]
        # reopen: the files alone give the same durable ends and records
        again = DurableLog(eng, str(tmp_path), range(P), cursor, segment_file_bytes=seg_file_bytes)
        assert [again.end(p) for p in range(P)] == ends
        assert [m for _, _, m in again.read(1, 5, 7)] == ref.sms[1].messages[5:12]
        # the offsets and terms jraft keeps in the log and raft_meta: a new term and a consumer
        # that read part of partition 2, then one more spill
        eng.become_leader(2, 7)
        sm = b.state_machine(f"{TOPIC}-2")
        got = sm.handleBatchRead(MessageBatchReadRequest("mid-consumer", 25, TOPIC, 2))
        assert sm.handleConsumerOffsetUpdateRequest(
            ConsumerOffsetUpdateRequest("mid-consumer", got.getOffset() + len(got.getMessages()), TOPIC, 2)).isSuccess()
        tier.spill()
        saved = [eng.consumer_offsets(p).copy() for p in range(P)]
        terms = [eng.state(p)["term"] for p in range(P)]
        assert terms[2] == 7 and saved[2][d.consumer("mid-consumer")] == 25
    # replay into a fresh engine: offsets and ring bytes checked against the files by replay(); the
    # consumer offsets and terms come back from offsets.bin / meta.json
    big = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 18, index_interval=256,
                       max_consumers=4, max_batch_records=4096)
    with make_engine(big) as fresh:
        out = replay(str(tmp_path), fresh, range(P), batch_records=500)
        assert out["records"] == sum(ends) and out["terms"] == 1 and out["offset_rows"] == P
        assert [fresh.state(p)["log_end_offset"] for p in range(P)] == ends
        assert [fresh.state(p)["term"] for p in range(P)] == terms
        for p in range(P):
            assert np.array_equal(fresh.consumer_offsets(p), saved[p]), p
        # the restarted broker serves the mid consumer from where it committed
        b2 = PartitionBroker(d, fresh, messages_as_str=False)
        nxt = b2.state_machine(f"{TOPIC}-2").handleBatchRead(MessageBatchReadRequest("mid-consumer", 5, TOPIC, 2))
        assert nxt.getOffset() == 25 and nxt.getMessages() == ref.sms[2].messages[25:30]
    return ends


@pytest.mark.parametrize("seg_file_bytes", [1 << 30, 4096])
def test_durable_tier_oracle_handle(oracle_mod, tmp_path, seg_file_bytes):
    _flow(oracle_mod.OracleEngine, tmp_path, seg_file_bytes)


def test_durable_tier_detects_corruption(oracle_mod, tmp_path):
    d = PartitionDirectory({TOPIC: 1}, max_consumers=2)
    cfg = EngineConfig(num_partitions=1, replication_factor=1, segment_bytes=1 << 14, index_interval=256,
                       max_consumers=2)
    with oracle_mod.OracleEngine(cfg) as eng:
        tier = DurableLog(eng, str(tmp_path), [0], d.consumer("__durable_tier"))
        PartitionBroker(d, eng, messages_as_str=False, durable=tier).process_append(
            [MessageAppendRequest([b"abc" * k], TOPIC, 0) for k in range(50)])
        assert tier.spill() == 50
    seg = next((tmp_path / "p000000").glob("*.seg"))
    raw = bytearray(seg.read_bytes())
    raw[33] ^= 0x55  # record 0 is empty (16-byte header); this is payload byte 1 of record 1
    seg.write_bytes(bytes(raw))
    with oracle_mod.OracleEngine(cfg) as fresh:
        with pytest.raises(Exception):
            replay(str(tmp_path), fresh, [0])


@pytest.mark.gpu
def test_durable_tier_gpu(tmp_path):
    from ripplemq_amd.engine import Engine
    _flow(Engine, tmp_path, 4096)


@pytest.mark.parametrize("cut", ["mid_payload", "zero_filled"])
def test_durable_tier_reopen_torn_tail(oracle_mod, tmp_path, cut):
    # a crash in the middle of a segment write (fsync off) leaves a torn last record: the reopened
    # tier cuts the file back to its last whole record, and the next spill writes the rest again
    d = PartitionDirectory({TOPIC: 1}, max_consumers=2)
    cfg = EngineConfig(num_partitions=1, replication_factor=1, segment_bytes=1 << 14, index_interval=256,
                       max_consumers=2)
    msgs = [bytes([k]) * (3 * k) for k in range(40)]
    with oracle_mod.OracleEngine(cfg) as eng:
        tier = DurableLog(eng, str(tmp_path), [0], d.consumer("__durable_tier"))
        b = PartitionBroker(d, eng, messages_as_str=False, durable=tier)
        b.process_append([MessageAppendRequest([m], TOPIC, 0) for m in msgs])
        assert tier.spill() == 40
        seg = next((tmp_path / "p000000").glob("*.seg"))
        raw = seg.read_bytes()
        whole = len(raw)
        # the last record (offset 39, 117 B payload: 16 + 128 bytes) torn
        last = whole - (16 + 128)
        torn = raw[:last + 40] if cut == "mid_payload" else raw[:last] + bytes(16 + 128)
        seg.write_bytes(torn)
        # the engine's durable cursor still says 40: as after a crash, it restarts from the files
        eng.commit_consumer_offset(np.zeros(1, np.uint32), np.full(1, d.consumer("__durable_tier"), np.uint32),
                                   np.zeros(1, np.uint64))
        again = DurableLog(eng, str(tmp_path), [0], d.consumer("__durable_tier"))
        assert again.end(0) == 39 and seg.stat().st_size == last
        assert again.spill() == 1 and again.end(0) == 40
        assert seg.read_bytes() == raw
        assert [m for _, _, m in again.read(0, 0, 100)] == msgs


def test_zero_filled_first_segment_is_torn(oracle_mod, tmp_path):
    # a segment whose first offset is 0 and whose first write was zero-filled by the file
    # system would parse as an empty message at offset 0 (header 0, length 0, CRC32C of nothing = 0).
    # No spill completed (no meta.json names a durable end), so the reopened tier drops it.
    d = PartitionDirectory({TOPIC: 1}, max_consumers=2)
    cfg = EngineConfig(num_partitions=1, replication_factor=1, segment_bytes=1 << 14, index_interval=256,
                       max_consumers=2)
    part = tmp_path / "p000000"
    part.mkdir()
    (part / f"{0:020d}.seg").write_bytes(bytes(48))
    with oracle_mod.OracleEngine(cfg) as eng:
        tier = DurableLog(eng, str(tmp_path), [0], d.consumer("__durable_tier"))
        assert tier.end(0) == 0 and not list(part.glob("*.seg"))


def test_native_record_scan_matches_the_format(oracle_mod):
    # rmq_scan_records (host, engine library) on FORMAT.md records the oracle wrote: positions,
    # whole-record counts, CRC32C and padding checks, cuts
    from ripplemq_amd.tier import record_positions, whole_records
    cfg = EngineConfig(num_partitions=1, replication_factor=1, segment_bytes=1 << 16, index_interval=256)
    lens = np.array([0, 1, 15, 16, 17, 100, 1000], np.uint32)
    pay = np.random.default_rng(5).integers(0, 256, int(lens.sum()), dtype=np.uint8)
    with oracle_mod.OracleEngine(cfg) as eng:
        eng.append(np.zeros(len(lens), np.uint32), lens, pay)
        st = eng.state(0)
        buf = eng.read_segment(0, 0, 0, st["log_end_pos"])
    rs = 16 + (lens.astype(np.int64) + 15) // 16 * 16
    want = np.concatenate([[0], np.cumsum(rs)])
    assert np.array_equal(record_positions(buf), want)
    assert whole_records(buf, 0) == (len(lens), int(want[-1]))
    assert whole_records(buf[:-1], 0) == (len(lens) - 1, int(want[-2]))  # cut short
    bad = buf.copy()
    bad[int(want[-2]) + 16 + 999] ^= 1  # the last payload byte: a CRC mismatch in the tail
    assert whole_records(bad, 0) == (len(lens) - 1, int(want[-2]))
    pad = buf.copy()
    pad[int(want[2]) + 16 + 15] = 7  # record 2 (15 B payload): its pad byte, records follow
    with pytest.raises(Exception):
        whole_records(pad, 0)


def test_tier_attached_to_a_running_engine(oracle_mod, tmp_path):
    """A tier opened on an engine whose rings already dropped records (bench.py's tier leg): its
    files start at each partition's log start (`start=`); without it the first spill asks for
    offset 0, which is gone, and refuses with RMQ_EOFFSET instead of spilling a gap."""
    from ripplemq_amd import _abi as A
    from ripplemq_amd.engine import EngineError
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 13, index_interval=256,
                       max_consumers=4, max_batch_records=4096)
    g = np.random.default_rng(7)
    msgs = {p: [] for p in range(P)}
    with oracle_mod.OracleEngine(cfg) as eng:
        for _ in range(30):
            pidx = g.integers(0, P, 50).astype(np.uint32)
            lens = g.integers(1, 120, 50).astype(np.uint32)
            pay = g.integers(0, 256, int(lens.sum())).astype(np.uint8)
            eng.append(pidx, lens, pay)
            pos = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
            for i, p in enumerate(pidx.tolist()):
                msgs[p].append(bytes(pay[pos[i]:pos[i + 1]]))
        starts = np.array([eng.state(p)["log_start_offset"] for p in range(P)], np.int64)
        assert starts.min() > 0
        with pytest.raises(EngineError) as ex:
            DurableLog(eng, str(tmp_path / "plain"), range(P), 3).spill()
        assert ex.value.status == A.RMQ_EOFFSET
        tier = DurableLog(eng, str(tmp_path / "late"), range(P), 3, start=starts)
        assert tier.spill() == sum(len(msgs[p]) for p in range(P)) - int(starts.sum())
        for p in range(P):
            assert tier.end(p) == len(msgs[p])
            got = [m for _, _, m in tier.read(p, int(starts[p]), len(msgs[p]))]
            assert got == msgs[p][int(starts[p]):], p
