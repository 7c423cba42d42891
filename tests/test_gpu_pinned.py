"""GPU tests pinned by something other than the oracle, plus full-size and concurrency cases.

* RFC 3720 §B.4 CRC32C vectors appended as records: the CRC field read back from the ring must be
  the published value (tests/golden/crc32c_kat.txt), with no oracle involved.
* BASELINE configs[0]'s plumbing stream through the engine: one topic, one partition, 10k x 100 B
  messages produced one per request (sample-producer/.../Main.java:31-37, PartitionClient.java:39-40),
  then a consumer draining it read-then-commit with max 10 (sample-consumer/.../Main.java:62-91,
  ConsumerClientImpl.java:61-117), checked against tests/refmodel.py (the literal restatement of
  PartitionStateMachine.java).
* configs[1]'s fetch leg at full size (256 partitions, 64k x 100 B batches) against the oracle.
* Fetch while batches are still in the append pipeline: every record a fetch returns must be
  byte-identical to that record in the fully applied log, and the fetch must not flush the pipeline.
"""
import numpy as np
import pytest

from kat import vectors
from parity import compare_state, run_ops
from refmodel import Broker
from ripplemq_amd.engine import Engine, EngineConfig, parse_records
from ripplemq_amd.state_machine import (ConsumerOffsetUpdateRequest, MessageAppendRequest, MessageBatchReadRequest,
                                        PartitionBroker, PartitionDirectory)
from ripplemq_amd.workload import StreamSpec, make_batch

pytestmark = pytest.mark.gpu


def test_kat_crc_read_back_from_ring():
    kat = vectors()
    # every vector 8 times: on 3 partitions and at every payload alignment 0..7 (explicit offsets)
    recs, pay, offs, pids = [], bytearray(), [], []
    for k in range(8):
        for i, (_, data, crc) in enumerate(kat):
            pay += bytes(k % 8)
            offs.append(len(pay))
            pay += data
            recs.append((data, crc))
            pids.append((i + k) % 3)
    cfg = EngineConfig(num_partitions=3, replication_factor=2, segment_bytes=1 << 16, index_interval=256)
    lens = np.array([len(d) for d, _ in recs], np.uint32)
    with Engine(cfg) as eng:
        out, st = eng.append(np.array(pids, np.uint32), lens, np.frombuffer(bytes(pay) + bytes(16), np.uint8),
                             np.array(offs, np.uint64))
        assert st["appended"] == len(recs)
        for p in range(3):
            want = [(d, c) for (d, c), q in zip(recs, pids) if q == p]
            used = eng.state(p)["log_end_pos"]
            for r in range(2):
                got = parse_records(eng.read_segment(r, p, 0, used))
                assert [o for o, _, _ in got] == list(range(len(want)))
                assert [(b, c) for _, c, b in got] == want, f"partition {p} replica {r}: CRC or payload differs"


def test_configs0_plumbing_stream():
    topic = "topic1"
    d = PartitionDirectory({topic: 1}, max_consumers=4)
    cfg = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 21, index_interval=1024,
                       max_consumers=4, max_batch_records=4096)
    ref = Broker(topic, 1)
    g = np.random.default_rng(0x52495050)
    msgs = [bytes(g.integers(0, 256, 100, dtype=np.uint8)) for _ in range(10_000)]
    with Engine(cfg) as eng:
        b = PartitionBroker(d, eng, messages_as_str=False)
        for k in range(0, len(msgs), 1000):  # 1000 single-message requests per engine batch
            resp = b.process_append([MessageAppendRequest([m], topic, 0) for m in msgs[k:k + 1000]])
            assert all(r.isSuccess() for r in resp)
            for m in msgs[k:k + 1000]:
                ref.produce(0, m)
        sm = b.state_machine(f"{topic}-0")
        drained = []
        while True:
            got = sm.handleBatchRead(MessageBatchReadRequest("sample-consumer", 10, topic, 0))
            want, off = ref.sms[0].handle_batch_read("sample-consumer", 10)
            assert got.getOffset() == off and got.getMessages() == want
            if not want:
                break
            drained += got.getMessages()
            assert sm.handleConsumerOffsetUpdateRequest(
                ConsumerOffsetUpdateRequest("sample-consumer", off + len(want), topic, 0)).isSuccess()
            ref.sms[0].handle_consumer_offset_update_request("sample-consumer", off + len(want))
        assert drained == msgs
        assert sm.getConsumerOffset("sample-consumer") == 10_000


def test_config_A_fetch_leg(oracle_mod):
    cfg = EngineConfig(num_partitions=256, replication_factor=3, segment_bytes=1 << 24, index_interval=1024,
                       max_consumers=4, max_batch_records=65536)
    spec = StreamSpec(256, 65536, "rr", size=100, config_index=1)
    g = np.random.default_rng(11)
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        ops = [("append", make_batch(spec, b)) for b in range(3)]
        P, C = 256, 4
        p = np.repeat(np.arange(P), C)
        c = np.tile(np.arange(C), P)
        for mx in (10, 1024):
            ops.append(("consumer_commit", p, c, g.integers(0, 3 * 65536 // P + 5, P * C)))
            ops.append(("fetch", p, c, np.full(P * C, mx)))
        run_ops(dev, ora, cfg, ops, check=False)
        compare_state(dev, ora, cfg)


def test_fetch_during_pipelined_appends(oracle_mod):
    cfg = EngineConfig(num_partitions=64, replication_factor=3, segment_bytes=1 << 20, index_interval=256,
                       max_consumers=2, max_batch_records=4096, pipeline_depth=2)
    spec = StreamSpec(64, 3000, "zipf", size=(1, 200), config_index=41)
    batches = [make_batch(spec, b) for b in range(12)]
    P = 64
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as full:
        for b in batches:
            full.append(b.pidx, b.lens, b.payload)
        p, c = np.arange(P), np.zeros(P, np.uint32)
        seen, last_hw = 0, np.zeros(P, np.int64)
        for k, b in enumerate(batches):
            dev.append_async(b.pidx, b.lens, b.payload)
            rc, res, buf, _ = dev.fetch(p, c, np.full(P, 1 << 20))
            assert np.all(res["status"] == 0)
            hw = res["count"].astype(np.int64)  # consumer offsets are 0: count = high watermark
            assert np.all(hw >= last_hw), "the high watermark went back"
            last_hw = hw
            _, want, wbuf, _ = full.fetch(p, c, res["count"])
            assert np.array_equal(res["bytes"], want["bytes"])
            assert np.array_equal(buf, wbuf), f"fetch after batch {k} returned bytes the full log does not hold"
            seen += int(hw.sum())
        applied_before_sync = int(last_hw.sum())
        dev.sync()
        _, res, _, _ = dev.fetch(p, c, np.full(P, 1 << 20))
        assert int(res["count"].sum()) == sum(b.n for b in batches)
        assert applied_before_sync < sum(b.n for b in batches), "fetches flushed the pipeline"
        assert seen > 0, "no fetch saw committed records while appends were in flight"


def test_fetch_sees_retention_of_applied_groups(oracle_mod):
    """Hot partitions wrap their 64 KiB rings while batches are in flight: after every submission
    the partition state (read without flushing) and a fetch from offset 0 must equal the oracle
    after the batches applied so far, retention of the last applied group included (it runs in the
    launch that applies the group, so no fetch reads ring bytes that group overwrote)."""
    P = 16
    cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 16, index_interval=256,
                       max_consumers=2, max_batch_records=4096, pipeline_depth=2)
    spec = StreamSpec(P, 1500, "zipf", size=(1, 160), config_index=43)
    batches = [make_batch(spec, b) for b in range(14)]
    pp, cc = np.arange(P, dtype=np.uint32), np.zeros(P, np.uint32)
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        applied, checked, moved = 0, 0, 0
        for b in batches:
            dev.append_async(b.pidx, b.lens, b.payload)
            st = [dev.state(p) for p in range(P)]
            leo = [s["log_end_offset"] for s in st]
            while [ora.state(p)["log_end_offset"] for p in range(P)] != leo:
                assert applied < len(batches), "device state matches no prefix of the batches"
                nb = batches[applied]
                ora.append(nb.pidx, nb.lens, nb.payload)
                applied += 1
            assert st == [ora.state(p) for p in range(P)], f"state after {applied} applied batches"
            _, res, buf, _ = dev.fetch(pp, cc, np.full(P, 1 << 20, np.uint32))
            _, want, wbuf, _ = ora.fetch(pp, cc, np.full(P, 1 << 20, np.uint32))
            for k in ("status", "start_offset", "count", "bytes"):
                assert np.array_equal(res[k], want[k]), (k, applied)
            assert np.array_equal(buf, wbuf)
            checked += 1
            moved += int(np.count_nonzero(res["start_offset"]))
        assert checked == len(batches) and moved > 0, "scenario must fetch across retention"
        dev.sync()


def test_fetch_many_requests(oracle_mod):
    """One fetch call places 20k requests (several passes of the placement scan) with unknown
    partitions, bad consumers and zero-record slices mixed in, then the same requests into an
    output buffer that ends mid-way (ENOSPC after the cut), over several calls."""
    P, C = 1024, 4
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 20, index_interval=512,
                       max_consumers=C, max_batch_records=65536)
    spec = StreamSpec(P, 40000, "zipf", size=(1, 400), config_index=7)
    g = np.random.default_rng(5)
    n = 20000
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        ops = [("append", make_batch(spec, b)) for b in range(3)]
        p = g.integers(0, P + 8, n)  # a few unknown partitions
        c = g.integers(0, C + 1, n)  # and bad consumer indices
        pc = np.repeat(np.arange(P), C)
        cc = np.tile(np.arange(C), P)
        ops.append(("consumer_commit", pc, cc, g.integers(0, 200, P * C)))
        mx = g.integers(0, 40, n)
        ops.append(("fetch", p, c, mx))
        ops.append(("fetch", p, c, mx, 1 << 20))  # ends mid-way: later requests are ENOSPC
        ops.append(("fetch", p[:300], c[:300], mx[:300]))
        ops.append(("fetch", p, c, np.full(n, 1000)))
        run_ops(dev, ora, cfg, ops, check=False)
        log = run_ops(dev, ora, cfg, [("fetch", p, c, mx, 1 << 20)], check=False)
        assert (log[0][1]["status"] == -4).any() and (log[0][1]["status"] == 0).any()
