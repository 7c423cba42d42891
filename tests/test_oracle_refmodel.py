"""The oracle against a literal Python restatement of PartitionStateMachine.java (tests/refmodel.py).

Pins the reference-visible semantics: per-partition 0-based contiguous offsets in apply order,
handleBatchRead's [off, min(off + max, size)) slice with getOrDefault(id, 0), last-writer-wins
unchecked consumer offsets, and the read-then-commit consume loop of ConsumerClientImpl.
"""
import numpy as np

from refmodel import Broker
from ripplemq_amd.engine import EngineConfig, parse_records
from ripplemq_amd.workload import StreamSpec, make_batch


def test_offsets_fetch_and_consumer_offsets(oracle_mod):
    P = 5
    cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 16, index_interval=256)
    ref = Broker("topic1", P)
    with oracle_mod.OracleEngine(cfg) as ora:
        g = np.random.default_rng(5)
        for b in range(4):
            batch = make_batch(StreamSpec(P, 200, "uniform", size=(0, 40), config_index=20), b)
            offs, st = ora.append(batch.pidx, batch.lens, batch.payload)
            assert st["appended"] == 200
            pos = 0
            for i in range(batch.n):
                msg = batch.payload[pos:pos + batch.lens[i]].tobytes()
                pos += int(batch.lens[i])
                assert offs[i] == ref.produce(int(batch.pidx[i]), msg)
            # consumers: arbitrary (even backwards / beyond size) commits, then reads
            p = g.integers(0, P, 30)
            c = g.integers(0, 3, 30)
            o = g.integers(0, 400, 30)
            ora.commit_consumer_offset(p, c, o)
            for pi, ci, oi in zip(p, c, o):
                ref.sms[pi].handle_consumer_offset_update_request(f"c{ci}", int(oi))
            mx = g.integers(0, 25, 30)
            _, res, buf, _ = ora.fetch(p, c, mx)
            for k, (pi, ci, m) in enumerate(zip(p, c, mx)):
                msgs, off = ref.sms[pi].handle_batch_read(f"c{ci}", int(m))
                assert res[k]["start_offset"] == off and res[k]["count"] == len(msgs)
                recs = parse_records(buf[res[k]["out_pos"]:res[k]["out_pos"] + res[k]["bytes"]])
                assert [r[2] for r in recs] == msgs
                assert [r[0] for r in recs] == list(range(off, off + len(msgs)))
                for r in recs:
                    assert r[1] == oracle_mod.crc32c(r[2])


def test_consume_loop_read_then_commit(oracle_mod):
    P = 3
    cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 16, index_interval=256)
    ref = Broker("topic1", P)
    with oracle_mod.OracleEngine(cfg) as ora:
        msgs = [f"test-message-{i}".encode() for i in range(47)]
        for i, m in enumerate(msgs):  # ProducerClientImpl: one message per request, round-robin
            off, _ = ora.append(np.array([i % P]), np.array([len(m)]), np.frombuffer(m, np.uint8))
            assert int(off[0]) == ref.produce(i % P, m)
        for _ in range(8):
            for p in range(P):
                got_ref, off_ref = ref.consume(p, "consumer-1")
                _, res, buf, _ = ora.fetch([p], [0], [10])
                ora.commit_consumer_offset([p], [0], [int(res[0]["start_offset"] + res[0]["count"])])
                assert int(res[0]["start_offset"]) == off_ref
                assert [r[2] for r in parse_records(buf)] == got_ref


def test_not_leader_and_unknown_partition(oracle_mod):
    cfg = EngineConfig(num_partitions=4, replication_factor=3, segment_bytes=1 << 16, index_interval=256)
    with oracle_mod.OracleEngine(cfg) as ora:
        ora.set_replicas(1, [2, 0, 1], 0)  # leader elsewhere
        offs, st = ora.append(np.array([0, 1, 9, 0]), np.array([1, 1, 1, 1]), np.arange(4, dtype=np.uint8))
        assert list(offs) == [0, 2**64 - 1, 2**64 - 1, 1]
        assert st["rejected_not_leader"] == 1 and st["rejected_no_partition"] == 1
        rc, status = ora.commit_consumer_offset([1, 9, 0, 0], [0, 0, 99, 0], [1, 1, 1, 1])
        assert list(status) == [-1, -2, -3, 0]
        _, res, _, _ = ora.fetch([1, 9, 0], [0, 0, 0], [10, 10, 10])
        assert list(res["status"]) == [-1, -2, 0]


def test_quorum_commit_rule(oracle_mod):
    cfg = EngineConfig(num_partitions=1, replication_factor=5, segment_bytes=1 << 16, index_interval=256)
    with oracle_mod.OracleEngine(cfg) as ora:
        ora.set_replicas(0, [0, 1, 2, 3, 4], 0)
        ora.become_leader(0, 2)
        ora.append(np.zeros(10, np.uint32), np.ones(10, np.uint32), np.ones(10, np.uint8))
        assert ora.state(0)["commit"] == 0                       # only the leader has it
        ora.ack([0, 0], [1, 2], [4, 7])                          # rows: 10,4,7,0,0 -> 3rd largest 4
        assert ora.state(0)["commit"] == 4
        ora.ack([0], [3], [9])                                   # 10,4,7,9,0 -> 7
        assert ora.state(0)["commit"] == 7 and ora.state(0)["high_watermark"] == 7
        ora.ack([0], [4], [50])                                  # clamped to log end 10 -> 9
        assert ora.state(0)["commit"] == 9
        ora.become_leader(0, 3)                                  # new term: remote matches reset
        assert ora.state(0)["commit"] == 9 and ora.state(0)["term_start"] == 10
        ora.ack([0], [1], [10])                                  # 10,10,0,0,0: no quorum yet
        assert ora.state(0)["commit"] == 9
        # a quorum holding the log up to term_start in the new term holds the leader-start entry
        # (jraft's configuration entry, virtual here): the earlier-term records commit with it
        ora.ack([0], [2], [10])                                  # 10,10,10,0,0 -> 10 >= term_start
        assert ora.state(0)["commit"] == 10
        ora.append(np.zeros(1, np.uint32), np.ones(1, np.uint32), np.ones(1, np.uint8))
        ora.ack([0, 0], [1, 2], [11, 11])
        assert ora.state(0)["commit"] == 11
