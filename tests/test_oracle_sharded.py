"""The partition-sharded CPU baseline (oracle ro_append_sharded) computes exactly what the
sequential oracle computes, batch after batch: offsets, stats, state, rings and index."""
import numpy as np
import pytest

from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.workload import StreamSpec, make_batch


@pytest.mark.parametrize("threads,mode,P", [(1, "zipf", 64), (3, "zipf", 64), (8, "uniform", 300), (5, "rr", 7)])
def test_sharded_equals_sequential(oracle_mod, threads, mode, P):
    I = 256
    cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 17, index_interval=I,
                       max_batch_records=4096)
    spec = StreamSpec(P, 1000, mode, size=(0, 150), config_index=21, invalid_frac=0.01)
    big = make_batch(StreamSpec(P, 2500, "uniform", size=100, config_index=24), 0)
    big.pidx[::2] = 0  # 1250 x 128 B for partition 0 > ring - I: partition 0 takes none of them
    batches = [make_batch(spec, b) for b in range(12)]
    batches.insert(3, big)
    with oracle_mod.OracleEngine(cfg) as seq, oracle_mod.OracleEngine(cfg) as par:
        for e in (seq, par):
            e.set_replicas(1 % P, [1, 0, 2], 0)  # a partition this rank does not lead
        exp = [seq.append(b.pidx, b.lens, b.payload) for b in batches]
        got = par.append_sharded(batches, threads)
        assert exp[3][1]["rejected_no_space"] == int(np.sum(big.pidx == 0))
        assert exp[3][1]["appended"] == len(big.pidx) - int(np.sum(big.pidx == 0)) - int(np.sum(big.pidx == 1 % P))
        for (oe, se), (og, sg) in zip(exp, got):
            assert se == sg
            assert np.array_equal(oe, og)
        for p in range(P):
            s = seq.state(p)
            assert s == par.state(p)
            for r in range(3):
                assert np.array_equal(seq.read_segment(r, p), par.read_segment(r, p))
            m_lo, m_hi = -(-s["log_start_pos"] // I), s["log_end_pos"] // I
            assert np.array_equal(seq.read_index(p, m_lo, m_hi - m_lo + 1), par.read_index(p, m_lo, m_hi - m_lo + 1))
        if mode == "zipf":  # hot partitions wrap their rings: retention is exercised
            assert max(seq.state(p)["log_start_offset"] for p in range(P)) > 0


def test_reserve_keeps_ring_bytes(oracle_mod):
    cfg = EngineConfig(num_partitions=4, replication_factor=2, segment_bytes=1 << 16, index_interval=256)
    b = make_batch(StreamSpec(4, 300, "uniform", size=(0, 90), config_index=25), 0)
    with oracle_mod.OracleEngine(cfg) as ora:
        ora.append(b.pidx, b.lens, b.payload)
        before = [ora.read_segment(r, p).copy() for p in range(4) for r in range(2)]
        ora.reserve(np.full(4, 1 << 16, np.uint64))
        after = [ora.read_segment(r, p) for p in range(4) for r in range(2)]
        assert all(np.array_equal(x, y) for x, y in zip(before, after))
