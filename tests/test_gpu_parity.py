"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle, bit for bit.

Every test runs the same op list through both (tests/parity.py) and compares offsets, stats,
partition state, ring bytes, sparse index, consumer offsets and fetch output.
"""
import numpy as np
import pytest

from parity import compare_state, run_ops
from ripplemq_amd.engine import Engine, EngineConfig
from ripplemq_amd.workload import Batch, StreamSpec, make_batch

pytestmark = pytest.mark.gpu


def pair(oracle_mod, **kw):
    cfg = EngineConfig(**kw)
    return cfg, Engine(cfg), oracle_mod.OracleEngine(cfg)


def test_small_mixed_sizes(oracle_mod):
    cfg, dev, ora = pair(oracle_mod, num_partitions=8, replication_factor=3, segment_bytes=1 << 20,
                         index_interval=256, max_batch_records=4096)
    with dev, ora:
        spec = StreamSpec(8, 300, "uniform", size=(0, 700), config_index=11)
        ops = [("append", make_batch(spec, b)) for b in range(6)]
        run_ops(dev, ora, cfg, ops, full_rings=True)


@pytest.mark.parametrize("P,mode", [(1, "rr"), (7, "uniform"), (256, "rr"), (300, "zipf"), (4096, "zipf")])
def test_partition_counts(oracle_mod, P, mode):
    cfg, dev, ora = pair(oracle_mod, num_partitions=P, replication_factor=3, segment_bytes=1 << 20,
                         index_interval=1024, max_batch_records=20000)
    with dev, ora:
        spec = StreamSpec(P, 5000, mode, size=100, config_index=12)
        ops = [("append", make_batch(spec, b)) for b in range(3)]
        run_ops(dev, ora, cfg, ops, full_rings=P <= 8)


def test_retention_wraps_ring(oracle_mod):
    # hot Zipf partitions wrap their 256 KB rings many times; log start follows the index rule
    cfg, dev, ora = pair(oracle_mod, num_partitions=64, replication_factor=3, segment_bytes=1 << 18,
                         index_interval=1024, max_batch_records=4096)
    with dev, ora:
        spec = StreamSpec(64, 2000, "zipf", size=(50, 150), config_index=13)
        ops = [("append", make_batch(spec, b)) for b in range(12)]
        run_ops(dev, ora, cfg, ops, full_rings=True)
        starts = [ora.state(p)["log_start_offset"] for p in range(64)]
        assert max(starts) > 0, "scenario must exercise retention"


def test_set_segments_grow_shrink_in_pool(oracle_mod):
    # rmq_set_segments (FORMAT.md §2): the hot Zipf partitions grow 4x inside the shared pool, cold
    # ones shrink (retention at the new size first); appends, retention, fetch and consumer commits
    # then continue bit-exact with the oracle, and every ring is compared whole (zeros outside the
    # retained log)
    P, S = 32, 1 << 16
    cfg, dev, ora = pair(oracle_mod, num_partitions=P, replication_factor=3, segment_bytes=S,
                         index_interval=1024, max_batch_records=4096, pool_bytes=3 * P * S)
    with dev, ora:
        spec = StreamSpec(P, 3000, "zipf", size=(1, 300), config_index=56)
        first = [make_batch(spec, b) for b in range(5)]
        load = np.bincount(np.concatenate([b.pidx for b in first]), minlength=P)
        order = np.argsort(-load, kind="stable")
        hot, cold = order[:4], order[-6:]
        grow = ("set_segments", hot, np.full(4, 4 * S, np.uint64))
        shrink = ("set_segments", np.concatenate([cold, order[4:6]]), np.full(8, 4096, np.uint64))
        pp = np.arange(P, dtype=np.uint32)
        ops = [("append", b) for b in first] + [grow, shrink]
        ops += [("append", make_batch(spec, b)) for b in range(5, 12)]
        ops += [("consumer_commit", pp, np.zeros(P, np.uint32), pp * 7),
                ("fetch", pp, np.zeros(P, np.uint32), np.full(P, 64, np.uint32))]
        ops += [("set_segments", hot[:2], np.full(2, S, np.uint64))]  # shrink two grown rings back
        ops += [("append", make_batch(spec, b)) for b in range(12, 14)]
        run_ops(dev, ora, cfg, ops, full_rings=True)
        segs = [ora.state(p)["segment_bytes"] for p in range(P)]
        assert sorted(set(segs)) == [4096, S, 4 * S], segs
        assert ora.state(int(order[4]))["log_start_offset"] > 0, "a shrink must apply retention"


def test_config_d_shape_in_load_sized_pool(oracle_mod):
    # config D's shape on one GPU (RF 5, 4096 partitions, log-uniform 64 B..16 KB): rings sized from
    # the traffic (ripplemq_amd.rings) in one pool of a few GiB, where equal 16 MiB rings need 320 GiB
    from ripplemq_amd.rings import partition_traffic, pool_layout, ring_sizes
    from ripplemq_amd.workload import CONFIGS
    spec = CONFIGS["D"]
    batches = [make_batch(spec, q) for q in range(4)]
    mean, peak = partition_traffic(batches, spec.partitions)
    lay = pool_layout(ring_sizes(mean, peak, 64, 64 << 10, 1024))
    assert 5 * lay.pool_bytes < 16 << 30
    cfg, dev, ora = pair(oracle_mod, num_partitions=spec.partitions, replication_factor=5,
                         segment_bytes=lay.segment_bytes, pool_bytes=lay.pool_bytes, index_interval=1024,
                         max_batch_records=spec.records, max_batch_bytes=64 << 20)
    with dev, ora:
        P = spec.partitions
        g = np.random.default_rng(21)
        pp = g.integers(0, P, 512).astype(np.uint32)
        ops = [("set_segments", lay.grown, lay.grown_bytes)] + [("append", b) for b in batches]
        ops += [("fetch", pp, np.zeros(512, np.uint32), g.integers(1, 6, 512).astype(np.uint32))]
        run_ops(dev, ora, cfg, ops)


def test_set_segments_pool_exhausted_changes_nothing():
    # all or nothing: a pool without room for the new rings answers RMQ_ENOMEM and leaves every ring
    P, S = 16, 1 << 14
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=S, index_interval=1024,
                       max_batch_records=2048, pool_bytes=P * S + 4 * S)
    spec = StreamSpec(P, 1000, "uniform", size=(1, 100), config_index=57)
    from ripplemq_amd.engine import EngineError
    with Engine(cfg) as dev:
        b = make_batch(spec, 0)
        dev.append(b.pidx, b.lens, b.payload)
        before = [dev.state(p) for p in range(P)]
        rings = [dev.read_segment(0, p) for p in range(P)]
        with pytest.raises(EngineError) as ex:
            dev.set_segments(np.arange(3, dtype=np.uint32), np.full(3, 4 * S, np.uint64))
        assert "ENOMEM" in str(ex.value)
        assert [dev.state(p) for p in range(P)] == before
        assert all(np.array_equal(dev.read_segment(0, p), r) for p, r in enumerate(rings))
        dev.set_segments(np.arange(1, dtype=np.uint32), np.full(1, 4 * S, np.uint64))  # one fits
        assert dev.state(0)["segment_bytes"] == 4 * S


def test_large_records_direct_path(oracle_mod):
    # log-uniform 64 B..16 KB (config D sizes): records longer than 112 B skip the LDS log image
    # and are stored piece by piece; long payloads take many Horner rounds per lane
    cfg, dev, ora = pair(oracle_mod, num_partitions=16, replication_factor=5, segment_bytes=1 << 23,
                         index_interval=1024, max_batch_records=4096, max_batch_bytes=32 << 20)
    with dev, ora:
        spec = StreamSpec(16, 700, "uniform", size=(64, 16384), config_index=14)
        ops = [("append", make_batch(spec, b)) for b in range(3)]
        run_ops(dev, ora, cfg, ops)


@pytest.mark.parametrize("big_wgs", [None, "1"])
def test_large_record_waves_in_groups(oracle_mod, monkeypatch, big_wgs):
    # records over 1 KB go to stage 3's large-record waves: rings that wrap inside a launch group
    # (dead pieces), a partition this engine does not lead, a no-space batch of large records, and
    # one workgroup taking the whole list (RMQ_BIG_WGS=1)
    if big_wgs:
        monkeypatch.setenv("RMQ_BIG_WGS", big_wgs)
    cfg, dev, ora = pair(oracle_mod, num_partitions=8, replication_factor=3, segment_bytes=1 << 18,
                         index_interval=1024, max_batch_records=4096, max_batch_bytes=8 << 20, pipeline_depth=4)
    with dev, ora:
        for e in (dev, ora):
            e.set_replicas(6, [1, 0, 2], 0)  # partition 6 led by rank 1
        spec = StreamSpec(8, 200, "uniform", size=(64, 16384), config_index=19)
        batches = [make_batch(spec, b) for b in range(9)]
        g = np.random.default_rng(19)
        hog_l = g.integers(4000, 16000, 90).astype(np.uint32)  # > 256 KiB for partition 0: no space
        hog = Batch(np.zeros(90, np.uint32), hog_l, g.integers(0, 256, int(hog_l.sum()), dtype=np.uint8))
        batches.insert(5, hog)
        _pipelined(dev, ora, batches)
        compare_state(dev, ora, cfg, full_rings=True)
        assert max(ora.state(p)["log_start_offset"] for p in range(8)) > 0, "rings must wrap"


def test_rejections_and_leadership(oracle_mod):
    cfg, dev, ora = pair(oracle_mod, num_partitions=16, replication_factor=3, segment_bytes=1 << 20,
                         index_interval=256, max_batch_records=4096)
    with dev, ora:
        spec = StreamSpec(16, 1500, "uniform", size=(1, 200), config_index=15, invalid_frac=0.05)
        ops = [("append", make_batch(spec, 0)),
               ("set_replicas", 3, [1, 0, 2], 0),        # partition 3 led by rank 1: not leader
               ("set_replicas", 5, [0, 1, 2], 0),        # partition 5: only slot 0 local
               ("become_leader", 5, 2),
               ("append", make_batch(spec, 1)),
               ("ack", [5], [1], [10]),                  # quorum needs 2 of 3: commit -> min(leo,10)
               ("ack", [5, 5], [2, 1], [7, 3]),          # max() keeps slot 1 at 10
               ("append", make_batch(spec, 2)),
               ("become_leader", 5, 3),                  # new term: prior entries wait for a new one
               ("ack", [5, 5], [1, 2], [10 ** 6, 10 ** 6]),
               ("append", make_batch(spec, 3)),
               ("ack", [5], [1], [10 ** 6]),
               ("fetch", np.arange(16), np.zeros(16), np.full(16, 10))]
        run_ops(dev, ora, cfg, ops, full_rings=True)


def test_no_space_and_edge_batches(oracle_mod):
    cfg, dev, ora = pair(oracle_mod, num_partitions=4, replication_factor=1, segment_bytes=1 << 12,
                         index_interval=64, max_batch_records=4096)
    with dev, ora:
        empty = Batch(np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
        one = Batch(np.array([2], np.uint32), np.array([5], np.uint32), np.arange(5, dtype=np.uint8))
        big = make_batch(StreamSpec(4, 400, "uniform", size=20, config_index=16), 0)  # > 4 KB - 64
        ok = make_batch(StreamSpec(4, 100, "uniform", size=(0, 20), config_index=16), 1)
        run_ops(dev, ora, cfg, [("append", empty), ("append", one), ("append", big), ("append", ok),
                                ("append", ok), ("append", big)], full_rings=True)


def test_rejected_long_records_next_to_short_ones(oracle_mod):
    # a wave whose stored records are all short (the LDS-image store path) but which also holds
    # rejected long records (no space): their piece counts must not turn into store flags
    cfg, dev, ora = pair(oracle_mod, num_partitions=2, replication_factor=2, segment_bytes=1 << 12,
                         index_interval=64, max_batch_records=4096)
    with dev, ora:
        g = np.random.default_rng(11)
        n = 192
        pidx = (np.arange(n) & 1).astype(np.uint32)                   # 0, 1, 0, 1, ...
        lens = np.where(pidx == 0, g.integers(241, 600, n), g.integers(0, 20, n)).astype(np.uint32)
        b = Batch(pidx, lens, g.integers(0, 256, int(lens.sum()), dtype=np.uint8))
        small = make_batch(StreamSpec(2, 60, "uniform", size=(0, 40), config_index=18), 0)
        run_ops(dev, ora, cfg, [("append", small), ("append", b), ("append", small), ("append", b)],
                full_rings=True)


def test_explicit_payload_offsets(oracle_mod):
    # caller-provided payload_off with gaps and unaligned starts
    cfg, dev, ora = pair(oracle_mod, num_partitions=8, replication_factor=2, segment_bytes=1 << 20,
                         index_interval=256, max_batch_records=4096)
    with dev, ora:
        g = np.random.default_rng(7)
        n = 900
        lens = g.integers(0, 300, n).astype(np.uint32)
        gaps = g.integers(0, 9, n).astype(np.uint64)
        off = np.cumsum(gaps + np.r_[0, lens[:-1]].astype(np.uint64)).astype(np.uint64)
        payload = g.integers(0, 256, int(off[-1] + lens[-1] + 16), dtype=np.uint8)
        b = Batch(g.integers(0, 8, n).astype(np.uint32), lens, payload)
        run_ops(dev, ora, cfg, [("append", b, off, payload)], full_rings=True)


@pytest.mark.parametrize("interval,seg", [(256, 1 << 16), (4096, 1 << 16)])
def test_consumer_fetch_paths(oracle_mod, interval, seg):
    # interval 4096: the records between an index entry and a fetch bound span several of the
    # resolve's 1 KiB header windows
    cfg, dev, ora = pair(oracle_mod, num_partitions=32, replication_factor=3, segment_bytes=seg,
                         index_interval=interval, max_consumers=4, max_batch_records=8192)
    with dev, ora:
        # 450 records (~50 KB) per batch fit the 64 KB rings; hot partitions wrap them (eviction)
        spec = StreamSpec(32, 450, "zipf", size=(1, 180), config_index=17)
        g = np.random.default_rng(3)
        ops = []
        for b in range(8):
            ops.append(("append", make_batch(spec, b)))
            n = 200
            p = g.integers(0, 33, n)            # includes an unknown partition (32)
            c = g.integers(0, 5, n)             # includes an invalid consumer id (4)
            o = g.integers(0, 1200, n)          # lagging, current, beyond hw, evicted
            ops.append(("consumer_commit", p, c, o))
            ops.append(("fetch", p, c, g.integers(0, 40, n)))
            ops.append(("fetch", p, c, np.full(n, 1024), 5000))  # output buffer too small
        ops.append(("set_replicas", 9, [2, 0, 1], 0))
        ops.append(("fetch", np.arange(32), np.zeros(32), np.full(32, 10)))
        run_ops(dev, ora, cfg, ops, full_rings=True)


def test_read_then_commit_consume_loop(oracle_mod):
    # ConsumerClientImpl.consume: read max 10, commit offset + n, until drained
    cfg, dev, ora = pair(oracle_mod, num_partitions=3, replication_factor=3, segment_bytes=1 << 16,
                         index_interval=256, max_batch_records=4096)
    with dev, ora:
        b = make_batch(StreamSpec(3, 95, "rr", size=12, config_index=18), 0)
        run_ops(dev, ora, cfg, [("append", b)])
        for _ in range(12):
            for eng in (dev, ora):
                _, res, _, _ = eng.fetch([0, 1, 2], [0, 0, 0], [10, 10, 10])
                eng.commit_consumer_offset([0, 1, 2], [0, 0, 0], res["start_offset"] + res["count"])
        compare_state(dev, ora, cfg)
        assert [int(dev.consumer_offsets(p)[0]) for p in range(3)] == [32, 32, 31]


def _pipelined(dev, ora, batches):
    """Submit every batch before waiting for any (the engine coalesces them into launch groups of
    cfg.pipeline_depth), then check each batch's offsets and stats against the oracle applying the
    batches one at a time."""
    subs = [dev.append_async(b.pidx, b.lens, b.payload) for b in batches]
    for (t, out), b in zip(subs, batches):
        sd = dev.wait(t)
        oo, so = ora.append(b.pidx, b.lens, b.payload)
        assert sd == so, f"append stats gpu={sd} cpu={so}"
        if not np.array_equal(out, oo):
            bad = np.flatnonzero(out != oo)
            raise AssertionError(f"out_offsets differ at {bad[:8]}: gpu={out[bad[:8]]} cpu={oo[bad[:8]]}")


@pytest.mark.parametrize("group", [1, 2, 3, 4, 8])
def test_pipelined_groups(oracle_mod, group):
    # back-to-back submissions: launch groups of `group` batches with retention after every batch,
    # a no-space batch inside a group, a partition this rank does not lead, unknown partitions
    cfg, dev, ora = pair(oracle_mod, num_partitions=64, replication_factor=3, segment_bytes=1 << 17,
                         index_interval=256, max_batch_records=4096, pipeline_depth=group)
    with dev, ora:
        spec = StreamSpec(64, 1400, "zipf", size=(0, 120), config_index=22, invalid_frac=0.01)
        big = make_batch(StreamSpec(64, 1100, "uniform", size=100, config_index=23), 0)
        big.pidx[:1050] = 7  # 1050 x 128 B > ring - I: partition 7 takes none of this batch's records
        for e in (dev, ora):
            e.set_replicas(5, [1, 0, 2], 0)
        batches = [make_batch(spec, b) for b in range(11)]
        batches.insert(5, big)
        _pipelined(dev, ora, batches)
        compare_state(dev, ora, cfg, full_rings=True)
        assert max(ora.state(p)["log_start_offset"] for p in range(64)) > 0, "scenario must exercise retention"
        assert dev.state(5)["log_end_offset"] == 0


@pytest.mark.parametrize("env", [{"RMQ_WG3_ALL": "0"}, {"RMQ_S3_FIRST": "1"}, {"RMQ_S3_LEAD": "5"}, {"RMQ_BIG_WGS": "3"},
                                 {"RMQ_S3_XCD": "0", "RMQ_S1_XCD": "1"}, {"RMQ_S1_XCD": "1", "RMQ_S1_WGS": "37"},
                                 {"RMQ_S3_ROLES": "0"}, {"RMQ_S3_ROLES": "1", "RMQ_S3_XCD": "0"},
                                 {"RMQ_S3_ROLES": "4"}])
def test_pipelined_dispatch_modes(oracle_mod, monkeypatch, env):
    # the non-default dispatch modes (read at rmq_create): resident task waves looping over the
    # group's tasks, stage-3 workgroups dispatched after the other roles, few large-record
    # workgroups (each wave then takes many records of the list), stage-3 tasks in block order
    # and stage-1 tiles in XCD order (also with fewer stage-1 workgroups than tiles, each then
    # ranking several)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg, dev, ora = pair(oracle_mod, num_partitions=4096, replication_factor=3, segment_bytes=1 << 24,
                         index_interval=1024, max_batch_records=65536, pipeline_depth=4)
    with dev, ora:
        spec = StreamSpec(4096, 65536, "zipf", size=100, config_index=2)
        _pipelined(dev, ora, [make_batch(spec, b) for b in range(6)])
        hot = np.argsort([-ora.state(p)["log_end_offset"] for p in range(4096)])
        compare_state(dev, ora, cfg, parts=list(hot[:16]) + list(range(0, 4096, 257)))


@pytest.mark.parametrize("roles", ["0", "1", "3"])
def test_stage3_roles_mixed_sizes(oracle_mod, monkeypatch, roles):
    # stage 3 in loader / storer waves (RMQ_S3_ROLES) against the oracle: records of 0 B to 3 KB
    # (image tasks, tasks whose loader stores medium records' pieces itself, large-record waves),
    # launch groups with retention and ring wrap, a no-space partition, a partition not led and
    # unknown partitions
    monkeypatch.setenv("RMQ_S3_ROLES", roles)
    cfg, dev, ora = pair(oracle_mod, num_partitions=300, replication_factor=3, segment_bytes=1 << 18,
                         index_interval=256, max_batch_records=20000, pipeline_depth=4)
    with dev, ora:
        for e in (dev, ora):
            e.set_replicas(9, [1, 0, 2], 0)
        short = StreamSpec(300, 20000, "zipf", size=(0, 112), config_index=31, invalid_frac=0.005)
        mixed = StreamSpec(300, 6000, "uniform", size=(0, 3000), config_index=32)
        batches = [make_batch(short if b % 3 else mixed, b) for b in range(10)]
        nsp = make_batch(StreamSpec(300, 3000, "uniform", size=100, config_index=33), 0)
        nsp.pidx[:2500] = 5  # 2500 x 128 B > ring - I: partition 5 takes none of this batch's records
        batches.insert(4, nsp)
        _pipelined(dev, ora, batches)
        # a fetch right after the last launch: the log starts of groups that outgrew a ring
        # (late_retention before the fetch kernels), consumers at offset 0 (RMQ_EOFFSET below a start)
        pidx = np.arange(300, dtype=np.uint32)
        rd, resd, bd, _ = dev.fetch(pidx, np.zeros(300, np.uint32), np.full(300, 50, np.uint32))
        ro, reso, bo, _ = ora.fetch(pidx, np.zeros(300, np.uint32), np.full(300, 50, np.uint32))
        assert rd == ro and np.array_equal(resd, reso) and np.array_equal(bd, bo), "fetch differs"
        compare_state(dev, ora, cfg, full_rings=True)
        assert max(ora.state(p)["log_start_offset"] for p in range(300)) > 0, "scenario must exercise retention"


def test_config_B_pipelined(oracle_mod):
    # BASELINE configs[2] batches submitted back to back in groups of 4
    cfg, dev, ora = pair(oracle_mod, num_partitions=4096, replication_factor=3, segment_bytes=1 << 24,
                         index_interval=1024, max_batch_records=65536, pipeline_depth=4)
    with dev, ora:
        spec = StreamSpec(4096, 65536, "zipf", size=100, config_index=2)
        _pipelined(dev, ora, [make_batch(spec, b) for b in range(6)])
        hot = np.argsort([-ora.state(p)["log_end_offset"] for p in range(4096)])
        compare_state(dev, ora, cfg, parts=list(hot[:32]) + list(range(0, 4096, 131)))


def test_config_B_full_batches(oracle_mod):
    # BASELINE configs[2] at full size: 4096 partitions, Zipf s=1.1, 64k x 100 B, RF=3
    # (16 MiB rings: a 64k x 128 B batch is exactly 8 MiB, over the 8 MiB - interval batch limit)
    cfg, dev, ora = pair(oracle_mod, num_partitions=4096, replication_factor=3, segment_bytes=1 << 24,
                         index_interval=1024, max_batch_records=65536)
    with dev, ora:
        spec = StreamSpec(4096, 65536, "zipf", size=100, config_index=2)
        ops = [("append", make_batch(spec, b)) for b in range(3)]
        log = run_ops(dev, ora, cfg, ops, check=False)
        assert all(st["appended"] == 65536 for _, st in log), log
        compare_state(dev, ora, cfg)  # all 4096 partitions: state, every replica's ring window, index


def test_config_A_full_batches(oracle_mod):
    cfg, dev, ora = pair(oracle_mod, num_partitions=256, replication_factor=3, segment_bytes=1 << 24,
                         index_interval=1024, max_batch_records=65536)
    with dev, ora:
        spec = StreamSpec(256, 65536, "rr", size=100, config_index=1)
        log = run_ops(dev, ora, cfg, [("append", make_batch(spec, b)) for b in range(3)], check=False)
        assert all(st["appended"] == 65536 for _, st in log), log
        compare_state(dev, ora, cfg)


@pytest.mark.parametrize("P", [4097, 20000])
def test_multi_pass_sort(oracle_mod, P):
    # P > 256: two 8-bit radix passes over the partition keys
    cfg, dev, ora = pair(oracle_mod, num_partitions=P, replication_factor=2, segment_bytes=1 << 18,
                         index_interval=1024, max_batch_records=8192)
    with dev, ora:
        spec = StreamSpec(P, 1500, "zipf", size=(1, 120), config_index=19, invalid_frac=0.02)
        ops = [("append", make_batch(spec, b)) for b in range(3)]
        run_ops(dev, ora, cfg, ops, check=False)
        parts = sorted({int(p) for b in range(3) for p in make_batch(spec, b).pidx if p < P})[:300]
        compare_state(dev, ora, cfg, parts=parts)


def test_pinned_host_batches(oracle_mod):
    # RMQ_MEM_PINNED: caller arrays in page-locked memory (rmq_host_alloc), one DMA per section
    # and out offsets written by a DMA, submitted back to back (slots reused across groups);
    # packed and explicit payload offsets, unknown partitions
    cfg, dev, ora = pair(oracle_mod, num_partitions=256, replication_factor=3, segment_bytes=1 << 18,
                         index_interval=256, max_batch_records=8192, pipeline_depth=4)
    with dev, ora:
        spec = StreamSpec(256, 5000, "zipf", size=(0, 300), config_index=31, invalid_frac=0.01)
        batches = [make_batch(spec, b) for b in range(14)]
        subs = []
        for k, b in enumerate(batches):
            n = b.n
            pidx, lens, out = dev.host_empty(n, np.uint32), dev.host_empty(n, np.uint32), dev.host_empty(n, np.uint64)
            pay = dev.host_empty(max(b.payload.size, 1), np.uint8)
            pidx[:], lens[:], pay[:b.payload.size] = b.pidx, b.lens, b.payload
            poff = None
            if k % 3 == 2:  # explicit offsets
                poff = dev.host_empty(n, np.uint64)
                poff[:] = b.payload_offsets()
            t = dev.append_pinned_async(pidx, lens, pay, out, payload_off=poff, payload_bytes=b.payload.size)
            subs.append((t, out, poff))
        for (t, out, poff), b in zip(subs, batches):
            sd = dev.wait(t)
            oo, so = ora.append(b.pidx, b.lens, b.payload)
            assert sd == so, f"append stats gpu={sd} cpu={so}"
            assert np.array_equal(out, oo)
        compare_state(dev, ora, cfg, full_rings=True)
