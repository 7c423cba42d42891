"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo), SURVEY §8(e).

Partition sharding must be invisible: routing a global stream to per-rank engines (each holding
its own partition range) gives exactly the offsets, partition state and replica-ring bytes of one
engine holding every partition. Ranks are separate processes talking over gloo (127.0.0.1), as
bench.py's ranks do; the max-over-ranks timing reduction is exercised on the way.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np

from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import merge_offsets, split_batch
from ripplemq_amd.workload import StreamSpec, make_batch

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_split_preserves_partition_order():
    g = np.random.default_rng(1)
    pidx = g.integers(0, 40, 500).astype(np.uint32)
    lens = g.integers(0, 30, 500).astype(np.uint32)
    shards = split_batch(pidx, lens, 4, 10)
    assert sum(len(s.records) for s in shards) == 500
    for s in shards:
        assert np.all(np.diff(s.records) > 0)                 # batch order kept
        assert np.all(s.pidx < 10)
        assert np.array_equal(pidx[s.records], s.pidx + 10 * s.rank)
    off = merge_offsets(500, shards, [np.arange(len(s.records), dtype=np.uint64) for s in shards])
    assert not np.any(off == np.iinfo(np.uint64).max)


def test_gloo_two_ranks_match_single_engine(oracle_mod, tmp_path):
    world, p_local, batches = 2, 12, 5
    out = tmp_path / "dist.json"
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(out),
                                       str(p_local), str(batches)], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    ranks = json.loads(out.read_text())
    assert [r["rank"] for r in ranks] == list(range(world))
    assert len({r["t_max"] for r in ranks}) == 1              # every rank got the same max

    # one engine holding all world * p_local partitions
    cfg = EngineConfig(num_partitions=world * p_local, replication_factor=3, segment_bytes=1 << 16,
                       index_interval=256)
    spec = StreamSpec(world * p_local, 700, "zipf", size=(0, 90), config_index=31)
    with oracle_mod.OracleEngine(cfg) as one:
        for k in range(batches):
            b = make_batch(spec, k)
            want, _ = one.append(b.pidx, b.lens, b.payload)
            shards = split_batch(b.pidx, b.lens, world, p_local)
            got = merge_offsets(b.n, shards, [np.asarray(ranks[r]["offs"][k]["offsets"], np.uint64)
                                              for r in range(world)])
            for r in range(world):
                assert ranks[r]["offs"][k]["records"] == shards[r].records.tolist()
            assert np.array_equal(got, want)
        for r in range(world):
            for p in range(p_local):
                assert ranks[r]["states"][p] == one.state(r * p_local + p)
                for rep in range(3):
                    ring = one.read_segment(rep, r * p_local + p).tobytes()
                    assert ranks[r]["rings"][rep][p] == oracle_mod.crc32c(ring)


def test_gloo_two_ranks_replication_rounds(oracle_mod, tmp_path):
    # the replica-log round protocol (FORMAT.md §9) between two rank processes over gloo equals the
    # in-process simulation of the same rounds (tests/repl_sim.py), rank by rank
    from repl_sim import exchange_round, place, rank_batches, rank_cfg
    from ripplemq_amd.sharding import rank_view

    world, ppr, rounds, group = 2, 6, 3, 2
    out = tmp_path / "repl.json"
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_repl_worker.py"), str(out),
                                       str(ppr), str(rounds), str(group)], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    got = json.loads(out.read_text())
    base = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 16, index_interval=256)
    views = [rank_view(r, world, ppr, 3) for r in range(world)]
    spec = StreamSpec(ppr, 500, "zipf", size=(0, 120), config_index=71)
    oras = [oracle_mod.OracleEngine(rank_cfg(base, views[r], r)) for r in range(world)]
    try:
        for r in range(world):
            place(oras[r], views[r], world)
        batches = [rank_batches(spec, r, rounds, group) for r in range(world)]
        for k in range(rounds):
            for r in range(world):
                for b in batches[r][k * group:(k + 1) * group]:
                    oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras)
        for r in range(world):
            assert got[r]["rank"] == r
            for p in range(len(views[r].gp)):
                assert got[r]["states"][p] == oras[r].state(p)
                assert got[r]["rings"][p] == [oracle_mod.crc32c(oras[r].read_segment(s, p).tobytes())
                                              for s in range(3)]
        leaders = [oras[r].state(p) for r in range(world) for p in range(views[r].led)]
        assert all(s["commit"] == s["log_end_offset"] > 0 for s in leaders if s["log_end_offset"])
    finally:
        for o in oras:
            o.close()
