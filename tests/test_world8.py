"""World-8 replication parity at BASELINE.json's multi-GPU shapes, on ONE GPU.

configs[3]: 8 ranks, 4,096 partitions led per rank (32,768 in all), RF 3, uniform 100 B records; each
rank's followers spread over all 7 peers (ripplemq_amd.sharding.replica_ranks; the intent of
PartitionAssigner.java:81-89). Rounds run pipelined (no rmq_sync between them), as the bench runs
them; small rings make most partitions wrap.

configs[4]: 8 ranks, 4,096 partitions in all (512 led per rank), RF 5, log-uniform 64 B..16 KB
records; 4 consumers per partition commit lagging offsets on the leaders and fetch at max = 10
(ConsumerClientImpl.java:21) and max = 1024 between the rounds (PartitionStateMachine.java:85-110).

The eight GPU engines share the in-process transport (each driven by its own host thread, as each
rank would be by its own process over RCCL) and every rank's states, rings, index, consumer offsets,
fetch results and round regions must equal eight oracles running the same rounds
(tests/repl_sim.py, tests/world_script.py). The RCCL path itself runs only on an 8-GPU node (the
driver's scaling job).
"""
from __future__ import annotations

import threading

import numpy as np
import pytest

from parity import compare_bulk
from repl_sim import exchange_round, mask_commit, notice_round, place, rank_cfg
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import rank_view
from ripplemq_amd.workload import StreamSpec, make_batch
from world_script import compare_outcomes, run_gpu, run_oracle

WORLD = 8


def c_shape():
    rf, ppr, group, rounds = 3, 4096, 2, 3
    base = EngineConfig(num_partitions=1, replication_factor=rf, segment_bytes=1 << 10, index_interval=256,
                        max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=group)
    views = [rank_view(r, WORLD, ppr, rf) for r in range(WORLD)]
    spec = StreamSpec(ppr, 4096, "uniform", size=100, config_index=3)
    batches = [[make_batch(spec, 1000 * r + k) for k in range(rounds * group)] for r in range(WORLD)]
    return base, views, batches, rounds, group


def d_shape(rounds=4, consumers=4):
    rf, ppr, group = 5, 4096 // WORLD, 2
    base = dict(num_partitions=1, replication_factor=rf, segment_bytes=1 << 15, index_interval=1024,
                max_batch_records=4096, max_batch_bytes=4 << 20, pipeline_depth=group)
    views = [rank_view(r, WORLD, ppr, rf) for r in range(WORLD)]
    spec = StreamSpec(ppr, 400, "uniform", size=(64, 16384), config_index=4)
    g = np.random.default_rng(0x52495054)
    appended = np.zeros((WORLD, ppr), np.int64)  # per led partition, every record a leader took
    script = []
    pp = np.repeat(np.arange(ppr, dtype=np.uint32), consumers)
    cc = np.tile(np.arange(consumers, dtype=np.uint32), ppr)
    for k in range(rounds):
        if k:  # consumers lagging the log end by U[0, log end], a few past it (empty fetches)
            commits = {}
            for r in range(WORLD):
                end = np.repeat(appended[r], consumers)
                lag = (g.random(end.size) * (end + 1)).astype(np.int64)
                off = end - lag + (g.random(end.size) < 0.05) * 3
                commits[r] = (pp, cc, off.astype(np.uint64))
            script.append(("commit", commits))
        rnd = {}
        for r in range(WORLD):
            rnd[r] = [make_batch(spec, 1000 * r + group * k + j) for j in range(group)]
            for b in rnd[r]:
                appended[r] += np.bincount(b.pidx, minlength=ppr)  # (upper bound: no-space rejections)
        script.append(("round", rnd))
        for mx in (10, 1024):
            script.append(("fetch", {r: (pp, cc, np.full(pp.size, mx, np.uint32)) for r in range(WORLD)}))
    return base, views, script


def _run_c_oracle(oracle_mod, base, views, batches, rounds, group):
    cfgs = [rank_cfg(base, views[r], r) for r in range(WORLD)]
    oras = [oracle_mod.OracleEngine(c) for c in cfgs]
    for r in range(WORLD):
        place(oras[r], views[r], WORLD)
    regions = None
    appended = 0
    for k in range(rounds):
        for r in range(WORLD):
            for b in batches[r][k * group:(k + 1) * group]:
                appended += oras[r].append(b.pidx, b.lens, b.payload)[1]["appended"]
        regions = exchange_round(oras, keep_regions=True)
    notice_round(oras)  # the final rmq_sync
    oras[0].appended_total = appended
    return cfgs, oras, regions


def test_world8_config_c_shape_oracle(oracle_mod):
    # the oracle side alone: every follower replica (two per partition, on 7 peers) holds its
    # leader's log, every leader's commit is its log end, and the rings wrapped
    base, views, batches, rounds, group = c_shape()
    cfgs, oras, _ = _run_c_oracle(oracle_mod, base, views, batches, rounds, group)
    try:
        peers = {r: set() for r in range(WORLD)}
        for r in range(WORLD):
            for p in range(views[r].led):
                peers[r] |= set(int(x) for x in views[r].ranks[p][1:])
            st = oras[r].states()
            led = st[:views[r].led]
            assert np.all(led["commit"] == led["log_end_offset"]) and np.all(led["leader_commit"] == led["commit"])
            fol = st[views[r].led:]
            assert np.all(fol["commit"] == fol["log_end_offset"])  # learned from the commit notices
            assert np.any(st["log_start_offset"] > 0)  # retention moved
        assert all(len(peers[r]) == WORLD - 1 for r in range(WORLD))  # followers over all 7 peers
        total = sum(int(o.counters()[0]) for o in oras)
        assert total == 2 * oras[0].appended_total  # (a few (batch, partition) cells overflow 1 KiB rings)
        assert oras[0].appended_total > 0.99 * sum(b.n for bs in batches for b in bs)
    finally:
        for o in oras:
            o.close()


def test_world8_config_d_shape_oracle(oracle_mod):
    base, views, script = d_shape(rounds=3)
    cfgs = [rank_cfg(EngineConfig(**base), views[r], r) for r in range(WORLD)]
    oras = [oracle_mod.OracleEngine(c) for c in cfgs]
    try:
        out = run_oracle(oras, views, script)
        stat = np.concatenate([rec[1]["status"] for k, s in enumerate(script) if s[0] == "fetch"
                               for rec in out[k] if rec is not None])
        counts = np.concatenate([rec[1]["count"] for k, s in enumerate(script) if s[0] == "fetch"
                                 for rec in out[k] if rec is not None])
        assert np.all(np.isin(stat, (0, -6))) and counts.sum() > 0 and np.any(counts == 0)
        assert np.any(counts > 10)  # max = 1024 reads
        assert all(int(o.counters()[1] + o.counters()[2]) == 0 for o in oras)
    finally:
        for o in oras:
            o.close()


@pytest.mark.gpu
def test_world8_config_c_shape_gpu(oracle_mod):
    from ripplemq_amd.engine import Engine, LocalHub

    base, views, batches, rounds, group = c_shape()
    cfgs = [rank_cfg(base, views[r], r) for r in range(WORLD)]
    hub = LocalHub(WORLD)
    engs = [Engine(c) for c in cfgs]
    errs = [None] * WORLD
    try:
        def body(r):
            try:
                e = engs[r]
                e.attach_local(hub)
                place(e, views[r])
                for b in batches[r]:
                    e.append_async(b.pidx, b.lens, b.payload)  # pipelined: one rmq_sync at the end
                e.sync()
            except BaseException as ex:  # noqa: BLE001 - reported below
                errs[r] = ex

        ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(WORLD)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(240)
            assert not t.is_alive(), "a rank hung"
        assert not any(errs), errs
        cfgs, oras, regions = _run_c_oracle(oracle_mod, base, views, batches, rounds, group)
        try:
            for r in range(WORLD):
                st = engs[r].replication_stats()
                c = oras[r].counters()
                assert st["rounds"] == rounds and st["refused_crc"] == 0 and st["refused_log"] == 0, st
                assert st["records_ingested"] == int(c[0]) and st["general_plans"] == 0, (st, c)
            for r in range(WORLD):
                def local_slots(p, r=r):
                    return [s for s in range(3) if views[r].ranks[p][s] == r]
                compare_bulk(engs[r], oras[r], cfgs[r], local_slots=local_slots)
                for d in range(WORLD):
                    if d != r:  # (pipelined rounds: the carried commit word is masked, see mask_commit)
                        assert np.array_equal(mask_commit(engs[r].read_outbox(d)), mask_commit(regions[r][d])), \
                            f"region {r}->{d}"
        finally:
            for o in oras:
                o.close()
    finally:
        for e in engs:
            e.close()
        hub.close()


@pytest.mark.gpu
def test_world8_config_d_shape_gpu(oracle_mod):
    from ripplemq_amd.engine import Engine, LocalHub

    base, views, script = d_shape()
    cfgs = [rank_cfg(EngineConfig(**base), views[r], r) for r in range(WORLD)]
    hub = LocalHub(WORLD)
    engs = [Engine(c) for c in cfgs]
    oras = []
    try:
        got = run_gpu(engs, hub, views, script)
        oras = [oracle_mod.OracleEngine(c) for c in cfgs]
        want = run_oracle(oras, views, script)
        compare_outcomes(script, got, want)
        for r in range(WORLD):
            def local_slots(p, r=r):
                return [s for s in range(5) if views[r].ranks[p][s] == r]
            compare_bulk(engs[r], oras[r], cfgs[r], local_slots=local_slots)
            st = engs[r].replication_stats()
            assert st["refused_crc"] == 0 and st["refused_log"] == 0, st
    finally:
        for o in oras:
            o.close()
        for e in engs:
            e.close()
        hub.close()
