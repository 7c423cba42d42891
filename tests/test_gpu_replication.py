"""GPU replica-log rounds (FORMAT.md §9) between engines on one GPU.

The engines of a world share the in-process transport (rmq_attach_local); each is driven by its own
thread, as each rank would be by its own process over RCCL. Every rank's state after rmq_sync —
leader and follower partition state, every local replica ring, the sparse index, the leaders'
matchIndex rows and commits — and the last round's region bytes must equal the oracle's
simulation of the same rounds (tests/repl_sim.py).
"""
import threading

import numpy as np
import pytest

from parity import compare_state
from repl_sim import exchange_round, place, rank_batches, rank_cfg
from ripplemq_amd.engine import Engine, EngineConfig, LocalHub
from ripplemq_amd.sharding import rank_view
from ripplemq_amd.workload import StreamSpec

pytestmark = pytest.mark.gpu


def run_ranks(world, body, timeout=240):
    errs = [None] * world

    def wrap(r):
        try:
            body(r)
        except BaseException as ex:  # noqa: BLE001 - reported below
            errs[r] = ex

    ts = [threading.Thread(target=wrap, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
        assert not t.is_alive(), "a rank hung"
    for r, ex in enumerate(errs):
        if ex is not None:
            raise AssertionError(f"rank {r}: {ex!r}") from ex


def scenario(oracle_mod, world, rf, ppr, group, rounds, spec, seg=1 << 16, interval=256):
    base = EngineConfig(num_partitions=1, replication_factor=rf, segment_bytes=seg, index_interval=interval,
                        max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=group)
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    cfgs = [rank_cfg(base, views[r], r) for r in range(world)]
    batches = [rank_batches(spec, r, rounds, group) for r in range(world)]
    hub = LocalHub(world)
    engs = [Engine(c) for c in cfgs]
    try:
        def body(r):
            e = engs[r]
            e.attach_local(hub)
            place(e, views[r])
            for b in batches[r]:
                e.append_async(b.pidx, b.lens, b.payload)
            e.sync()

        run_ranks(world, body)
        oras = [oracle_mod.OracleEngine(c) for c in cfgs]
        try:
            for r in range(world):
                place(oras[r], views[r], world)
            regions = None
            for k in range(rounds):
                for r in range(world):
                    for b in batches[r][k * group:(k + 1) * group]:
                        oras[r].append(b.pidx, b.lens, b.payload)
                regions = exchange_round(oras, keep_regions=True)
            stats = [engs[r].replication_stats() for r in range(world)]
            for r in range(world):
                assert stats[r]["rounds"] == rounds and stats[r]["refused_crc"] == 0, stats
                assert stats[r]["refused_log"] == 0, stats
                assert stats[r]["records_ingested"] == int(oras[r].counters()[0]), (stats, oras[r].counters())
            for r in range(world):
                def local_slots(p, r=r):
                    return [s for s in range(rf) if views[r].ranks[p][s] == r]
                compare_state(engs[r], oras[r], cfgs[r], local_slots=local_slots)
                for d in range(world):
                    if d != r:
                        assert np.array_equal(engs[r].read_outbox(d), regions[r][d]), f"region {r}->{d}"
            leaders = [oras[r].state(p) for r in range(world) for p in range(views[r].led)]
            assert all(s["commit"] == s["log_end_offset"] for s in leaders)
            assert sum(s["log_end_offset"] for s in leaders) > 0
        finally:
            for o in oras:
                o.close()
    finally:
        for e in engs:
            e.close()
        hub.close()


def test_three_ranks_rf3(oracle_mod):
    scenario(oracle_mod, world=3, rf=3, ppr=16, group=2, rounds=4,
             spec=StreamSpec(16, 1500, "zipf", size=(0, 150), config_index=61))


def test_two_ranks_two_follower_slots(oracle_mod):
    # world 2, RF 3: both followers of every partition live on the other rank (two slots there)
    scenario(oracle_mod, world=2, rf=3, ppr=8, group=3, rounds=3,
             spec=StreamSpec(8, 900, "uniform", size=(1, 300), config_index=62))


def test_four_ranks_rf5_large_records_wrap(oracle_mod):
    # config D's shape at small scale: RF 5, 64 B..16 KB records, rings wrapping inside a round
    scenario(oracle_mod, world=4, rf=5, ppr=6, group=2, rounds=3,
             spec=StreamSpec(6, 60, "uniform", size=(64, 16384), config_index=63), seg=1 << 18, interval=1024)


def test_leader_change_truncates_follower(oracle_mod):
    # Raft's follower truncation (FORMAT.md §9) on the GPU engines: rank 0's third round is lost
    # (rmq_fault_drop_rounds), and while those batches are still in flight the placement moves the
    # leadership of rank 0's partitions to replica slot 1, which starts term 2; the new leaders'
    # rounds make rank 0 drop its uncommitted tail and follow. Every rank, ring and region must equal
    # the oracle's run of the same script.
    from repl_sim import leader_change_script, run_script_oracle
    world, rf, ppr, group = 3, 3, 6, 2
    spec = StreamSpec(ppr, 300, "uniform", size=(0, 120), config_index=71)
    base = EngineConfig(num_partitions=1, replication_factor=rf, segment_bytes=1 << 16, index_interval=256,
                        max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=group)
    views, new, phases = leader_change_script(spec, world, rf, ppr, group)
    cfgs = [rank_cfg(base, views[r], r) for r in range(world)]
    hub = LocalHub(world)
    engs = [Engine(c) for c in cfgs]
    try:
        def body(r):
            e = engs[r]
            e.attach_local(hub)
            place(e, views[r])
            for k, (batches, drop, placement, bl) in enumerate(phases):
                if placement is not None:
                    place(e, placement[r])  # collective: drains the previous phase's batches first
                    for p, t in bl[r]:
                        e.become_leader(p, t)
                if r in drop:
                    e.fault_drop_rounds(1)
                for b in batches[r]:
                    e.append_async(b.pidx, b.lens, b.payload)
                if k != 2:  # the lost round's batches are still in flight at the placement change
                    e.sync()

        run_ranks(world, body)
        oras = [oracle_mod.OracleEngine(c) for c in cfgs]
        try:
            for r in range(world):
                place(oras[r], views[r], world)
            regions = run_script_oracle(oras, views, phases, world)
            for r in range(world):
                def local_slots(p, r=r):
                    return [s for s in range(rf) if views[r].ranks[p][s] == r]
                compare_state(engs[r], oras[r], cfgs[r], local_slots=local_slots)
                for d in range(world):
                    if d != r:
                        assert np.array_equal(engs[r].read_outbox(d), regions[r][d]), f"region {r}->{d}"
            stats = [engs[r].replication_stats() for r in range(world)]
            assert all(s["refused_crc"] == 0 and s["refused_log"] == 0 for s in stats), stats
            for p in range(ppr):  # rank 0 follows its former partitions at term 2, truncated to the leader
                st = engs[0].state(p)
                assert st["term"] == 2 and not st["is_leader"]
                assert st["log_end_offset"] == oras[0].state(p)["log_end_offset"]
        finally:
            for o in oras:
                o.close()
    finally:
        for e in engs:
            e.close()
        hub.close()
