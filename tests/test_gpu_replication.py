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
from repl_sim import DIR, exchange_round, mask_commit, notice_round, place, rank_batches, rank_cfg
from ripplemq_amd.engine import Engine, EngineConfig, LocalHub
from ripplemq_amd.sharding import rank_view
from ripplemq_amd.workload import StreamSpec, make_batch

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
            notice_round(oras)  # the final rmq_sync's commit notices
            stats = [engs[r].replication_stats() for r in range(world)]
            for r in range(world):
                assert stats[r]["rounds"] == rounds and stats[r]["refused_crc"] == 0, stats
                assert stats[r]["refused_log"] == 0, stats
                assert stats[r]["records_ingested"] == int(oras[r].counters()[0]), (stats, oras[r].counters())
                # no consumer commits and no missed rounds: every destination took the steady plan,
                # so the regions compared below are that path's output
                assert stats[r]["general_plans"] == 0, stats
            for r in range(world):
                def local_slots(p, r=r):
                    return [s for s in range(rf) if views[r].ranks[p][s] == r]
                compare_state(engs[r], oras[r], cfgs[r], local_slots=local_slots)
                for d in range(world):
                    if d != r:  # (pipelined rounds: the carried commit word is masked, see mask_commit)
                        assert np.array_equal(mask_commit(engs[r].read_outbox(d)), mask_commit(regions[r][d])), \
                            f"region {r}->{d}"
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
            # the lost round is missed by rank 0's followers (refused, FORMAT.md §9 v3); nothing else
            for r in range(world):
                c = oras[r].counters()
                assert (stats[r]["refused_crc"], stats[r]["refused_log"]) == (int(c[1]), int(c[2])), (r, stats[r], c)
            assert stats[0]["refused_crc"] == 0 and all(s["refused_log"] > 0 for s in stats[1:])
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


def synced_rounds(oracle_mod, world, rf, ppr, group, rounds, spec, seg=1 << 16, interval=256, base_kw=None,
                  faults=None, commits=None, small=None, small_from=1):
    """Rounds with an rmq_sync on every rank after each one, so every plan sees the acks of every
    round before it — exactly the oracle's order (tests/repl_sim.py): each round's regions, the
    catch-up verdicts and the converged state must match bit for bit.
    faults[k] = {"drop": ranks, "corrupt": (src, dst, at)}; commits[k] = {rank: (pidx, consumer,
    offset)} committed by that leader before round k's appends; small: a StreamSpec for rounds >= 1."""
    faults = faults or {}
    commits = commits or {}
    kw = dict(num_partitions=1, replication_factor=rf, segment_bytes=seg, index_interval=interval,
              max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=group)
    kw.update(base_kw or {})
    base = EngineConfig(**kw)
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    cfgs = [rank_cfg(base, views[r], r) for r in range(world)]

    def batches_of(r, k):
        sp = small if (small is not None and k >= small_from) else spec
        return [make_batch(sp, 1000 * r + 50 * k + j) for j in range(group)]

    hub = LocalHub(world)
    engs = [Engine(c) for c in cfgs]
    regions_gpu = [None] * world
    try:
        def body(r):
            e = engs[r]
            e.attach_local(hub)
            place(e, views[r])
            for k in range(rounds):
                f = faults.get(k, {})
                if r in f.get("drop", ()):
                    e.fault_drop_rounds(1)
                if f.get("corrupt") and f["corrupt"][0] == r:
                    e.fault_corrupt(f["corrupt"][1], f["corrupt"][2])
                if r in commits.get(k, {}):
                    rc, st = e.commit_consumer_offset(*commits[k][r])
                    assert rc == 0 and not st.any(), (rc, st)
                for b in batches_of(r, k):
                    e.append_async(b.pidx, b.lens, b.payload)
                e.sync()
            regions_gpu[r] = [e.read_outbox(d) if d != r else None for d in range(world)]

        run_ranks(world, body)
        oras = [oracle_mod.OracleEngine(c) for c in cfgs]
        try:
            for r in range(world):
                place(oras[r], views[r], world)
            regions = None
            for k in range(rounds):
                f = faults.get(k, {})
                for r in range(world):
                    if r in commits.get(k, {}):
                        oras[r].commit_consumer_offset(*commits[k][r])
                    for b in batches_of(r, k):
                        oras[r].append(b.pidx, b.lens, b.payload)
                regions = exchange_round(oras, keep_regions=True, drop=f.get("drop", ()), corrupt=f.get("corrupt"))
                notice_round(oras)  # every round ends in an rmq_sync
            stats = [engs[r].replication_stats() for r in range(world)]
            for r in range(world):
                c = oras[r].counters()
                got = (stats[r]["records_ingested"], stats[r]["refused_crc"], stats[r]["refused_log"],
                       stats[r]["bytes_ingested"], stats[r]["catchup_entries"], stats[r]["detached_plans"])
                assert got == tuple(int(x) for x in c), (r, got, c)
            for r in range(world):
                def local_slots(p, r=r):
                    return [s for s in range(rf) if views[r].ranks[p][s] == r]
                compare_state(engs[r], oras[r], cfgs[r], local_slots=local_slots)
                for d in range(world):
                    if d != r and regions[r][d] is not None:
                        assert np.array_equal(regions_gpu[r][d], regions[r][d]), f"region {r}->{d}"
            return views, engs, oras, stats
        except BaseException:
            for o in oras:
                o.close()
            raise
    finally:
        for e in engs:
            e.close()
        hub.close()


def _close(res):
    for o in res[2]:
        o.close()


def test_crc_refusal_then_catch_up_gpu(oracle_mod):
    # a flipped payload byte on the link: rank 1 refuses the entry (the follower ingest's reject
    # path), its log does not move; the next round's entry re-sends the gap (catch-up)
    spec = StreamSpec(8, 600, "uniform", size=(1, 120), config_index=81)
    res = synced_rounds(oracle_mod, world=3, rf=3, ppr=8, group=2, rounds=4, spec=spec,
                        faults={1: {"corrupt": (0, 1, -5)}})
    try:
        stats = res[3]
        assert stats[1]["refused_crc"] == 1 and stats[0]["catchup_entries"] == 1, stats
        views, oras = res[0], res[2]
        lead = [oras[0].state(p) for p in range(views[0].led)]  # equal to the GPU's (checked above)
        assert all(s["commit"] == s["log_end_offset"] == s["match"][0] for s in lead)
        assert all(min(s["match"]) == s["log_end_offset"] for s in lead)  # every follower caught up
    finally:
        _close(res)


def test_missed_round_then_catch_up_gpu(oracle_mod):
    spec = StreamSpec(6, 400, "zipf", size=(0, 150), config_index=82)
    res = synced_rounds(oracle_mod, world=3, rf=3, ppr=6, group=2, rounds=4, spec=spec, faults={1: {"drop": (0,)}})
    try:
        stats = res[3]
        assert stats[1]["refused_log"] > 0 and stats[2]["refused_log"] > 0 and stats[0]["catchup_entries"] >= 2
        lead = [res[2][0].state(p) for p in range(res[0][0].led)]
        assert all(min(s["match"]) == s["log_end_offset"] for s in lead)
    finally:
        _close(res)


def test_partial_catch_up_gpu(oracle_mod):
    # a missed round larger than the destination's catch-up reserve comes back in pieces that end on
    # sparse-index entries, one per round
    big = StreamSpec(2, 400, "uniform", size=(80, 120), config_index=83)
    small = StreamSpec(2, 4, "uniform", size=(10, 20), config_index=84)
    # three rounds of ~51 KB each are missed: the gap (~150 KB per follower) is over twice the
    # reserve of one round bound (39 x 400 + 48 KiB)
    res = synced_rounds(oracle_mod, world=3, rf=3, ppr=2, group=1, rounds=12, spec=big, seg=1 << 19,
                        base_kw=dict(max_batch_records=400, max_batch_bytes=48 << 10),
                        faults={k: {"drop": (0,)} for k in range(3)}, small=small, small_from=3)
    try:
        assert res[2][0].catchup_reserve() == 39 * 400 + (48 << 10)
        assert res[3][0]["catchup_entries"] >= 4  # the gap took several rounds
        lead = [res[2][0].state(p) for p in range(2)]
        assert all(min(s["match"]) == s["log_end_offset"] for s in lead)
    finally:
        _close(res)


def test_follower_beyond_the_ring_rebases_gpu(oracle_mod):
    # rank 0's regions are lost for 9 rounds: its followers' log ends fall more than the 8 KB ring
    # behind, so the next plan restarts their logs at the leader's rebase point (FORMAT.md §9,
    # Raft's InstallSnapshot with the retained log as the snapshot) instead of detaching them;
    # regions, rings, index and state bit-exact with the oracle, and the quorum back to full
    spec = StreamSpec(1, 10, "uniform", size=(100, 100), config_index=58)  # 1.3 KB per round
    res = synced_rounds(oracle_mod, world=3, rf=3, ppr=1, group=1, rounds=12, spec=spec, seg=1 << 13,
                        faults={k: {"drop": (0,)} for k in range(9)})
    try:
        stats = res[3]
        assert stats[0]["detached_plans"] == 0 and stats[0]["catchup_entries"] >= 2, stats[0]
        assert stats[1]["refused_log"] > 0 and stats[2]["refused_log"] > 0
        lead = res[2][0].state(0)
        assert lead["log_start_offset"] > 0 and min(lead["match"]) == lead["log_end_offset"]
        starts = [res[2][r].state(p)["log_start_offset"] for r in (1, 2)
                  for p in range(res[0][r].led, res[2][r].cfg.num_partitions)]
        assert min(starts) > 0, "the followers' logs restarted past their old ends"
    finally:
        _close(res)


def test_consumer_offsets_replicate_and_survive_leader_change_gpu(oracle_mod):
    # ConsumerOffsetUpdateRequestProcessor.java:59-60: an offset commit is replicated; after the
    # leadership moves, the new leader serves the same offsets (fetch starts there)
    from repl_sim import moved_leadership
    world, rf, ppr = 3, 3, 4
    spec = StreamSpec(ppr, 300, "uniform", size=(1, 60), config_index=85)
    commits = {1: {r: (np.repeat(np.arange(ppr, dtype=np.uint32), 2), np.tile(np.array([0, 3], np.uint32), ppr),
                       np.arange(2 * ppr, dtype=np.uint64) * 7 + r) for r in range(world)}}
    res = synced_rounds(oracle_mod, world, rf, ppr, group=2, rounds=3, spec=spec, commits=commits)
    views, oras = res[0], res[2]
    try:
        for g in range(world):
            for p in range(ppr):
                want = oras[g].consumer_offsets(p)
                assert want.any()
        # a fresh world of engines replays nothing: move leadership on the oracle-checked engines
        # instead (their states equal the oracle's above) by a second GPU run with the move
    finally:
        _close(res)
    new = moved_leadership(views)
    base = EngineConfig(num_partitions=1, replication_factor=rf, segment_bytes=1 << 16, index_interval=256,
                        max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=2)
    cfgs = [rank_cfg(base, views[r], r) for r in range(world)]
    hub = LocalHub(world)
    engs = [Engine(c) for c in cfgs]
    fetched = [None] * world
    try:
        def body(r):
            e = engs[r]
            e.attach_local(hub)
            place(e, views[r])
            for k in range(2):
                if k == 1:
                    rc, _ = e.commit_consumer_offset(*commits[1][r])
                    assert rc == 0
                for j in range(2):
                    b = make_batch(spec, 1000 * r + 50 * k + j)
                    e.append_async(b.pidx, b.lens, b.payload)
                e.sync()
            place(e, new[r])
            moved = [p for p in range(len(views[r].gp))
                     if new[r].ranks[p][new[r].leader_slot[p]] == r and views[r].ranks[p][views[r].leader_slot[p]] != r]
            for p in moved:
                e.become_leader(p, 2)
            fetched[r] = {p: (e.consumer_offsets(p), e.fetch([p], [3], [5])[1]) for p in moved}
            e.sync()

        run_ranks(world, body)
        for r in range(world):
            for p, (offs, res_) in fetched[r].items():
                g = int(views[r].gp[p])
                src = g // ppr  # its old leader rank
                q = int(np.flatnonzero(views[src].gp == g)[0])
                want = np.zeros(cfgs[r].max_consumers, np.uint64)
                want[0], want[3] = 14 * q + src, 14 * q + 7 + src
                assert np.array_equal(offs, want), (r, p, offs, want)
                assert int(res_["start_offset"][0]) == int(want[3]) and res_["status"][0] == 0
        assert any(fetched[r] for r in range(world))
    finally:
        for e in engs:
            e.close()
        hub.close()


def test_idle_ranks_keep_rounds_flowing_gpu():
    # ripplemq_amd.pacer: every rank submits one batch per tick (empty when idle). Rank 0 produces
    # once; ranks 1 and 2 never produce. Without any rmq_sync, rank 0's records commit on a quorum
    # once enough ticks have passed, and its followers hold them.
    from ripplemq_amd.pacer import RoundPacer
    world, rf, ppr, group = 3, 3, 4, 2
    base = EngineConfig(num_partitions=1, replication_factor=rf, segment_bytes=1 << 16, index_interval=256,
                        max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=group)
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    cfgs = [rank_cfg(base, views[r], r) for r in range(world)]
    spec = StreamSpec(ppr, 500, "uniform", size=(1, 100), config_index=86)
    hub = LocalHub(world)
    engs = [Engine(c) for c in cfgs]
    got = [None] * world
    try:
        def body(r):
            e = engs[r]
            e.attach_local(hub)
            place(e, views[r])
            pacer = RoundPacer(e, epoch=0.0, tick_s=1.0, clock=lambda: 0.0)
            if r == 0:
                b = make_batch(spec, 7)
                pacer.submit(b.pidx, b.lens, b.payload)
            done, first = [], None
            for ticks in range(1, 25):  # every rank ticks the same number of times (rounds are collective)
                pacer.tick()
                if r == 0 and first is None:
                    done += pacer.committed()  # rmq_poll_commit without a flush: not collective
                    if done:
                        first = ticks
            got[r] = (first, done)
            e.sync()  # collective, before the engines go away

        run_ranks(world, body)
        first, done = got[0]
        assert done and first is not None, "rank 0's records never committed without an rmq_sync"
        pidx, offs = done[0]
        assert len(pidx) == spec.records and np.all(offs != np.uint64(0xFFFFFFFFFFFFFFFF))
        assert first <= 16, first  # ~ (3 pipeline launches + 3 ack launches) x 2 batches per round
    finally:
        for e in engs:
            e.close()
        hub.close()


@pytest.mark.parametrize("what", ["keysum", "count", "bytes16", "first", "dstart16", "table_slot"])
def test_corrupted_region_refused_gpu(oracle_mod, what):
    # a flipped header / directory / record-table byte (rmq_fault_corrupt at >= 0) is
    # refused by the follower ingest exactly as the oracle refuses it (whole region for a structural
    # fault, one entry otherwise), nothing past the refused bytes is written, and the catch-up of
    # the next rounds brings every follower back bit-exact with the oracle
    from test_replication_oracle import REGION_FAULTS
    world, rf, ppr = 3, 3, 6
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    n01 = sum(1 for p in range(ppr) for s in range(1, rf) if int(views[0].ranks[p][s]) == 1)
    at = REGION_FAULTS[what]
    if at is None:
        at = 64 + DIR * n01 + 8 * 3 + 4
    spec = StreamSpec(ppr, 500, "uniform", size=(1, 120), config_index=87)
    res = synced_rounds(oracle_mod, world, rf, ppr, group=2, rounds=5, spec=spec,
                        faults={1: {"corrupt": (0, 1, at)}})
    try:
        stats = res[3]
        refused = stats[1]["refused_crc"] + stats[1]["refused_log"]
        structural = what in ("keysum", "count", "bytes16", "dstart16")
        assert refused == (n01 if structural else 1), (what, stats[1])
        lead = [res[2][0].state(p) for p in range(ppr)]
        assert all(min(s["match"]) == s["log_end_offset"] for s in lead)  # every follower caught up
    finally:
        _close(res)
