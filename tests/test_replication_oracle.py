"""Replica-log rounds on the CPU oracle (FORMAT.md §9): every follower ends with its
leader's log, bytes and offsets; quorum acks commit; refused rounds (CRC, log mismatch) do not."""
import numpy as np
import pytest

from repl_sim import DIR, exchange_round, place, rank_batches, rank_cfg
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import rank_view, replica_ranks
from ripplemq_amd.workload import StreamSpec, make_batch

BASE = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 16, index_interval=256,
                    max_batch_records=4096)


def build(oracle_mod, world, ppr, rf=3, base=BASE):
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    oras = []
    for r in range(world):
        b = EngineConfig(**{**base.__dict__, "replication_factor": rf})
        o = oracle_mod.OracleEngine(rank_cfg(b, views[r], r))
        place(o, views[r], world)
        oras.append(o)
    return views, oras


def local_of(views, rank, gp):
    return int(np.flatnonzero(views[rank].gp == gp)[0])


def check_followers(views, oras, ppr, rf, full_ring=True):
    W = len(oras)
    for g in range(W):
        for gp in range(g * ppr, (g + 1) * ppr):
            lp = local_of(views, g, gp)
            ls = oras[g].state(lp)
            assert ls["commit"] == ls["log_end_offset"], (gp, ls)
            ring = oras[g].read_segment(0, lp)
            for slot, r in enumerate(replica_ranks(g, gp, W, rf)):
                if r == g:
                    continue
                fp = local_of(views, r, gp)
                fs = oras[r].state(fp)
                assert fs["log_end_offset"] == ls["log_end_offset"] and fs["log_end_pos"] == ls["log_end_pos"]
                assert fs["is_leader"] == 0
                assert np.array_equal(oras[r].read_segment(slot, fp), ring), f"gp {gp} slot {slot} ring"


@pytest.mark.parametrize("world,rf", [(2, 3), (3, 3), (4, 3), (8, 3), (8, 5)])
def test_rounds_replicate_every_log(oracle_mod, world, rf):
    ppr, G, R = 8, 2, 3
    views, oras = build(oracle_mod, world, ppr, rf)
    spec = StreamSpec(ppr, 300, "zipf", size=(0, 150), config_index=51)
    try:
        batches = [rank_batches(spec, r, R, G) for r in range(world)]
        for k in range(R):
            for r in range(world):
                for b in batches[r][k * G:(k + 1) * G]:
                    _, st = oras[r].append(b.pidx, b.lens, b.payload)
                    assert st["appended"] == b.n
            exchange_round(oras)
        check_followers(views, oras, ppr, rf)
        assert sum(int(o.counters()[0]) for o in oras) == (rf - 1) * sum(b.n for bs in batches for b in bs)
    finally:
        for o in oras:
            o.close()


def test_retention_on_followers_per_round(oracle_mod):
    # 64 KB rings: the hot partitions wrap inside a round; follower rings still equal the leader's
    world, ppr, G, R = 3, 4, 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 400, "zipf", size=(40, 160), config_index=52)
    try:
        for k in range(R):
            for r in range(world):
                for b in rank_batches(spec, r, R, G)[k * G:(k + 1) * G]:
                    oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras)
        check_followers(views, oras, ppr, 3)
        assert max(o.state(p)["log_start_offset"] for o in oras for p in range(len(views[0].gp))) > 0
    finally:
        for o in oras:
            o.close()


def test_refused_rounds_do_not_commit_on_their_own(oracle_mod):
    world, ppr = 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 200, "uniform", size=(1, 100), config_index=53)
    try:
        for r in range(world):
            b = rank_batches(spec, r, 1, 1)[0]
            oras[r].append(b.pidx, b.lens, b.payload)
        # rank 0's region to rank 1 has a flipped payload byte: rank 1 refuses the entry it hits,
        # rank 2 accepts everything, so rank 0's partitions still commit on the quorum {0, 2}
        regions = exchange_round(oras, keep_regions=True, corrupt=(0, 1, -5))
        assert oras[1].counters()[1] == 1
        for gp in range(ppr):
            s = oras[0].state(local_of(views, 0, gp))
            assert s["commit"] == s["log_end_offset"]
        # rank 2 misses rank 0's next round: the round after that no longer continues its log
        for k in (1, 2):
            for r in range(world):
                b = rank_batches(spec, r, 3, 1)[k]
                oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras, skip=(0, 2) if k == 1 else None)
        assert oras[2].counters()[2] > 0
        assert regions[0][1].size > 0
    finally:
        for o in oras:
            o.close()


def test_leader_change_truncates_follower(oracle_mod):
    # Raft's follower truncation (FORMAT.md §9): rank 0's third round is lost, leadership of its
    # partitions moves to slot 1 at term 2; rank 0 drops its uncommitted tail and follows
    from repl_sim import leader_change_script, run_script_oracle
    world, rf, ppr, group = 3, 3, 6, 2
    spec = StreamSpec(ppr, 300, "uniform", size=(0, 120), config_index=71)
    base = EngineConfig(num_partitions=1, replication_factor=rf, segment_bytes=1 << 16, index_interval=256,
                        max_batch_records=4096, pipeline_depth=group)
    views, new, phases = leader_change_script(spec, world, rf, ppr, group)
    cfgs = [rank_cfg(base, views[r], r) for r in range(world)]
    oras = [oracle_mod.OracleEngine(c) for c in cfgs]
    try:
        for r in range(world):
            place(oras[r], views[r], world)
        # before the change: rank 0 holds a tail nobody else has
        run_script_oracle(oras, views, phases[:3], world)
        s0 = [oras[0].state(p) for p in range(ppr)]
        assert all(s["log_end_offset"] > s["commit"] for s in s0)
        f1 = {int(views[1].gp[i]): oras[1].state(i) for i in range(len(views[1].gp))}
        assert all(f1[int(views[0].gp[p])]["log_end_offset"] == s0[p]["commit"] for p in range(ppr)
                   if int(views[0].gp[p]) in f1)
        run_script_oracle(oras, views, phases[3:], world)
        c = oras[0].counters()
        assert c[1] == 0 and c[2] == 0, c  # nothing refused: rank 0 truncated and accepted
        for p in range(ppr):  # rank 0 now follows: same log end and term as the new leader
            g = int(views[0].gp[p])
            r1 = int(views[0].ranks[p][1])
            q = int(np.flatnonzero(views[r1].gp == g)[0])
            lead, fol = oras[r1].state(q), oras[0].state(p)
            assert fol["log_end_offset"] == lead["log_end_offset"] and fol["term"] == 2 == lead["term"]
            assert lead["commit"] == lead["log_end_offset"] > s0[p]["commit"]
            assert fol["log_end_pos"] == lead["log_end_pos"]
            a = oras[0].read_segment(int(np.flatnonzero(views[0].ranks[p] == 0)[0]), p)
            b = oras[r1].read_segment(int(np.flatnonzero(views[r1].ranks[q] == r1)[0]), q)
            lo, hi = fol["log_start_pos"], fol["log_end_pos"]
            S = fol["segment_bytes"]
            idx = (np.arange(lo, hi) % S)
            assert np.array_equal(a[idx], b[idx])
    finally:
        for o in oras:
            o.close()


def _follower_views(views, oras, g, gp):
    """[(rank, local pidx, slot)] of the followers of global partition gp led by rank g."""
    W = len(oras)
    rf = views[0].ranks.shape[1]
    out = []
    for slot, r in enumerate(replica_ranks(g, gp, W, rf)):
        if r != g:
            out.append((r, local_of(views, r, gp), slot))
    return out


def test_crc_refusal_then_catch_up(oracle_mod):
    # FORMAT.md §9 v3: a corrupted record makes the follower refuse that entry (its log does not
    # move), the refused ack becomes a catch-up request, and the next round's entry for that
    # follower starts at its log end and re-sends the gap from the leader's ring
    world, ppr = 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 200, "uniform", size=(1, 100), config_index=54)
    try:
        def rnd(k, **kw):
            for r in range(world):
                b = rank_batches(spec, r, 4, 1)[k]
                oras[r].append(b.pidx, b.lens, b.payload)
            return exchange_round(oras, keep_regions=True, **kw)

        rnd(0)
        before = [oras[1].state(p) for p in range(len(views[1].gp))]
        regions = rnd(1, corrupt=(0, 1, -5))
        assert oras[1].counters()[1] == 1  # one entry refused for its CRC
        after = [oras[1].state(p) for p in range(len(views[1].gp))]
        for st in before + after:  # (a refused entry still comes from a live leader: heard either way)
            st.pop("heard_round")
        moved = [p for p in range(len(views[1].gp)) if after[p] != before[p]]
        unmoved = [p for p in range(len(views[1].gp)) if after[p] == before[p]]
        assert unmoved and moved  # the refused entry's partition stayed, the others advanced
        c0 = oras[0].counters()
        rnd(2)  # the plan of round 2 sends the gap first
        assert oras[0].counters()[4] == c0[4] + 1  # one catch-up entry
        check_followers(views, oras, ppr, 3)
        assert regions[0][1].size > 0
    finally:
        for o in oras:
            o.close()


def test_missed_round_then_catch_up(oracle_mod):
    world, ppr = 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 300, "zipf", size=(0, 150), config_index=55)
    try:
        for k in range(4):
            for r in range(world):
                b = rank_batches(spec, r, 4, 1)[k]
                oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras, drop=(0,) if k == 1 else ())
            if k == 1:
                # every follower of rank 0 missed the round; rank 0's partitions have not committed it
                assert oras[1].counters()[2] > 0 and oras[2].counters()[2] > 0
                assert all(oras[0].state(p)["commit"] < oras[0].state(p)["log_end_offset"]
                           for p in range(ppr))
        check_followers(views, oras, ppr, 3)
        assert oras[0].counters()[4] >= 2  # catch-up entries to both followers
    finally:
        for o in oras:
            o.close()


def test_partial_catch_up_after_three_missed_rounds(oracle_mod):
    # the GPU test's scenario (test_partial_catch_up_gpu) on the oracle alone
    world, ppr = 3, 2
    base = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 19, index_interval=256,
                        max_batch_records=400, max_batch_bytes=48 << 10, pipeline_depth=1)
    views, oras = build(oracle_mod, world, ppr, base=base)
    big = StreamSpec(2, 400, "uniform", size=(80, 120), config_index=83)
    small = StreamSpec(2, 4, "uniform", size=(10, 20), config_index=84)
    try:
        for k in range(12):
            for r in range(world):
                b = make_batch(small if k >= 3 else big, 1000 * r + 50 * k)
                oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras, drop=(0,) if k < 3 else ())
        assert oras[0].counters()[4] >= 4
        check_followers(views, oras, ppr, 3)
    finally:
        for o in oras:
            o.close()


def test_partial_catch_up_within_the_reserve(oracle_mod):
    # a gap larger than the destination's catch-up reserve is re-sent in pieces that end on sparse
    # index entries, one per round, until the follower holds the leader's log again
    world, ppr = 3, 2
    base = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 17, index_interval=256,
                        max_batch_records=64, max_batch_bytes=2048, pipeline_depth=1)
    views, oras = build(oracle_mod, world, ppr, base=base)
    assert oras[0].catchup_reserve() == 39 * 64 + 2048
    big = StreamSpec(ppr, 400, "uniform", size=(80, 120), config_index=56)
    small = StreamSpec(ppr, 4, "uniform", size=(10, 20), config_index=57)
    try:
        for r in range(world):
            b = rank_batches(big, r, 1, 1)[0]
            oras[r].append(b.pidx, b.lens, b.payload)
        exchange_round(oras, drop=(0,))
        rounds = 0
        while rounds < 40:
            for r in range(world):
                b = rank_batches(small, r, 40, 1)[rounds]
                oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras)
            rounds += 1
            lead = [oras[0].state(p) for p in range(ppr)]
            if all(s["commit"] == s["log_end_offset"] for s in lead):
                break
        assert 4 <= rounds < 40, rounds  # ~50 KB of gap per follower at < 4.5 KB per round
        check_followers(views, oras, ppr, 3)
    finally:
        for o in oras:
            o.close()


def _logical(o, slot, p, a, b):
    """Bytes [a, b) of partition p's log as stored in replica slot `slot` of engine o."""
    ring = o.read_segment(slot, p)
    S = ring.size
    return np.array([ring[x % S] for x in range(a, b)], np.uint8)


def test_gap_beyond_the_ring_rebases(oracle_mod):
    # a follower whose log end the leader's ring no longer holds restarts its log at the rebase
    # point (FORMAT.md §9: Raft's InstallSnapshot with the leader's retained log as the snapshot)
    # and is caught up from there; its retained records equal the leader's
    world, ppr = 3, 1
    base = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 13, index_interval=256)
    views, oras = build(oracle_mod, world, ppr, base=base)
    spec = StreamSpec(ppr, 10, "uniform", size=(100, 100), config_index=58)  # 1.3 KB per round
    try:
        gp = int(views[0].gp[0])
        (r1, p1, s1), (r2, p2, s2) = _follower_views(views, oras, 0, gp)
        far_rank, far_p, far_slot = (r1, p1, s1) if r1 == 1 else (r2, p2, s2)
        for k in range(12):
            for r in range(world):
                b = rank_batches(spec, r, 12, 1)[k]
                oras[r].append(b.pidx, b.lens, b.payload)
            # round 0 is missed by both followers; rank 1 loses rounds 1..8 as well (no region, no
            # ack): by then its log end lies more than the 8 KB ring behind
            exchange_round(oras, drop=(0,) if k == 0 else (), skip=(0, 1) if 1 <= k <= 8 else None)
            if k == 8:
                before = oras[far_rank].state(far_p)
        assert oras[0].counters()[5] == 0  # every plan toward rank 1 found its rebase point
        lead = oras[0].state(0)
        far = oras[far_rank].state(far_p)
        assert before["log_end_offset"] < far["log_start_offset"], "the follower's log restarted"
        assert far["log_end_offset"] == lead["log_end_offset"] and far["log_end_pos"] == lead["log_end_pos"]
        assert lead["commit"] == lead["log_end_offset"]
        a, b = far["log_start_pos"], far["log_end_pos"]
        assert b > a
        assert np.array_equal(_logical(oras[far_rank], far_slot, far_p, a, b),
                              _logical(oras[0], lead["leader_slot"], 0, a, b))
    finally:
        for o in oras:
            o.close()


def test_consumer_offsets_replicate_and_survive_leader_change(oracle_mod):
    # ConsumerOffsetUpdateRequestProcessor.java:59-60 applies an offset commit through Raft on every
    # replica; after leadership moves, the new leader serves the same offsets
    from repl_sim import moved_leadership
    world, ppr = 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 300, "uniform", size=(1, 60), config_index=59)
    C = oras[0].cfg.max_consumers
    try:
        for k in range(2):
            for r in range(world):
                b = rank_batches(spec, r, 3, 1)[k]
                oras[r].append(b.pidx, b.lens, b.payload)
            if k == 1:
                for r in range(world):  # every leader commits offsets of its partitions
                    led = np.arange(views[r].led, dtype=np.uint32)
                    rc, st = oras[r].commit_consumer_offset(np.repeat(led, 2), np.tile([0, 3], len(led)),
                                                            np.arange(2 * len(led), dtype=np.uint64) * 7 + r)
                    assert rc == 0 and not st.any()
            exchange_round(oras)
        for g in range(world):
            for gp in range(g * ppr, (g + 1) * ppr):
                want = oras[g].consumer_offsets(local_of(views, g, gp))
                assert want.any()
                for r, p, _ in _follower_views(views, oras, g, gp):
                    assert np.array_equal(oras[r].consumer_offsets(p), want), (g, gp, r)
        # leadership of rank 0's partitions moves to replica slot 1, term 2
        new = moved_leadership(views)
        for r in range(world):
            place(oras[r], new[r])
        for p in range(ppr):
            gp = int(views[0].gp[p])
            r1 = int(views[0].ranks[p][1])
            q = local_of(views, r1, gp)
            oras[r1].become_leader(q, 2)
            want = oras[0].consumer_offsets(p)
            assert np.array_equal(oras[r1].consumer_offsets(q), want)
            _, res, _, _ = oras[r1].fetch([q], [3], [5])
            assert int(res["start_offset"][0]) == int(want[3]) and res["status"][0] == 0
        assert C >= 4
    finally:
        for o in oras:
            o.close()


# Byte positions of a region (FORMAT.md §9) a corrupted link may flip: header key sum, directory
# words of entry 1 (count, bytes/16, first offset, table start, data start/16), the record-table
# slot of record 3 (its data position), and a payload byte of the last record.
REGION_FAULTS = {"keysum": 16, "count": 64 + DIR + 0, "bytes16": 64 + DIR + 4, "first": 64 + DIR + 8,
                 "tstart": 64 + DIR + 16, "dstart16": 64 + DIR + 20, "table_slot": None, "payload": -5}


@pytest.mark.parametrize("what", sorted(REGION_FAULTS))
def test_corrupted_region_refused_then_caught_up(oracle_mod, what):
    # a flipped directory / header / table byte must never be accepted (a wrong count or
    # byte total would move the follower's log end over bytes no record fills): the region's
    # structure (entries tile the table and data sections, every slot inside its entry, the records
    # filling each entry exactly) refuses it; catch-up heals it in the next rounds
    world, ppr = 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 200, "uniform", size=(1, 100), config_index=55)
    n_entries = oras[0].pair_entries(0, 1)
    at = REGION_FAULTS[what]
    if at is None:
        at = 64 + DIR * n_entries + 8 * 3 + 4
    try:
        def rnd(k, **kw):
            for r in range(world):
                b = rank_batches(spec, r, 5, 1)[k]
                oras[r].append(b.pidx, b.lens, b.payload)
            return exchange_round(oras, keep_regions=True, **kw)

        rnd(0)
        c1 = oras[1].counters().copy()
        rnd(1, corrupt=(0, 1, at))
        c = oras[1].counters()
        refused = int(c[1] - c1[1] + c[2] - c1[2])
        structural = what not in ("payload", "first", "table_slot")
        assert refused == (n_entries if structural else 1), (what, c, c1)
        if what == "keysum":  # unreadable header: every entry refused like a missed round
            assert c[2] - c1[2] == n_entries
        for k in (2, 3, 4):
            rnd(k)
        check_followers(views, oras, ppr, 3)
    finally:
        for o in oras:
            o.close()
