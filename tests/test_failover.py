"""Failover correctness of the replica-log rounds (FORMAT.md §6, §9 v4).

Reference: every replica of a jraft partition group applies the committed entries
(PartitionStateMachine.onApply, mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:37-62),
so a new leader's handleBatchRead (:85-110) serves every committed message at once; jraft elects only
a replica holding every committed entry (Raft's vote restriction; election timeout
PartitionRaftServer.java:85) and commits the earlier terms' entries through the configuration entry
it appends at leader start [jraft]; replicas move to other brokers on membership changes
(PartitionManager.java:72-109, PartitionAssigner.java:68-89).

Each scenario is a step script (tests/world_script.py) run on per-rank oracles (CPU tests here,
checking the behaviour) and, marked gpu, on GPU engines over the in-process transport, where every
recorded outcome (become_leader statuses, fetch results and bytes, every round's regions) and every
rank's final state, rings, index and consumer offsets must equal the oracle's.
"""
from __future__ import annotations

import numpy as np
import pytest

from parity import compare_state
from repl_sim import led_batches, moved_leadership, rank_cfg
from ripplemq_amd import _abi as A
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import RankView, rank_view
from ripplemq_amd.workload import StreamSpec, make_batch
from world_script import compare_outcomes, run_gpu, run_oracle

BASE = dict(num_partitions=1, replication_factor=3, segment_bytes=1 << 16, index_interval=256,
            max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=2)


def _round(spec, world, k, group=2, ranks=None):
    return {r: [make_batch(spec, 1000 * r + 50 * k + j) for j in range(group)]
            for r in (range(world) if ranks is None else ranks)}


def new_leader_script(world=3, rf=3, ppr=4):
    """Two rounds with consumer commits on the leaders, then rank 0's partitions move to replica
    slot 1 (term 2) and the new leaders serve consumer 3 right away, before any new round."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    spec = StreamSpec(ppr, 300, "uniform", size=(1, 60), config_index=91)
    new = moved_leadership(views)
    commits = {r: (np.arange(ppr, dtype=np.uint32), np.full(ppr, 3, np.uint32),
                   np.arange(ppr, dtype=np.uint64) * 5 + 3) for r in range(world)}
    moved = {}
    for r in range(world):
        v = new[r]
        m = [int(p) for p in range(len(v.gp))
             if v.ranks[p][v.leader_slot[p]] == r and views[r].ranks[p][views[r].leader_slot[p]] != r]
        if m:
            moved[r] = m
    script = [("commit", commits), ("round", _round(spec, world, 0)), ("round", _round(spec, world, 1)),
              ("place", new), ("lead", {r: [(p, 2) for p in m] for r, m in moved.items()}),
              ("fetch", {r: (np.array(m, np.uint32), np.full(len(m), 3, np.uint32), np.full(len(m), 1000, np.uint32))
                         for r, m in moved.items()}),
              ("round", {r: led_batches(spec, new[r], r, 2, 55) for r in range(world)}),
              ("fetch", {r: (np.array(m, np.uint32), np.full(len(m), 3, np.uint32), np.full(len(m), 1000, np.uint32))
                         for r, m in moved.items()})]
    return views, script, BASE


def stale_replica_script(world=3, rf=3, ppr=4):
    """Rank 2 misses two of rank 0's rounds (a lost link, rmq_fault_isolate); rank 1 holds them and
    rank 0 commits on the quorum {0, 1}; the commit notices tell rank 2 how far the leader committed.
    Moving leadership of rank 0's partitions to rank 2 is refused (RMQ_ESTALE: rank 2 lacks committed
    records); moving it to rank 1 succeeds and the new leaders serve and replicate."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    spec = StreamSpec(ppr, 300, "uniform", size=(1, 60), config_index=92)

    def to_rank(target):
        out = []
        for v in views:
            ls = v.leader_slot.copy()
            for p in range(len(v.gp)):
                if int(v.ranks[p][v.leader_slot[p]]) == 0:
                    ls[p] = int(np.flatnonzero(v.ranks[p] == target)[0])
            out.append(RankView(v.rank, v.gp, v.ranks, ls.astype(np.uint32), v.led))
        return out

    to2, to1 = to_rank(2), to_rank(1)
    mine = {t: [int(p) for p in range(len(views[t].gp)) if int(views[t].ranks[p][views[t].leader_slot[p]]) == 0]
            for t in (1, 2)}
    script = [("round", _round(spec, world, 0)),
              ("round", _round(spec, world, 1), {"lost": [(0, 2)]}),
              ("round", _round(spec, world, 2), {"lost": [(0, 2)]}),
              ("place", to2), ("lead", {2: [(p, 2) for p in mine[2]]}),
              # the placement named rank 2, its become_leader was refused: it serves nothing (a
              # placement never starts a leadership by itself)
              ("fetch", {2: (np.array(mine[2], np.uint32), np.zeros(len(mine[2]), np.uint32),
                             np.full(len(mine[2]), 10, np.uint32))}),
              ("place", to1), ("lead", {1: [(p, 2) for p in mine[1]]}),
              ("round", {r: led_batches(spec, to1[r], r, 2, 66) for r in range(world)}),
              ("round", {r: led_batches(spec, to1[r], r, 2, 67) for r in range(world)}),
              ("fetch", {1: (np.array(mine[1], np.uint32), np.zeros(len(mine[1]), np.uint32),
                             np.full(len(mine[1]), 10_000, np.uint32))})]
    return views, script, BASE


def fresh_replica_script(seg=1 << 16, world=4, rf=3, ppr=2):
    """Partition 0 of rank 0 has replicas on ranks {0, a, b}; rank f holds a local partition slot
    for it but no replica. After three rounds the placement moves replica slot 2 from rank b to
    rank f (PartitionManager.handleMembershipChange's reassignment): rank f's log is empty, its
    first round is refused (log mismatch) and the leader's catch-up fills it from offset 0, or —
    when the leader's ring no longer holds offset 0 (small seg) — rebases it (FORMAT.md §9)."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    g = 0
    row = views[0].ranks[0].copy()
    a, b = int(row[1]), int(row[2])
    f = next(r for r in range(world) if r not in (0, a, b))
    vf = views[f]
    views[f] = RankView(f, np.append(vf.gp, np.uint64(g)), np.vstack([vf.ranks, row[None, :]]).astype(np.uint32),
                        np.append(vf.leader_slot, np.uint32(0)).astype(np.uint32), vf.led)
    new_row = row.copy()
    new_row[2] = f
    new = []
    for v in views:
        rk = v.ranks.copy()
        for p in range(len(v.gp)):
            if int(v.gp[p]) == g:
                rk[p] = new_row
        new.append(RankView(v.rank, v.gp, rk, v.leader_slot, v.led))
    spec = StreamSpec(ppr, 40 if seg < (1 << 16) else 200, "uniform", size=(1, 100), config_index=93)
    script = [("round", _round(spec, world, k)) for k in range(3)]
    script += [("place", new)] + [("round", _round(spec, world, k)) for k in range(3, 7)]
    return views, script, dict(BASE, segment_bytes=seg), (f, g)


def unknown_term_vote_script(world=4, rf=3, ppr=2):
    """A follower filled by a PARTIAL catch-up that ends below the leader's term start does not
    know the term of its last entry (the round word carries 0); it must keep an upper bound of it
    (the term before the leader's), never 0, or it would grant a candidate of an older last term
    with a shorter log (Raft's election restriction). Partition 0 (rank 0) runs five
    term-1 rounds, rank 0 starts term 2, replica slot 2 moves to the empty rank f; the catch-up
    reserve (one round bound: small batches here) covers only a prefix of f's gap, below term 2's
    start. Then f answers RequestVotes of term 3 from a candidate whose last log term is 1: one log
    shorter than f's (refused), one as long (granted, term 4)."""
    views, script, base, (f, g) = fresh_replica_script(1 << 16, world, rf, ppr)
    base = dict(base, max_batch_records=64, max_batch_bytes=8192)
    spec = StreamSpec(ppr, 60, "uniform", size=(50, 100), config_index=95)
    new = script[3][1]
    lead = [("lead", {0: [(0, 2)]})]
    script = [("round", _round(spec, world, k)) for k in range(5)] + lead + [("place", new)]
    script += [("round", _round(spec, world, 5)), ("state", [f]), ("round", _round(spec, world, 6)), ("state", [f])]
    script += [("vote", {f: [(g, 3, 1, 1, -1), (g, 4, 1, 1, 0)]}), ("state", [f])]
    return views, script, base, (f, g)


def _check_unknown_term_vote(script, out, f):
    ks = [k for k, s in enumerate(script) if s[0] == "state"]
    fp = len(out[ks[0]][f]) - 1  # rank f's slot of partition 0 (its last local partition)
    first, second = out[ks[0]][f][fp], out[ks[1]][f][fp]
    assert first["log_end_offset"] == 0  # refused: its log did not match
    # the partial catch-up: some records, below the term start, the last term unknown (reported 0)
    assert 0 < second["log_end_offset"] and second["last_log_term"] == 0, second
    votes = out[[k for k, s in enumerate(script) if s[0] == "vote"][0]][f]
    assert votes == [False, True], votes


def test_unknown_last_term_votes_strictly(oracle_mod):
    views, script, base, (f, g) = unknown_term_vote_script()
    cfgs, oras, out = _oracle_run(oracle_mod, views, script, base)
    try:
        _check_unknown_term_vote(script, out, f)
    finally:
        _close(oras)


def offset_ticket_script(world=3, rf=3, ppr=4):
    """Consumer-offset completion (ConsumerOffsetUpdateRequestProcessor.java:40-49,60: the reply comes
    from the Raft closure, after the commit). Rank 0 commits offsets (ticket T1): pending until a
    round carries the row to a quorum — its first round is lost (rmq_fault_drop_rounds), so T1 stays
    pending until the catch-up round; then T2 is committed and leadership moves before any round
    carries it: T2 fails (RMQ_ENOTLEADER) and the new leaders hold T1's offsets, the acknowledged ones."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    spec = StreamSpec(ppr, 200, "uniform", size=(1, 60), config_index=94)
    new = moved_leadership(views)
    moved = {}
    for r in range(world):
        v = new[r]
        m = [int(p) for p in range(len(v.gp))
             if v.ranks[p][v.leader_slot[p]] == r and views[r].ranks[p][views[r].leader_slot[p]] != r]
        if m:
            moved[r] = m
    c1 = (np.arange(ppr, dtype=np.uint32), np.ones(ppr, np.uint32), np.arange(ppr, dtype=np.uint64) + 7)
    c2 = (np.arange(ppr, dtype=np.uint32), np.ones(ppr, np.uint32), np.arange(ppr, dtype=np.uint64) + 100)
    script = [("round", _round(spec, world, 0)),
              ("commit", {0: c1}), ("poll", {0: 1}),
              ("round", _round(spec, world, 1), {"drop": (0,)}), ("poll", {0: 1}),
              ("round", _round(spec, world, 2)), ("poll", {0: 1}),
              ("commit", {0: c2}), ("poll", {0: 7}),
              ("place", new), ("lead", {r: [(p, 2) for p in m] for r, m in moved.items()}),
              ("poll", {0: 7})]
    return views, script, BASE, c1


def election_script(world=3, rf=3, ppr=4):
    """Leader election (jraft's election timer and RequestVote,
    PartitionRaftServer.java:85,89; onLeaderStart, PartitionStateMachine.java:121-126). Rank 0's links
    to both followers are cut for two rounds (regions and commit notices lost, rmq_fault_cut): ranks 1
    and 2 report its partitions silent after two rounds, no others, and none after three. Rank 1 runs
    for leader of each of them in term 2: its own vote and rank 2's (2 of 3); rank 0, whose log holds
    the two uncommitted rounds, denies it and steps down on the newer term. Rank 2 then runs in the
    same term and gets no vote. A placement naming rank 2 is refused by become_leader (RMQ_ETERM: it
    voted for rank 1 in term 2); naming rank 1 succeeds once, a second call at term 2 is refused; the
    new leaders replicate and rank 0 truncates its uncommitted tail."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    spec = StreamSpec(ppr, 300, "uniform", size=(1, 60), config_index=95)

    def to_rank(target):
        out = []
        for v in views:
            ls = v.leader_slot.copy()
            for p in range(len(v.gp)):
                if int(v.ranks[p][v.leader_slot[p]]) == 0:
                    ls[p] = int(np.flatnonzero(v.ranks[p] == target)[0])
            out.append(RankView(v.rank, v.gp, v.ranks, ls.astype(np.uint32), v.led))
        return out

    to2, to1 = to_rank(2), to_rank(1)
    gids = list(range(ppr))  # rank 0's partitions
    mine = {t: [int(p) for p in range(len(views[t].gp)) if int(views[t].gp[p]) in gids] for t in (1, 2)}
    cut = {"cut": [(0, 1), (0, 2)]}
    script = [("round", _round(spec, world, 0)),
              ("round", _round(spec, world, 1), cut),
              ("round", _round(spec, world, 2), cut),
              ("silent", {1: 2, 2: 2}),
              ("silent", {1: 3, 2: 3}),
              ("elect", [(1, g, 2) for g in gids]),
              ("elect", [(2, g, 2) for g in gids]),
              ("place", to2), ("lead", {2: [(p, 2) for p in mine[2]]}),
              ("place", to1), ("lead", {1: [(p, 2) for p in mine[1]]}),
              ("lead", {1: [(p, 2) for p in mine[1]]}),
              ("round", {r: led_batches(spec, to1[r], r, 2, 68) for r in range(world)}),
              ("round", {r: led_batches(spec, to1[r], r, 2, 69) for r in range(world)}),
              ("fetch", {1: (np.array(mine[1], np.uint32), np.zeros(len(mine[1]), np.uint32),
                             np.full(len(mine[1]), 10_000, np.uint32))})]
    return views, script, BASE, mine


def divergent_notice_script(world=3, rf=3, ppr=4):
    """A commit notice may not commit a tail its log never matched in the notice's term (Raft: the
    follower's commit is min(leaderCommit, the last entry verified in the term)). Rank 0's round 1
    reaches nobody (its records stay in its log, uncommitted), leadership of its partitions moves to
    replica slot 1 at term 2, and the new leaders' first round to rank 0 is lost while the drain's
    commit notices reach it: rank 0 adopts term 2 and learns the new commit, but its own commit stays
    where it was; the next round truncates its tail and its commit follows the leader's."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    spec = StreamSpec(ppr, 300, "uniform", size=(1, 60), config_index=96)
    new = moved_leadership(views)
    moved = {}
    for r in range(world):
        v = new[r]
        m = [int(p) for p in range(len(v.gp))
             if v.ranks[p][v.leader_slot[p]] == r and views[r].ranks[p][views[r].leader_slot[p]] != r]
        if m:
            moved[r] = m
    script = [("round", _round(spec, world, 0)),
              ("state", [0]),
              ("round", _round(spec, world, 1), {"drop": (0,)}),
              ("place", new), ("lead", {r: [(p, 2) for p in m] for r, m in moved.items()}),
              ("round", {r: led_batches(spec, new[r], r, 2, 71) for r in range(world)},
               {"lost": [(r, 0) for r in moved]}),
              ("state", [0]),
              ("round", {r: led_batches(spec, new[r], r, 2, 72) for r in range(world)}),
              ("state", [0])]
    return views, script, BASE, ppr


def _check_divergent_notice(script, out, ppr):
    s0, s1, s2 = (out[_k(script, "state", i)][0] for i in range(3))
    for p in range(ppr):  # rank 0's former partitions (local pidx 0..ppr-1 on rank 0)
        assert s1[p]["term"] == 2 and s1[p]["leader_commit"] > s0[p]["commit"], (s0[p], s1[p])
        assert s1[p]["commit"] == s0[p]["commit"], (s0[p], s1[p])  # not over the unmatched tail
        assert s1[p]["log_end_offset"] > s1[p]["commit"]  # (the tail is there)
        assert s2[p]["commit"] > s0[p]["commit"] and s2[p]["last_log_term"] == 2, s2[p]


def _check_election(script, out, mine):
    """The election script's outcomes (oracle or GPU alike)."""
    s1, s3 = _k(script, "silent", 0), _k(script, "silent", 1)
    assert out[s1][1] == mine[1] and out[s1][2] == mine[2], out[s1]  # exactly rank 0's partitions
    assert out[s3][1] == [] and out[s3][2] == [], out[s3]
    e1, e2 = _k(script, "elect", 0), _k(script, "elect", 1)
    for g in range(len(mine[1])):  # rank 1: its own vote and rank 2's; rank 0 denies
        assert (g, 1, True) in out[e1][1] and (g, 1, True) in out[e1][2] and (g, 1, False) in out[e1][0]
    assert all(not granted for r in range(3) for (_, _, granted) in out[e2][r])  # one leader per term
    l2, l1, l1b = (out[_k(script, "lead", i)] for i in range(3))
    assert l2[2] and all(st == A.RMQ_ETERM for st in l2[2]), l2
    assert l1[1] and all(st == A.RMQ_OK for st in l1[1]), l1
    assert l1b[1] and all(st == A.RMQ_ETERM for st in l1b[1]), l1b
    rc, res, _ = out[_k(script, "fetch")][1]
    assert rc == 0 and np.all(res["status"] == 0) and np.all(res["count"] > 0)


def _cfgs(views, base):
    return [rank_cfg(EngineConfig(**base), views[r], r) for r in range(len(views))]


def _oracle_run(oracle_mod, views, script, base):
    cfgs = _cfgs(views, base)
    oras = [oracle_mod.OracleEngine(c) for c in cfgs]
    return cfgs, oras, run_oracle(oras, views, script)


def _close(oras):
    for o in oras:
        o.close()


def _k(script, kind, nth=0):
    return [k for k, s in enumerate(script) if s[0] == kind][nth]


# ---------------------------------------------------------------------------------------------
# CPU (oracle) behaviour


def test_new_leader_serves_committed_records(oracle_mod):
    views, script, base = new_leader_script()
    cfgs, oras, out = _oracle_run(oracle_mod, views, script, base)
    try:
        assert all(s == A.RMQ_OK for r in out[_k(script, "lead")] if r for s in r)
        before = out[_k(script, "fetch", 0)]
        for r, rec in enumerate(before):
            if rec is None:
                continue
            rc, res, _ = rec
            assert rc == 0 and np.all(res["status"] == 0)
            # every committed record from the consumer's offset on, before any round of the new term
            assert np.all(res["count"] > 0), res
            for i, p in enumerate(script[_k(script, "fetch", 0)][1][r][0]):
                g = int(views[r].gp[p])
                src, q = g // 4, g % 4  # its old leader (ppr 4) and local index there
                appended = sum(int((b.pidx == q).sum()) for k in (1, 2) for b in script[k][1][src])
                assert res["count"][i] == min(1000, appended - int(res["start_offset"][i]))
    finally:
        _close(oras)


def test_stale_replica_cannot_lead(oracle_mod):
    views, script, base = stale_replica_script()
    cfgs, oras, out = _oracle_run(oracle_mod, views, script, base)
    try:
        lead2, lead1 = out[_k(script, "lead", 0)][2], out[_k(script, "lead", 1)][1]
        assert lead2 and all(s == A.RMQ_ESTALE for s in lead2), lead2
        assert lead1 and all(s == A.RMQ_OK for s in lead1), lead1
        rc, res, _ = out[_k(script, "fetch", 0)][2]
        assert np.all(res["status"] == A.RMQ_ENOTLEADER), res  # the refused replica is no leader
        rc, res, _ = out[_k(script, "fetch", 1)][1]
        assert rc == 0 and np.all(res["status"] == 0) and np.all(res["count"] > 0)
    finally:
        _close(oras)


def test_leader_election(oracle_mod):
    views, script, base, mine = election_script()
    cfgs, oras, out = _oracle_run(oracle_mod, views, script, base)
    try:
        _check_election(script, out, mine)
        for r in range(3):  # rank 0 follows rank 1 in term 2 and holds the new leader's log
            for p in range(len(views[r].gp)):
                st = oras[r].state(p)
                if int(views[r].gp[p]) < 4:
                    assert st["term"] == 2 and st["is_leader"] == (r == 1), (r, p, st)
                    # ranks 1 and 2 voted for rank 1 in term 2; rank 0 denied it (its own vote of term 1)
                    assert (st["voted_term"], st["voted_for"]) == ((2, 1) if r else (1, 0)), (r, p, st)
        lead = [oras[1].state(p) for p in mine[1]]
        fol = [oras[0].state(p) for p in range(4)]
        assert [x["log_end_offset"] for x in lead] == [x["log_end_offset"] for x in fol]
    finally:
        _close(oras)


def test_notice_does_not_commit_an_unmatched_tail(oracle_mod):
    views, script, base, ppr = divergent_notice_script()
    cfgs, oras, out = _oracle_run(oracle_mod, views, script, base)
    try:
        _check_divergent_notice(script, out, ppr)
    finally:
        _close(oras)


@pytest.mark.parametrize("seg", [1 << 16, 1 << 13])
def test_replica_moved_to_a_fresh_rank(oracle_mod, seg):
    views, script, base, (f, g) = fresh_replica_script(seg)
    cfgs, oras, out = _oracle_run(oracle_mod, views, script, base)
    try:
        lead = oras[0].state(0)
        fp = len(views[f].gp) - 1
        fol = oras[f].state(fp)
        assert fol["log_end_offset"] == lead["log_end_offset"] and fol["log_end_pos"] == lead["log_end_pos"]
        assert min(lead["match"]) == lead["log_end_offset"] == lead["commit"]
        if seg < (1 << 16):
            assert lead["log_start_offset"] > 0 and fol["log_start_offset"] > 0  # rebased
        c = oras[0].counters()
        assert c[4] >= 1, c  # a catch-up entry filled it
    finally:
        _close(oras)


def test_offset_commit_waits_for_a_quorum(oracle_mod):
    views, script, base, c1 = offset_ticket_script()
    cfgs, oras, out = _oracle_run(oracle_mod, views, script, base)
    try:
        polls = [out[k][0] for k, s in enumerate(script) if s[0] == "poll"]
        assert polls == [A.RMQ_PENDING, A.RMQ_PENDING, A.RMQ_OK, A.RMQ_PENDING, A.RMQ_ENOTLEADER], polls
        for r in range(len(views)):  # the new leaders of rank 0's partitions hold T1's offsets
            for p in range(len(views[r].gp)):
                g = int(views[r].gp[p])
                if g < 4 and r != 0 and oras[r].state(p)["is_leader"]:
                    assert int(oras[r].consumer_offsets(p)[1]) == int(c1[2][g]), (r, p)
    finally:
        _close(oras)


# ---------------------------------------------------------------------------------------------
# GPU engines vs the oracle


def _gpu_vs_oracle(oracle_mod, views, script, base):
    from ripplemq_amd.engine import Engine, LocalHub

    cfgs = _cfgs(views, base)
    world = len(views)
    hub = LocalHub(world)
    engs = [Engine(c) for c in cfgs]
    oras = []
    try:
        got = run_gpu(engs, hub, views, script)
        oras = [oracle_mod.OracleEngine(c) for c in cfgs]
        want = run_oracle(oras, views, script)
        compare_outcomes(script, got, want)
        final = next((s[1] for s in reversed(script) if s[0] == "place"), views)
        for r in range(world):
            def local_slots(p, r=r):
                return [s for s in range(cfgs[r].replication_factor) if final[r].ranks[p][s] == r]
            compare_state(engs[r], oras[r], cfgs[r], local_slots=local_slots)
        return got, want
    finally:
        _close(oras)
        for e in engs:
            e.close()
        hub.close()


@pytest.mark.gpu
def test_new_leader_serves_committed_records_gpu(oracle_mod):
    views, script, base = new_leader_script()
    got, _ = _gpu_vs_oracle(oracle_mod, views, script, base)
    for rec in got[_k(script, "fetch", 0)]:
        if rec is not None:
            assert np.all(rec[1]["count"] > 0), rec[1]


@pytest.mark.gpu
def test_unknown_last_term_votes_strictly_gpu(oracle_mod):
    views, script, base, (f, g) = unknown_term_vote_script()
    got, _ = _gpu_vs_oracle(oracle_mod, views, script, base)
    _check_unknown_term_vote(script, got, f)


@pytest.mark.gpu
def test_stale_replica_cannot_lead_gpu(oracle_mod):
    views, script, base = stale_replica_script()
    got, _ = _gpu_vs_oracle(oracle_mod, views, script, base)
    assert all(s == A.RMQ_ESTALE for s in got[_k(script, "lead", 0)][2])


@pytest.mark.gpu
@pytest.mark.parametrize("seg", [1 << 16, 1 << 13])
def test_replica_moved_to_a_fresh_rank_gpu(oracle_mod, seg):
    views, script, base, _ = fresh_replica_script(seg)
    _gpu_vs_oracle(oracle_mod, views, script, base)


@pytest.mark.gpu
def test_offset_commit_waits_for_a_quorum_gpu(oracle_mod):
    views, script, base, _ = offset_ticket_script()
    got, _ = _gpu_vs_oracle(oracle_mod, views, script, base)
    polls = [got[k][0] for k, s in enumerate(script) if s[0] == "poll"]
    assert polls == [A.RMQ_PENDING, A.RMQ_PENDING, A.RMQ_OK, A.RMQ_PENDING, A.RMQ_ENOTLEADER], polls


@pytest.mark.gpu
def test_leader_election_gpu(oracle_mod):
    views, script, base, mine = election_script()
    got, _ = _gpu_vs_oracle(oracle_mod, views, script, base)
    _check_election(script, got, mine)


@pytest.mark.gpu
def test_notice_does_not_commit_an_unmatched_tail_gpu(oracle_mod):
    views, script, base, ppr = divergent_notice_script()
    got, _ = _gpu_vs_oracle(oracle_mod, views, script, base)
    _check_divergent_notice(script, got, ppr)
