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
        rc, res, _ = out[_k(script, "fetch")][1]
        assert rc == 0 and np.all(res["status"] == 0) and np.all(res["count"] > 0)
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
