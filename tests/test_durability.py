"""Durability on every replica (Weak #7, Missing #4).

jraft keeps the whole log and its raft_meta (currentTerm, votedFor) on every node of a partition
group (mq-broker/src/main/java/metadata/raft/PartitionRaftServer.java:53,85,88-90), and a restarted
node replays it (PartitionStateMachine.java:26). Two consequences checked here, on per-rank oracles
(CPU) and on GPU engines over the in-process transport (bit for bit against the oracles):

* a follower's durable tier spills its OWN replica (RMQ_FETCH_REPLICA reads up to its commit), so
  after leadership moves to it, a consumer below the new leader's rings is served from the new
  leader's files, equal to the reference state machine's message list (tests/refmodel.py);
* a vote is durable before it is answered (DurableLog.save_vote): a replica that voted in term 3 and
  restarts from its files refuses a second candidate in term 3 and grants the same one again.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from refmodel import Broker
from repl_sim import moved_leadership, rank_cfg
from ripplemq_amd import _abi as A
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import rank_view
from ripplemq_amd.tier import DurableLog, replay, split_records
from ripplemq_amd.workload import StreamSpec, make_batch
from world_script import compare_outcomes, run_gpu, run_oracle

BASE = dict(num_partitions=1, replication_factor=3, segment_bytes=1 << 14, index_interval=256,
            max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=2, max_consumers=4)
CURSOR = 3  # the tiers' position-cache key (no consumer slot is used)


def _round(spec, world, k, group=2):
    return {r: [make_batch(spec, 1000 * r + 50 * k + j) for j in range(group)] for r in range(world)}


def durable_script(world=3, rf=3, ppr=2, rounds=5):
    """Rounds on every rank, each followed by a spill of every rank's tier; then rank 0's partitions
    move to replica slot 1 (term 2). The new leaders' rings no longer hold offset 0 (RMQ_EOFFSET);
    every replica's files do. Then term-3 elections for rank 0's first partition g0: the new leader
    runs first (its own vote and the third replica's: both saved before they count), then the old
    leader runs in the same term and gets no vote."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    spec = StreamSpec(ppr, 200, "uniform", size=(1, 60), config_index=97)
    new = moved_leadership(views)
    moved = {}
    for r in range(world):
        v = new[r]
        m = [int(p) for p in range(len(v.gp))
             if v.ranks[p][v.leader_slot[p]] == r and views[r].ranks[p][views[r].leader_slot[p]] != r]
        if m:
            moved[r] = m
    g0 = 0
    row = [int(x) for x in views[0].ranks[0]]
    r1 = row[1]                                    # the new leader of g0 (replica slot 1)
    rv = next(x for x in row if x not in (0, r1))  # the third replica: the voter that restarts
    script = []
    for k in range(rounds):
        script += [("round", _round(spec, world, k)), ("spill", list(range(world)))]
    script += [("place", new), ("lead", {r: [(p, 2) for p in m] for r, m in moved.items()}),
               ("fetch", {r: (np.array(m, np.uint32), np.zeros(len(m), np.uint32), np.full(len(m), 100000, np.uint32))
                          for r, m in moved.items()}),
               ("tier_read", {r: (g0, 0, 100000) for r in row}),
               ("elect", [(r1, g0, 3)]),
               ("elect", [(0, g0, 3)])]
    return views, script, dict(g0=g0, r1=r1, rv=rv, row=row, spec=spec, rounds=rounds, ppr=ppr)


def _reference_messages(info, world=3):
    """The reference state machine's message list of g0 (messages.addAll in apply order): rank 0's
    records of its local partition 0, round by round (tests/refmodel.py)."""
    ref = Broker("t", 1)
    for k in range(info["rounds"]):
        for b in _round(info["spec"], world, k)[0]:
            pos = np.concatenate([[0], np.cumsum(b.lens.astype(np.int64))])
            for i in np.flatnonzero(b.pidx == 0):
                ref.produce(0, bytes(b.payload[pos[i]:pos[i + 1]]))
    return ref.sms[0].messages


def _tiers(engs, views, root):
    return [DurableLog(engs[r], os.path.join(root, f"rank{r}"), range(len(views[r].gp)), CURSOR)
            for r in range(len(engs))]


def _check(script, out, info, root, views, make_engine):
    """The outcomes both runs must show (oracle or GPU alike), and the restarted voter."""
    g0, r1, rv = info["g0"], info["r1"], info["rv"]
    fk = next(k for k, s in enumerate(script) if s[0] == "fetch")
    rc, res, _ = out[fk][r1]
    assert rc == 0 and np.all(res["status"] == A.RMQ_EOFFSET), res  # below the new leader's rings
    want = _reference_messages(info)
    tk = next(k for k, s in enumerate(script) if s[0] == "tier_read")
    for r in info["row"]:  # every replica persisted the committed prefix it held, bytes equal
        n, img = out[tk][r]
        got = [m for _, _, m in split_records(img)]
        assert n > len(want) // 2 and got == want[:n], (r, n, len(want))
    # the new leader serves from offset 0 through its own files (the broker's fallback on RMQ_EOFFSET)
    assert out[tk][r1][0] >= int(res["start_offset"][0])
    e1, e2 = (k for k, s in enumerate(script) if s[0] == "elect")
    assert (g0, r1, True) in out[e1][r1] and (g0, r1, True) in out[e1][rv], out[e1]
    assert all(not g for r in range(3) for (_, _, g) in out[e2][r]), out[e2]
    # the vote was on disk when it was answered (no spill since)
    p = int(np.flatnonzero(views[rv].gp == g0)[0])
    meta = json.load(open(os.path.join(root, f"rank{rv}", f"p{p:06d}", "meta.json")))
    assert (meta["term"], meta["voted_term"], meta["voted_for"], meta["led"]) == (3, 3, r1, 0), meta
    # the voter restarts: a fresh engine rebuilt from its files alone refuses rank 0 in term 3 and
    # grants r1 again (Raft: one vote per term, kept across restarts)
    big = EngineConfig(**dict(BASE, segment_bytes=1 << 20))
    with make_engine(rank_cfg(big, views[rv], rv)) as fresh:
        replay(os.path.join(root, f"rank{rv}"), fresh, range(len(views[rv].gp)), batch_records=500)
        st = fresh.state(p)
        assert (st["voted_term"], st["voted_for"], st["term"]) == (3, r1, 3), st
        assert not fresh.vote(p, 3, 0, 99, 1 << 40)
        assert fresh.vote(p, 3, r1, 2, st["log_end_offset"])


def test_follower_tier_and_durable_votes(oracle_mod, tmp_path):
    views, script, info = durable_script()
    cfgs = [rank_cfg(EngineConfig(**BASE), views[r], r) for r in range(3)]
    oras = [oracle_mod.OracleEngine(c) for c in cfgs]
    try:
        tiers = _tiers(oras, views, str(tmp_path))
        out = run_oracle(oras, views, script, tiers=tiers)
        _check(script, out, info, str(tmp_path), views, oracle_mod.OracleEngine)
    finally:
        for o in oras:
            o.close()


@pytest.mark.gpu
def test_follower_tier_and_durable_votes_gpu(oracle_mod, tmp_path):
    from ripplemq_amd.engine import Engine, LocalHub

    views, script, info = durable_script()
    cfgs = [rank_cfg(EngineConfig(**BASE), views[r], r) for r in range(3)]
    hub = LocalHub(3)
    engs = [Engine(c) for c in cfgs]
    oras = []
    try:
        tiers = _tiers(engs, views, str(tmp_path / "gpu"))
        got = run_gpu(engs, hub, views, script, tiers=tiers)
        oras = [oracle_mod.OracleEngine(c) for c in cfgs]
        want = run_oracle(oras, views, script, tiers=_tiers(oras, views, str(tmp_path / "cpu")))
        compare_outcomes(script, got, want)
        _check(script, got, info, str(tmp_path / "gpu"), views, Engine)
    finally:
        for o in oras:
            o.close()
        for e in engs:
            e.close()
        hub.close()
