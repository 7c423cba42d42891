"""Step scripts over a world of replica-log ranks — test infrastructure.

A script is a list of steps, each applied by every rank in order: on the GPU engines (one host
thread per rank, the in-process transport, as each rank would be driven by its own process over
RCCL) and on per-rank oracles (tests/repl_sim.py rounds). Steps:

  ("place", views)                  rmq_set_placement of every rank's view (collective)
  ("commit", {rank: (pidx, consumer, offset)})   leader consumer-offset commits (status and ticket)
  ("poll", {rank: k})               rmq_poll_commit of the offset ticket that step k's commit got
  ("round", {rank: [batches]}, faults)          the batches form ONE launch group on every rank,
        then rmq_sync (rounds, acks, commit notices); faults = {"drop": ranks, "lost": [(src, dst)],
        "cut": [(src, dst)] (the region and the drain's commit notices lost), "corrupt": (src, dst, at)}
  ("lead", {rank: [(pidx, term)]})  rmq_become_leader; the status of each call is recorded
  ("fetch", {rank: (pidx, consumer, max)})      rmq_fetch; results and bytes are recorded
  ("silent", {rank: silent_rounds}) rmq_leader_silent (rounds only); the partitions are recorded
  ("state", ranks)                  every partition state of those ranks is recorded
  ("elect", [(candidate, gid, term)])  Raft elections: the candidate's (last_log_term, log end) of
        global partition gid go as a vote request to every replica of gid in the current placement
        (the candidate first); every rank records its votes [(gid, candidate, granted)]; with durable
        tiers a granted vote is saved (DurableLog.save_vote) before it counts
  ("vote", {rank: [(gid, term, cand, last_log_term, dleo)]})  RequestVotes with explicit candidate
        logs (log end = the voter's own log end + dleo); the grants are recorded
  ("spill", ranks)                  DurableLog.spill of those ranks' tiers (records moved)
  ("tier_read", {rank: (gid, off, max)})  records [off, off + max) of gid from that rank's tier files

run_oracle / run_gpu return the recorded outcomes per step and rank, so a test compares them and
then every rank's state, rings, index and consumer offsets.
"""
from __future__ import annotations

import threading

import numpy as np

from repl_sim import exchange_round, notice_round, place
from ripplemq_amd import _abi as A
from ripplemq_amd.engine import EngineError


def _lead(eng, p, t):
    try:
        eng.become_leader(int(p), int(t))
        return A.RMQ_OK
    except EngineError as ex:
        return ex.status


def _local(view, gid):
    hit = np.flatnonzero(view.gp == gid)
    return int(hit[0]) if hit.size else None


def _voters(view, gid, cand):
    """Replica ranks of global partition gid (the candidate first) in a rank's view of the placement."""
    p = _local(view, gid)
    ranks = [int(x) for x in view.ranks[p]]
    return [cand] + [r for r in ranks if r != cand]


def _vote(eng, tier, p, term, cand, lt, leo):
    g = bool(eng.vote(p, term, cand, lt, leo))
    if g and tier is not None:
        tier.save_vote(p, term, cand)  # durable before the grant is answered (raft_meta votedFor)
    return g


def _vote_rel(eng, tier, p, term, cand, lt, dleo):
    """A RequestVote whose candidate log ends dleo records from the voter's own log end."""
    return _vote(eng, tier, p, term, cand, lt, int(eng.state(p)["log_end_offset"]) + int(dleo))


def run_oracle(oras, views0, script, tiers=None):
    world = len(oras)
    tiers = tiers or [None] * world
    for r in range(world):
        place(oras[r], views0[r], world)
    views = list(views0)
    out = []
    for step in script:
        kind = step[0]
        rec = [None] * world
        if kind == "place":
            views = list(step[1])
            for r in range(world):
                place(oras[r], step[1][r])
        elif kind == "commit":
            for r, args in step[1].items():
                rc, st = oras[r].commit_consumer_offset(*args)
                rec[r] = (rc, st, oras[r].last_offset_ticket)
        elif kind == "poll":
            for r, k in step[1].items():
                rec[r] = oras[r].poll_offsets(out[k][r][2])
        elif kind == "round":
            f = step[2] if len(step) > 2 else {}
            for r in range(world):
                for b in step[1].get(r, []):
                    oras[r].append(b.pidx, b.lens, b.payload)
            cut = list(f.get("cut", ()))
            rec = exchange_round(oras, keep_regions=True, drop=f.get("drop", ()),
                                 lost=list(f.get("lost", ())) + cut, corrupt=f.get("corrupt"))
            notice_round(oras, lost=cut)
        elif kind == "lead":
            for r, items in step[1].items():
                rec[r] = [_lead(oras[r], p, t) for p, t in items]
        elif kind == "fetch":
            for r, (pidx, cons, mx) in step[1].items():
                rc, res, buf, used = oras[r].fetch(pidx, cons, mx)
                rec[r] = (rc, res, buf[:used])
        elif kind == "silent":
            for r, k in step[1].items():
                rec[r] = [int(x) for x in oras[r].leader_silent(k)]
        elif kind == "state":
            for r in step[1]:
                rec[r] = [oras[r].state(p) for p in range(len(views[r].gp))]
        elif kind == "elect":
            rec = [[] for _ in range(world)]
            for cand, gid, term in step[1]:
                st = oras[cand].state(_local(views[cand], gid))
                for v in _voters(views[cand], gid, cand):
                    g = _vote(oras[v], tiers[v], _local(views[v], gid), term, cand, st["last_log_term"],
                              st["log_end_offset"])
                    rec[v].append((gid, cand, g))
        elif kind == "vote":
            for r, items in step[1].items():
                rec[r] = [_vote_rel(oras[r], tiers[r], _local(views[r], gid), term, cand, lt, dleo)
                          for gid, term, cand, lt, dleo in items]
        elif kind == "spill":
            for r in step[1]:
                rec[r] = tiers[r].spill()
        elif kind == "tier_read":
            for r, (gid, off, mx) in step[1].items():
                rec[r] = tiers[r].read_images(_local(views[r], gid), off, mx)
        else:
            raise ValueError(kind)
        out.append(rec)
    return out


def run_gpu(engs, hub, views0, script, timeout=240, tiers=None):
    world = len(engs)
    tiers = tiers or [None] * world
    out = [[None] * world for _ in script]
    errs = [None] * world
    bar = threading.Barrier(world, timeout=timeout)
    shared = {}

    def body(r):
        try:
            e = engs[r]
            e.attach_local(hub)
            place(e, views0[r])
            views = list(views0)
            for k, step in enumerate(script):
                kind = step[0]
                if kind == "place":
                    views = list(step[1])
                    place(e, step[1][r])
                elif kind == "commit":
                    if r in step[1]:
                        rc, st = e.commit_consumer_offset(*step[1][r])
                        out[k][r] = (rc, st, e.last_offset_ticket)
                elif kind == "poll":
                    if r in step[1]:
                        out[k][r] = e.poll_offsets(out[step[1][r]][r][2])
                elif kind == "round":
                    f = step[2] if len(step) > 2 else {}
                    if r in f.get("drop", ()):
                        e.fault_drop_rounds(1)
                    for s, d in f.get("lost", ()):
                        if s == r:
                            e.fault_isolate(d, 1)
                    for s, d in f.get("cut", ()):
                        if s == r:
                            e.fault_cut(d, 1)
                    if f.get("corrupt") and f["corrupt"][0] == r:
                        e.fault_corrupt(f["corrupt"][1], f["corrupt"][2])
                    for b in step[1].get(r, []):
                        e.append_async(b.pidx, b.lens, b.payload)
                    if not step[1].get(r):  # rounds are collective: an idle rank submits an empty batch
                        e.append_async(np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
                    e.sync()
                    out[k][r] = [e.read_outbox(d) if d != r else None for d in range(world)]
                elif kind == "lead":
                    if r in step[1]:
                        out[k][r] = [_lead(e, p, t) for p, t in step[1][r]]
                elif kind == "fetch":
                    if r in step[1]:
                        rc, res, buf, used = e.fetch(*step[1][r])
                        out[k][r] = (rc, res, buf[:used])
                elif kind == "silent":
                    if r in step[1]:
                        out[k][r] = [int(x) for x in e.leader_silent(step[1][r])]
                elif kind == "state":
                    if r in step[1]:
                        out[k][r] = [e.state(p) for p in range(len(views[r].gp))]
                elif kind == "elect":
                    # one election after another, as the oracle runs them: the candidate publishes its
                    # log's (last term, end), then each replica votes in order
                    out[k][r] = []
                    for cand, gid, term in step[1]:
                        bar.wait()
                        if r == cand:
                            st = e.state(_local(views[r], gid))
                            shared[(k, gid, cand)] = (st["last_log_term"], st["log_end_offset"])
                        bar.wait()
                        lt, leo = shared[(k, gid, cand)]
                        for v in _voters(views[cand], gid, cand):
                            if v == r:
                                g = _vote(e, tiers[r], _local(views[r], gid), term, cand, lt, leo)
                                out[k][r].append((gid, cand, g))
                            bar.wait()
                elif kind == "vote":
                    if r in step[1]:
                        out[k][r] = [_vote_rel(e, tiers[r], _local(views[r], gid), term, cand, lt, dleo)
                                     for gid, term, cand, lt, dleo in step[1][r]]
                elif kind == "spill":
                    if r in step[1]:
                        out[k][r] = tiers[r].spill()
                elif kind == "tier_read":
                    if r in step[1]:
                        gid, off, mx = step[1][r]
                        out[k][r] = tiers[r].read_images(_local(views[r], gid), off, mx)
        except BaseException as ex:  # noqa: BLE001 - reported below
            errs[r] = ex
            bar.abort()

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
        assert not t.is_alive(), "a rank hung"
    for r, ex in enumerate(errs):
        if ex is not None:
            raise AssertionError(f"rank {r}: {ex!r}") from ex
    return out


def rounds_of(script) -> list[int]:
    """Indices of the round steps (the GPU side pads idle ranks with an empty batch: for the
    oracle, a round with no batches on a rank is the same round)."""
    return [k for k, s in enumerate(script) if s[0] == "round"]


def compare_outcomes(script, got, want):
    """The recorded outcomes of every step: become_leader statuses, fetch results and bytes, the
    region every leader sent every follower in each round, consumer-commit statuses."""
    for k, step in enumerate(script):
        for r in range(len(want[k])):
            g, w = got[k][r], want[k][r]
            if step[0] == "round":  # w: the regions rank r sent, by destination
                for d in range(len(want[k])):
                    if d != r and w[d] is not None and w[d].size:
                        assert np.array_equal(g[d], w[d]), f"step {k}: region {r}->{d}"
            elif step[0] == "lead" and w is not None:
                assert list(g) == list(w), (k, r, g, w)
            elif step[0] == "fetch" and w is not None:
                assert g[0] == w[0], (k, r, g[0], w[0])
                assert np.array_equal(g[1], w[1]), f"step {k} rank {r} fetch results\n gpu={g[1]}\n cpu={w[1]}"
                assert np.array_equal(g[2], w[2]), f"step {k} rank {r} fetched bytes"
            elif step[0] == "commit" and w is not None:
                assert g[0] == w[0] and np.array_equal(g[1], w[1]), (k, r, g, w)
            elif step[0] == "poll" and w is not None:
                assert g == w, (k, r, g, w)
            elif step[0] in ("silent", "elect", "vote", "state", "spill", "tier_read") and w is not None:
                assert g == w, (k, step[0], r, g, w)
