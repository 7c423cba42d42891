"""A world of ranks running ripplemq_amd.election.ElectionDriver between replica-log rounds — test
infrastructure for tests/test_election.py.

Scenario (every rank, in order, per round k): append this rank's batches for the partitions its
current placement says it leads; one replication round (regions, ingest, acks, then the drain's
commit notices), where during rounds ISOLATED rank 0's regions and notices to the others are lost
(rmq_fault_cut: its followers stop hearing from it, its records there stay uncommitted); then one
collective election tick. Rank 0's followers detect the silence, elect one of themselves, every rank
moves the leader slot, the winner starts its term; from the next round on the new leader appends
and replicates, and rank 0, heard again, steps down (the RequestVote of the newer term) and
truncates its uncommitted tail.

Two drivers of the same scenario: per-rank oracles in threads (the round exchange done by one thread
between barriers, tests/repl_sim.py) and GPU engines in threads over the in-process transport.
"""
from __future__ import annotations

import threading

import numpy as np

from repl_sim import exchange_round, led_batches, notice_round, place
from ripplemq_amd.election import ElectionDriver, ThreadChannel
from ripplemq_amd.workload import StreamSpec

WORLD, RF, PPR = 3, 3, 2
ROUNDS = 12
ISOLATED = range(2, 6)
SPEC = StreamSpec(PPR, 200, "uniform", size=(1, 60), config_index=98)


def _salt(k: int) -> int:
    return 7000 + 97 * k


def _run_threads(world, body, timeout=240):
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


def run_oracle_world(oras, views, seed=5, rounds=ROUNDS):
    """Returns (per rank: the elections of each tick, the final placement view)."""
    world = len(oras)
    for r in range(world):
        place(oras[r], views[r], world)
    ch = ThreadChannel(world)
    bar = threading.Barrier(world, timeout=120)
    drivers = [ElectionDriver(oras[r], views[r], ch.endpoint(r), seed=seed) for r in range(world)]
    log = [[None] * rounds for _ in range(world)]

    def body(r):
        d = drivers[r]
        for k in range(rounds):
            for b in led_batches(SPEC, d.view, r, 2, _salt(k) + 1000 * r):
                oras[r].append(b.pidx, b.lens, b.payload)
            bar.wait()
            if r == 0:  # the round, for every rank at once (regions, ingest, acks; the notices)
                cut = [(0, 1), (0, 2)] if k in ISOLATED else []
                exchange_round(oras, lost=cut)
                notice_round(oras, lost=cut)
            bar.wait()
            log[r][k] = [(e.gid, e.term, e.leader, e.started) for e in d.tick()]

    _run_threads(world, body)
    return log, [d.view for d in drivers]


def run_gpu_world(engs, hub, views, seed=5, rounds=ROUNDS):
    world = len(engs)
    ch = ThreadChannel(world)
    log = [[None] * rounds for _ in range(world)]
    final = [None] * world

    def body(r):
        e = engs[r]
        e.attach_local(hub)
        place(e, views[r])
        d = ElectionDriver(e, views[r], ch.endpoint(r), seed=seed)
        for k in range(rounds):
            if r == 0 and k in ISOLATED:
                for dst in (1, 2):
                    e.fault_cut(dst, 1)
            bs = led_batches(SPEC, d.view, r, 2, _salt(k) + 1000 * r)
            for b in bs:
                e.append_async(b.pidx, b.lens, b.payload)
            if not bs:
                e.append_async(np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
            e.sync()
            log[r][k] = [(x.gid, x.term, x.leader, x.started) for x in d.tick()]
        final[r] = d.view

    _run_threads(world, body)
    return log, final


def check_world(log, final, engines):
    """Exactly one leader per (partition, term); every rank saw the same elections; rank 0's
    partitions have new leaders of newer terms, which hold the committed records and commit new ones;
    every replica of them ends with the same log."""
    world = len(log)
    for k in range(len(log[0])):
        assert all(log[r][k] == log[0][k] for r in range(world)), (k, [log[r][k] for r in range(world)])
    els = [x for tick in log[0] for x in tick]
    terms = {}
    for gid, term, leader, started in els:
        assert (gid, term) not in terms, f"two leaders of partition {gid} in term {term}"
        terms[(gid, term)] = leader
    # rank 0's partitions, each with a started leader of a newer term (one of the followers, or rank
    # 0 itself in a later term once a split vote made it step down: its log is the most complete)
    moved = {gid: (term, leader) for gid, term, leader, started in els if started}
    assert set(moved) == set(range(PPR)), els
    assert all(term >= 2 for term, _ in moved.values()), moved
    for gid, (term, leader) in moved.items():
        sts = []
        for r in range(world):
            hit = np.flatnonzero(final[r].gp == gid)
            if not hit.size:
                continue
            p = int(hit[0])
            assert int(final[r].ranks[p][final[r].leader_slot[p]]) == leader
            sts.append(engines[r].state(p))
        assert len(sts) == RF
        new = [s for s in sts if s["is_leader"]]
        assert len(new) == 1 and new[0]["term"] == term and new[0]["commit"] == new[0]["log_end_offset"] > 0, sts
        assert all(s["log_end_offset"] == new[0]["log_end_offset"] for s in sts), sts  # rank 0 truncated
    return moved
