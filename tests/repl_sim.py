"""Replica-log rounds (FORMAT.md §9) simulated over per-rank oracle engines — test infrastructure.

Each rank has its own OracleEngine holding the partitions it hosts (ripplemq_amd.sharding.rank_view:
leader slot 0, followers spread over the peers). A round = the batches the GPU engine groups into
one launch group (cfg.pipeline_depth): every rank appends its batches, then every leader's region
for every follower is ingested there and the follower's acks go back to the leader.
"""
from __future__ import annotations

import numpy as np

from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import RankView, rank_view
from ripplemq_amd.workload import Batch, StreamSpec, make_batch


def rank_cfg(base: EngineConfig, view, rank: int) -> EngineConfig:
    d = dict(base.__dict__)
    d.update(num_partitions=len(view.gp), rank=rank)
    return EngineConfig(**d)


def place(eng, view, world: int | None = None):
    if world is not None and hasattr(eng, "set_world"):
        eng.set_world(world)
    n = len(view.gp)
    eng.set_placement(np.arange(n, dtype=np.uint32), view.gp, view.ranks, view.leader_slot)


def rank_batches(spec: StreamSpec, rank: int, rounds: int, group: int):
    """Batches of one rank: a stream over its led partitions (local pidx [0, led)), salted by rank."""
    return [make_batch(spec, 1000 * rank + k) for k in range(rounds * group)]


def exchange_round(oras, keep_regions: bool = False, corrupt=None, skip=None, drop=(), lost=()):
    """Regions of every leader to every follower, ingested there; acks back to the leaders (FORMAT.md
    §9 v3: a refused ack leaves a catch-up request for the next round's plan).
    corrupt=(src, dst, byte): flip one byte of that region (byte < 0: from the end of its data
    section, i.e. a payload byte of its last record); skip=(src, dst): drop that region and its
    acks; drop: leaders whose round sends no region (rmq_fault_drop_rounds: their followers miss
    the round and refuse every entry of it); lost: (src, dst) pairs whose region is lost on the way
    (rmq_fault_isolate: dst misses src's round)."""
    W = len(oras)
    rnd = [o.round_no() for o in oras]
    regions = [[oras[s].round_region(d) if d != s else None for d in range(W)] for s in range(W)]
    for s in drop:
        regions[s] = [None if d == s else np.zeros(0, np.uint8) for d in range(W)]
    for s, d in lost:
        regions[s][d] = np.zeros(0, np.uint8)
    for o in oras:
        o.end_round()
    for s in range(W):
        for d in range(W):
            if d == s or (skip and (s, d) == tuple(skip)):
                continue
            if regions[s][d].size == 0 and s not in drop and (s, d) not in lost:
                continue
            reg = regions[s][d]
            if corrupt and (s, d) == tuple(corrupt[:2]):
                reg = reg.copy()
                at = corrupt[2]
                if at < 0:
                    at += int(reg[32:40].view(np.uint64)[0])  # rows_off: end of the data section
                reg[at] ^= 0x5A
            acks = oras[d].ingest(s, reg)
            oras[s].apply_acks(d, acks, rnd[s])
    return regions if keep_regions else None


DIR = 48  # directory entry bytes of a round region (FORMAT.md §9 v4)


def mask_commit(region: np.ndarray) -> np.ndarray:
    """A region with the leader-commit word of every directory entry zeroed (FORMAT.md §9 v4). A
    pipelined GPU run plans a round before the acks of the rounds just before it are in (it carries
    the commit its launch started with), the oracle after them: the word is compared in the synced
    runs, and masked in the pipelined ones."""
    if region is None or region.size < 64:
        return region
    r = region.copy()
    n = int(r[4:8].view(np.uint32)[0])
    for k in range(n):
        r[64 + DIR * k + 32:64 + DIR * k + 40] = 0
    return r


def notice_round(oras, lost=()):
    """The commit notices of a drain (FORMAT.md §9 v4): every leader's {commit, term} per entry to
    each follower, which learns its leader's commit. The GPU engines exchange them at every drain
    that had rounds in flight (rmq_sync, and the drain of a placement change). lost: (src, dst)
    pairs whose notices are lost (rmq_fault_cut)."""
    W = len(oras)
    notes = [[oras[s].commit_notice(d) if d != s else None for d in range(W)] for s in range(W)]
    for s in range(W):
        for d in range(W):
            if d != s and len(notes[s][d]) and (s, d) not in set(map(tuple, lost)):
                oras[d].apply_notice(s, notes[s][d])


def moved_leadership(views, old_leader: int = 0, new_slot: int = 1):
    """Placement after a leader change: every partition `old_leader` leads moves its leadership to
    replica slot `new_slot` (a follower that holds the same committed log)."""
    out = []
    for v in views:
        ls = v.leader_slot.copy()
        moved = v.ranks[np.arange(len(v.gp)), ls] == old_leader
        ls[moved] = new_slot
        out.append(RankView(v.rank, v.gp, v.ranks, ls.astype(np.uint32), v.led))
    return out


def led_batches(spec: StreamSpec, view, rank: int, count: int, salt: int):
    """Batches over the partitions `view` names this rank the leader of (all local pidx if none:
    every record is then rejected as not leader)."""
    mine = np.flatnonzero(view.ranks[np.arange(len(view.gp)), view.leader_slot] == rank).astype(np.uint32)
    out = []
    for k in range(count):
        b = make_batch(StreamSpec(max(len(mine), 1), spec.records, spec.mode, size=spec.size,
                                  config_index=spec.config_index), salt + 1000 * rank + k)
        pidx = mine[b.pidx] if len(mine) else b.pidx
        out.append(Batch(pidx.astype(np.uint32), b.lens, b.payload))
    return out


def leader_change_script(spec: StreamSpec, world: int, rf: int, ppr: int, group: int):
    """Raft's follower-truncation case: rank 0 leads, two rounds reach every follower, the third
    round of rank 0 is lost (rank 0 keeps those records, uncommitted), leadership of rank 0's
    partitions moves to replica slot 1 at term 2 while batches are still in flight, and the new
    leaders append: rank 0, now a follower, must truncate its log to the new leaders' and accept.
    Returns (views, new views, phases): each phase is (batches per rank, drop set, placement or
    None, become_leader list per rank [(local pidx, term)])."""
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    new = moved_leadership(views)
    phases = []
    for k in range(2):
        phases.append(([[make_batch(spec, 1000 * r + k * group + j) for j in range(group)] for r in range(world)],
                       (), None, [[] for _ in range(world)]))
    phases.append(([[make_batch(spec, 1000 * r + 2 * group + j) for j in range(group)] for r in range(world)],
                   (0,), None, [[] for _ in range(world)]))
    bl = []
    for r in range(world):
        v = new[r]
        moved = np.flatnonzero((v.ranks[np.arange(len(v.gp)), v.leader_slot] == r) &
                               (views[r].ranks[np.arange(len(v.gp)), views[r].leader_slot] != r))
        bl.append([(int(p), 2) for p in moved])
    phases.append(([led_batches(spec, new[r], r, group, 77) for r in range(world)], (), new, bl))
    phases.append(([led_batches(spec, new[r], r, group, 99) for r in range(world)], (), None, [[] for _ in range(world)]))
    return views, new, phases


def run_script_oracle(oras, views, phases, world):
    """The script on per-rank oracles: a phase's batches form one round (one launch group)."""
    regions = None
    for batches, drop, placement, bl in phases:
        if placement is not None:
            for r in range(world):
                place(oras[r], placement[r])
            for r in range(world):
                for p, t in bl[r]:
                    oras[r].become_leader(p, t)
        for r in range(world):
            for b in batches[r]:
                oras[r].append(b.pidx, b.lens, b.payload)
        regions = exchange_round(oras, keep_regions=True, drop=drop)
        notice_round(oras)  # every phase ends in a drain (rmq_sync, or the next placement's)
    return regions
