"""Replica-log rounds (FORMAT.md §9) simulated over per-rank oracle engines — test infrastructure.

Each rank has its own OracleEngine holding the partitions it hosts (ripplemq_amd.sharding.rank_view:
leader slot 0, followers spread over the peers). A round = the batches the GPU engine groups into
one launch group (cfg.pipeline_depth): every rank appends its batches, then every leader's region
for every follower is ingested there and the follower's acks go back to the leader.
"""
from __future__ import annotations

import numpy as np

from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import rank_view
from ripplemq_amd.workload import StreamSpec, make_batch


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


def exchange_round(oras, keep_regions: bool = False, corrupt=None, skip=None):
    """Regions of every leader to every follower, ingested there; acks back to the leaders.
    corrupt=(src, dst, byte): flip one byte of that region; skip=(src, dst): drop that region and
    its acks (the follower misses the round)."""
    W = len(oras)
    regions = [[oras[s].round_region(d) if d != s else None for d in range(W)] for s in range(W)]
    for o in oras:
        o.end_round()
    for s in range(W):
        for d in range(W):
            if d == s or regions[s][d].size == 0 or (skip and (s, d) == tuple(skip)):
                continue
            reg = regions[s][d]
            if corrupt and (s, d) == tuple(corrupt[:2]):
                reg = reg.copy()
                reg[corrupt[2]] ^= 0x5A
            acks = oras[d].ingest(s, reg)
            oras[s].apply_acks(d, acks)
    return regions if keep_regions else None
