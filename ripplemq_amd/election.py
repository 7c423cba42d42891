"""Partition-Raft leader election across ranks: the host loop around the engine's primitives.

The reference runs one jraft node per partition group and replica; the node's election timer
(1000 ms, ``mq-broker/src/main/java/metadata/raft/PartitionRaftServer.java:85``) starts an election
when the leader goes silent, RequestVote goes to the other replicas, votedFor is persisted in
raft_meta before the reply (``:89``), and the winner's state machine gets ``onLeaderStart``
(``PartitionStateMachine.java:121-126``), which ``PartitionManager.handlePartitionLeaderChange``
turns into the cluster's new leader map (``PartitionManager.java:248-275``).

The engine holds the per-partition parts of that: ``rmq_leader_silent`` (no
round entry or commit notice of the current term from the leader), ``rmq_vote`` (RequestVote: one
vote per term, the candidate's log at least as up to date), ``rmq_become_leader`` (one leader per
term, never a replica lacking committed records) and ``rmq_set_placement``. ``ElectionDriver`` is the
loop that uses them on every rank, in collective ticks (like ``RoundPacer``: every rank calls
``tick()`` at the same point, after a round):

1. each followed partition counts the ticks its leader has been silent; it becomes a candidate here
   after ``silent_rounds`` rounds of silence plus a per-(rank, partition, term) randomized delay of
   up to ``jitter_ticks`` ticks (jraft's randomized election timeout), so competing candidates of one
   partition rarely start in the same tick;
2. a candidate takes term = max(term, voted term) + 1 and votes for itself (persisted first);
3. RequestVotes go to every rank over the host channel (one all-gather), each replica answers the
   requests for partitions it holds (``rmq_vote``, the grant saved by the durable tier before it
   counts), answers come back by a second all-gather;
4. a candidate with a quorum (RF / 2 + 1 grants) wins; every rank applies the new leader slot to its
   placement (``rmq_set_placement``, collective), the winner starts its term
   (``rmq_become_leader``) and its ``on_leader_start(gid, term)`` hook runs: the place for
   ``PartitionManager.handlePartitionLeaderChange``.

Every rank sees the same requests and answers, so every rank computes the same winners; a voter
grants at most one candidate per term (persisted), so a term has at most one winner.
"""
from __future__ import annotations

import threading
import zlib
from dataclasses import dataclass

import numpy as np

from . import _abi as A
from .engine import EngineError
from .sharding import RankView


class GlooChannel:
    """Host channel over a torch.distributed process group (gloo): all-gather of small objects."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist, self.group = dist, group

    def allgather(self, obj):
        out = [None] * self.dist.get_world_size(self.group)
        self.dist.all_gather_object(out, obj, group=self.group)
        return out


class ThreadChannel:
    """The same between threads of one process (ranks on one GPU over the in-process transport)."""

    def __init__(self, world: int, timeout: float = 120.0):
        self.world = world
        self._bar = threading.Barrier(world, timeout=timeout)
        self._slots = [None] * world
        self._lock = threading.Lock()

    def endpoint(self, rank: int) -> "_ThreadEndpoint":
        return _ThreadEndpoint(self, rank)


class _ThreadEndpoint:
    def __init__(self, ch: ThreadChannel, rank: int):
        self.ch, self.rank = ch, rank

    def allgather(self, obj):
        ch = self.ch
        ch._bar.wait()
        ch._slots[self.rank] = obj
        ch._bar.wait()
        out = list(ch._slots)
        ch._bar.wait()
        return out


@dataclass
class Election:
    gid: int
    term: int
    leader: int     # the winning rank
    started: bool   # its rmq_become_leader succeeded


def _flat(xs):
    return [y for x in xs for y in x]


class ElectionDriver:
    """Leader election of the partitions one rank holds (see the module docstring).

    engine: the rank's engine (or the oracle's handle); view: its placement (RankView, updated as
    elections move leaders); channel: GlooChannel / ThreadChannel endpoint; tier: a DurableLog of
    the rank's partitions (votes are saved before they are answered) or None; on_leader_start:
    callback(gid, term) on the rank that starts a term."""

    def __init__(self, engine, view: RankView, channel, *, tier=None, on_leader_start=None,
                 silent_rounds: int = 2, jitter_ticks: int = 3, timeout_ms: int = 0, seed: int = 0):
        self.engine, self.view, self.ch, self.tier = engine, view, channel, tier
        self.on_leader_start = on_leader_start
        self.rank = int(view.rank)
        self.silent_rounds, self.jitter, self.timeout_ms, self.seed = silent_rounds, jitter_ticks, timeout_ms, seed
        self.rf = view.ranks.shape[1]
        self.quorum = self.rf // 2 + 1
        self._silent = np.zeros(len(view.gp), np.int64)  # consecutive ticks each partition was silent
        self.history: list[Election] = []

    def _local(self, gid: int):
        hit = np.flatnonzero(self.view.gp == gid)
        return int(hit[0]) if hit.size else None

    def _delay(self, gid: int, term: int) -> int:
        """The randomized part of the election timeout, in ticks (deterministic from the seed)."""
        if self.jitter <= 1:
            return 0
        h = zlib.crc32(np.array([self.seed, self.rank, gid, term], np.uint64).tobytes())
        return int(h % self.jitter)

    def _vote(self, p: int, term: int, cand: int, lterm: int, leo: int) -> bool:
        granted = bool(self.engine.vote(p, term, cand, lterm, leo))
        if granted and self.tier is not None:
            self.tier.save_vote(p, term, cand)  # raft_meta before the answer leaves this rank
        return granted

    def tick(self) -> list[Election]:
        """One collective election step (every rank, at the same point). Returns the elections
        decided in it, the same list on every rank."""
        eng, v = self.engine, self.view
        silent = np.zeros(len(v.gp), bool)
        silent[np.asarray(eng.leader_silent(self.silent_rounds, self.timeout_ms), np.int64)] = True
        self._silent = np.where(silent, self._silent + 1, 0)
        requests = []
        for p in np.flatnonzero(silent).tolist():
            gid = int(v.gp[p])
            st = eng.state(p)
            term = max(int(st["term"]), int(st["voted_term"])) + 1
            if self._silent[p] <= self._delay(gid, term):
                continue
            if self._vote(p, term, self.rank, int(st["last_log_term"]), int(st["log_end_offset"])):
                requests.append((gid, term, self.rank, int(st["last_log_term"]), int(st["log_end_offset"])))
        reqs = sorted(_flat(self.ch.allgather(requests)))
        answers = []
        for gid, term, cand, lt, leo in reqs:
            p = self._local(gid)
            if cand == self.rank or p is None:
                continue
            answers.append((gid, term, cand, self.rank, self._vote(p, term, cand, lt, leo)))
        ans = _flat(self.ch.allgather(answers))
        tally = {(g, t, c): 1 for g, t, c, _, _ in reqs}  # (the candidate's own vote)
        for g, t, c, _, ok in ans:
            if ok:
                tally[(g, t, c)] += 1
        winners: dict[int, tuple[int, int]] = {}
        for (g, t, c), k in sorted(tally.items()):
            if k >= self.quorum and (g not in winners or t > winners[g][0]):
                winners[g] = (t, c)
        if not winners:
            return []
        # every rank moves the winners' leader slots in its placement (collective), then each winner
        # starts its term
        ls = v.leader_slot.copy()
        for g, (t, c) in winners.items():
            p = self._local(g)
            if p is not None:
                ls[p] = int(np.flatnonzero(v.ranks[p] == c)[0])
        self.view = RankView(v.rank, v.gp, v.ranks, ls.astype(np.uint32), v.led)
        eng.set_placement(np.arange(len(v.gp), dtype=np.uint32), v.gp, v.ranks, self.view.leader_slot)
        mine = []
        for g, (t, c) in sorted(winners.items()):
            p = self._local(g)
            self._silent[p] = 0
            if c != self.rank:
                continue
            try:
                eng.become_leader(p, t)
                ok = True
            except EngineError as ex:  # RMQ_ESTALE / RMQ_ETERM: the next election goes on from here
                if ex.status not in (A.RMQ_ESTALE, A.RMQ_ETERM):
                    raise
                ok = False
            mine.append((g, ok))
            if ok and self.on_leader_start is not None:
                self.on_leader_start(g, t)
        started = dict(_flat(self.ch.allgather(mine)))
        out = [Election(g, t, c, bool(started.get(g, False))) for g, (t, c) in sorted(winners.items())]
        self.history += out
        return out
