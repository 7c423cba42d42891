"""Round pacing for engines with a replication transport (host glue, no data-path compute).

With a transport attached, replication rounds are collective: every rank must submit the same
sequence of ``rmq_append`` calls (empty batches count), because each launch group of
``cfg.pipeline_depth`` batches is one round exchanged with every peer (FORMAT.md §9,
``include/ripplemq_engine.h``). The reference has no such coupling — every partition is its own
jraft group (``PartitionManager.java:111-176``) — so a broker built on the engine needs a policy
that keeps rounds flowing when its ranks see different traffic, and lets a lone produce request
commit without a collective ``rmq_sync``:

* every rank submits exactly ONE batch per tick of a shared clock (``epoch`` + k * ``tick_s``):
  the records queued since its previous tick, or an empty batch when it has none — so an idle
  rank still closes rounds, and a busy one never runs ahead of the others;
* a request's records commit once their round's acks are in: ``committed(pidx, offsets)`` reads the
  commit indices (``rmq_poll_commit`` without a flush) and answers per record, as the reference's
  ``PartitionClosure`` answers a ``MessageAppendRequest`` after the BallotBox commit
  (``MessageAppendRequestProcessor.java:39-48``).

Latency is about (pipeline stages + ack delay) x depth x tick: with depth 4 and 100 us ticks a
record commits within ~2 ms; throughput is one batch per tick per rank.
"""
from __future__ import annotations

import time

import numpy as np

from . import _abi as A
from .engine import EngineError


class RoundPacer:
    """One rank's tick loop over its engine (``Engine`` with a transport attached)."""

    def __init__(self, engine, epoch: float, tick_s: float, clock=time.monotonic):
        self.engine = engine
        self.epoch = float(epoch)
        self.tick_s = float(tick_s)
        self.clock = clock
        self.ticks = 0                      # batches submitted
        self._pidx: list[np.ndarray] = []
        self._lens: list[np.ndarray] = []
        self._pay: list[np.ndarray] = []
        self.tickets: list[tuple[int, np.ndarray, np.ndarray]] = []  # (ticket, pidx, out offsets)
        self.rejected: list[tuple[np.ndarray, np.ndarray, dict | None]] = []  # batches with rejected records

    def submit(self, pidx, lens, payload) -> None:
        """Queue records for the next tick (any partitions this rank leads)."""
        self._pidx.append(np.ascontiguousarray(pidx, np.uint32))
        self._lens.append(np.ascontiguousarray(lens, np.uint32))
        self._pay.append(np.ascontiguousarray(payload, np.uint8))

    def due(self) -> int:
        """Ticks of the shared clock that have passed and this rank has not submitted yet."""
        return max(0, int((self.clock() - self.epoch) // self.tick_s) - self.ticks)

    def tick(self) -> int:
        """Submit one batch: everything queued, or an empty batch. Returns its ticket."""
        if self._pidx:
            pidx = np.concatenate(self._pidx)
            lens = np.concatenate(self._lens)
            pay = np.concatenate(self._pay)
            self._pidx, self._lens, self._pay = [], [], []
        else:
            pidx = np.zeros(0, np.uint32)
            lens = np.zeros(0, np.uint32)
            pay = np.zeros(0, np.uint8)
        t, out = self.engine.append_async(pidx, lens, pay)
        self.ticks += 1
        if len(pidx):
            self.tickets.append((t, pidx, out))
        return t

    def pump(self) -> int:
        """Submit every due tick (the first carries the queued records). Returns batches submitted."""
        n = self.due()
        for _ in range(n):
            self.tick()
        return n

    def committed(self) -> list[tuple[np.ndarray, np.ndarray]]:
        """The queued requests whose every record is committed (offset < commit index), oldest
        first, as (pidx, offsets); they leave the pending list. A batch is complete (its offsets
        written) once rmq_poll_commit answers RMQ_OK for its ticket, which needs no flush.

        A batch with rejected records (RMQ_OFFSET_NONE) leaves the list too and is reported in
        ``self.rejected`` as (pidx, offsets, stats): its accepted records still commit, and the
        requests queued behind it are not held up by it."""
        done = []
        if not self.tickets:
            return done
        commit = self.engine.commit_snapshot()
        while self.tickets:
            t, pidx, out = self.tickets[0]
            if self.engine.poll(t) is None:
                break
            ok = out != np.uint64(A.RMQ_OFFSET_NONE)
            if np.any(ok & (out >= commit[pidx])):
                break
            self.tickets.pop(0)
            if not np.all(ok):
                try:
                    stats = self.engine.wait(t)  # which rule rejected them (not leader, no space, ...)
                except EngineError:
                    stats = None  # older than the engine's stats ring
                self.rejected.append((pidx, out, stats))
                continue
            done.append((pidx, out))
        return done
