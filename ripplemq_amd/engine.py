"""Python handle over the C-ABI engine (numpy in, numpy out).

Thin host glue for tests, tools and bench.py: every call goes straight to
``libripplemq_engine.so``; nothing here computes the data path.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from dataclasses import dataclass

import numpy as np

from . import _abi as A


class EngineError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {A.STATUS_NAMES.get(status, status)}")


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise EngineError(rc, what)
    return rc


def _ptr(a: np.ndarray | None) -> int | None:
    return None if a is None else a.ctypes.data


_PTRS: dict = {}  # id(array) -> (weak reference, data address): arrays a caller reuses call after call
_PTR_CACHE = os.environ.get("RMQ_PY_PTR_CACHE", "1") != "0"  # (A/B of the cache)


def _ptr_reused(a: np.ndarray) -> int:
    """_ptr of an array passed again and again (a fetch's request and result rows, views of
    page-locked memory from fetch_rows): numpy's .ctypes.data costs ~1.5 us a call, a checked cache
    entry ~0.5 us."""
    if a.base is None or not _PTR_CACHE:  # (an array owning its data can be resized in place: not cached)
        return a.ctypes.data
    e = _PTRS.get(id(a))
    if e is not None and e[0]() is a:
        return e[1]
    if len(_PTRS) > 256:
        _PTRS.clear()
    p = a.ctypes.data
    try:
        _PTRS[id(a)] = (weakref.ref(a), p)
    except TypeError:  # (an object without weak references: no cache)
        pass
    return p


FETCH_RES_DTYPE = np.dtype([
    ("start_offset", "<u8"), ("out_pos", "<u8"), ("count", "<u4"), ("bytes", "<u4"),
    ("status", "<i4"), ("reserved", "<u4"),
])
STATE_FIELDS = ("log_end_offset", "log_end_pos", "log_start_offset", "log_start_pos", "commit",
                "high_watermark", "term", "term_start", "leader_commit", "last_log_term", "voted_term",
                "voted_for", "led", "heard_round")


@dataclass
class EngineConfig:
    num_partitions: int
    replication_factor: int = 3
    segment_bytes: int = 1 << 20
    index_interval: int = 1024
    max_consumers: int = 8
    max_batch_records: int = 65536
    pipeline_depth: int = 2          # batches per pipeline launch group (1..8)
    max_batch_bytes: int = 64 << 20
    device: int = 0
    rank: int = 0
    pool_bytes: int = 0              # ring bytes per replica shared by all partitions (0: P * segment)

    def to_c(self) -> A.RmqConfig:
        c = A.RmqConfig()
        for f, _ in A.RmqConfig._fields_:
            setattr(c, f, getattr(self, f))
        return c


# numpy mirror of rmq_partition_state (bulk read-back)
STATE_DTYPE = np.dtype({"names": [f for f, _ in A.RmqPartitionState._fields_],
                        "formats": ["<u8"] * 8 + [("<u8", A.RMQ_MAX_RF), ("<u4", A.RMQ_MAX_RF), "<u4", "<u4",
                                                  "<u8", "<u8", "<u8", "<u8", "<u4", "<u4", "<u8"],
                        "offsets": [getattr(A.RmqPartitionState, f).offset for f, _ in A.RmqPartitionState._fields_],
                        "itemsize": C.sizeof(A.RmqPartitionState)})


def state_to_dict(s: A.RmqPartitionState, rf: int) -> dict:
    d = {f: int(getattr(s, f)) for f in STATE_FIELDS}
    d["match"] = [int(s.match[r]) for r in range(rf)]
    d["replica_rank"] = [int(s.replica_rank[r]) for r in range(rf)]
    d["leader_slot"] = int(s.leader_slot)
    d["is_leader"] = int(s.is_leader)
    d["segment_bytes"] = int(s.segment_bytes)
    return d


class FetchTicket:
    """An rmq_fetch_async in flight: its ticket and the arrays the engine writes into."""
    __slots__ = ("ticket", "req", "res", "out")

    def __init__(self, ticket: int, req: np.ndarray, res: np.ndarray, out: np.ndarray | None):
        self.ticket, self.req, self.res, self.out = ticket, req, res, out


class Engine:
    """One engine = one HIP device, P partitions, RF co-located or placed replicas."""

    def __init__(self, cfg: EngineConfig, lib_path: str | None = None):
        self.lib = A.load(lib_path) if lib_path else A.load()
        self.cfg = cfg
        h = C.c_void_p()
        c = cfg.to_c()
        _check(self.lib.rmq_create(C.byref(c), C.byref(h)), "rmq_create")
        self.h = h
        self._keep: dict[int, tuple] = {}
        self._pinned: dict[int, np.ndarray] = {}  # rmq_host_alloc buffers by address
        # fetches in flight by ticket: the engine holds raw pointers to their arrays (results, output,
        # page-locked requests) until rmq_fetch_poll answers them or the engine is destroyed
        self._fetching: dict[int, "FetchTicket"] = {}
        # append_device reuses one argument block: a producer loop calls it once per batch
        self._dbatch = A.RmqBatch(0, A.RMQ_MEM_DEVICE)
        self._dticket = C.c_uint64()
        self._dargs = (C.byref(self._dbatch), C.byref(self._dticket))
        self.transport = False  # a replication transport is attached (rounds are collective)
        self.last_offset_ticket = 0

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.rmq_destroy(self.h)
            self.h = None
            self._keep.clear()
            self._fetching.clear()  # (rmq_destroy waited for every fetch)
            for p in list(self._pinned):  # after the engine: no DMA reads them any more
                self.lib.rmq_host_free(None, C.c_void_p(p))
            self._pinned.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- control
    def set_replicas(self, pidx: int, ranks, leader_slot: int) -> None:
        r = (C.c_uint32 * len(ranks))(*ranks)
        _check(self.lib.rmq_set_replicas(self.h, pidx, r, len(ranks), leader_slot), "rmq_set_replicas")

    def set_placement(self, pidx, keys, ranks, leader_slot) -> None:
        """rmq_set_placement: ranks is [n][RF]; keys may be None (unchanged)."""
        pidx = np.ascontiguousarray(pidx, np.uint32)
        ranks = np.ascontiguousarray(ranks, np.uint32).reshape(len(pidx), self.cfg.replication_factor)
        leader_slot = np.ascontiguousarray(leader_slot, np.uint32)
        keys = None if keys is None else np.ascontiguousarray(keys, np.uint64)
        _check(self.lib.rmq_set_placement(self.h, len(pidx), _ptr(pidx), _ptr(keys), _ptr(ranks), _ptr(leader_slot)),
               "rmq_set_placement")

    def attach_local(self, hub: "LocalHub") -> None:
        _check(self.lib.rmq_attach_local(self.h, hub.h), "rmq_attach_local")
        self.transport = True

    def attach_rccl(self, comm_id: bytes, world: int) -> None:
        buf = (C.c_uint8 * 128).from_buffer_copy(comm_id)
        _check(self.lib.rmq_attach_rccl(self.h, buf, world), "rmq_attach_rccl")
        self.transport = True

    def replication_stats(self) -> dict:
        st = A.RmqReplStats()
        _check(self.lib.rmq_replication_stats(self.h, C.byref(st)), "rmq_replication_stats")
        return {f: int(getattr(st, f)) for f, _ in A.RmqReplStats._fields_}

    def read_outbox(self, dst: int) -> np.ndarray:
        n = C.c_uint64()
        _check(self.lib.rmq_read_outbox(self.h, dst, None, 0, C.byref(n)), "rmq_read_outbox")
        out = np.zeros(max(int(n.value), 1), np.uint8)
        _check(self.lib.rmq_read_outbox(self.h, dst, _ptr(out), out.size, C.byref(n)), "rmq_read_outbox")
        return out[:int(n.value)]

    def fault_drop_rounds(self, n: int = 1) -> None:
        """Tests: the next n rounds this engine leads carry no records (rmq_fault_drop_rounds)."""
        _check(self.lib.rmq_fault_drop_rounds(self.h, n), "rmq_fault_drop_rounds")

    def fault_isolate(self, dst: int, n: int = 1) -> None:
        """Tests: the next n rounds this engine sends to dst are lost (rmq_fault_isolate)."""
        _check(self.lib.rmq_fault_isolate(self.h, dst, n), "rmq_fault_isolate")

    def fault_corrupt(self, dst: int, at: int) -> None:
        """Tests: the next round sent to dst has one byte flipped (rmq_fault_corrupt)."""
        _check(self.lib.rmq_fault_corrupt(self.h, dst, at), "rmq_fault_corrupt")

    def fault_cut(self, dst: int, n: int = 1) -> None:
        """Tests: as fault_isolate, and the next drain's commit notices to dst are lost (rmq_fault_cut)."""
        _check(self.lib.rmq_fault_cut(self.h, dst, n), "rmq_fault_cut")

    def become_leader(self, pidx: int, term: int) -> None:
        _check(self.lib.rmq_become_leader(self.h, pidx, term), "rmq_become_leader")

    def vote(self, pidx: int, term: int, candidate: int, cand_last_log_term: int, cand_log_end: int) -> bool:
        """Raft RequestVote on this replica (rmq_vote): True if the vote was granted."""
        g = C.c_uint32(0)
        _check(self.lib.rmq_vote(self.h, pidx, term, candidate, cand_last_log_term, cand_log_end, C.byref(g)),
               "rmq_vote")
        return bool(g.value)

    def set_replica_cursor(self, pidx, offset) -> None:
        """Where RMQ_FETCH_REPLICA reads of these partitions start (rmq_set_replica_cursor)."""
        pidx = np.ascontiguousarray(pidx, np.uint32)
        offset = np.ascontiguousarray(offset, np.uint64)
        _check(self.lib.rmq_set_replica_cursor(self.h, len(pidx), _ptr(pidx), _ptr(offset)), "rmq_set_replica_cursor")

    def set_vote(self, pidx: int, term: int, voted_for: int) -> None:
        """Replay of a persisted vote (rmq_set_vote)."""
        _check(self.lib.rmq_set_vote(self.h, pidx, term, voted_for), "rmq_set_vote")

    def leader_silent(self, silent_rounds: int, timeout_ms: int = 0) -> np.ndarray:
        """Followed partitions whose leader has been silent (rmq_leader_silent)."""
        n = C.c_uint32(0)
        _check(self.lib.rmq_leader_silent(self.h, silent_rounds, timeout_ms, None, 0, C.byref(n)), "rmq_leader_silent")
        out = np.zeros(max(n.value, 1), np.uint32)
        _check(self.lib.rmq_leader_silent(self.h, silent_rounds, timeout_ms, _ptr(out), n.value, C.byref(n)),
               "rmq_leader_silent")
        return out[:n.value]

    # ---- append
    def append_async(self, pidx: np.ndarray, lens: np.ndarray, payload: np.ndarray,
                     payload_off: np.ndarray | None = None) -> tuple[int, np.ndarray]:
        pidx = np.ascontiguousarray(pidx, dtype=np.uint32)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        if payload_off is not None:
            payload_off = np.ascontiguousarray(payload_off, dtype=np.uint64)
        out = np.empty(len(pidx), dtype=np.uint64)
        b = A.RmqBatch(len(pidx), A.RMQ_MEM_HOST, _ptr(pidx), _ptr(lens), _ptr(payload_off),
                       _ptr(payload) if payload.size else None, payload.size)
        t = C.c_uint64()
        _check(self.lib.rmq_append(self.h, C.byref(b), _ptr(out), C.byref(t)), "rmq_append")
        self._keep[t.value] = (pidx, lens, payload, payload_off, out)
        return t.value, out

    # ---- page-locked host batches (RMQ_MEM_PINNED)
    def host_empty(self, count: int, dtype) -> np.ndarray:
        """A numpy array in page-locked host memory (rmq_host_alloc), freed with the engine or by
        host_release. Batches whose arrays all come from here go to the device by DMA alone."""
        dtype = np.dtype(dtype)
        nbytes = max(int(count) * dtype.itemsize, 16)
        p = C.c_void_p()
        _check(self.lib.rmq_host_alloc(self.h, nbytes, C.byref(p)), "rmq_host_alloc")
        buf = (C.c_uint8 * nbytes).from_address(p.value)
        arr = np.frombuffer(buf, np.uint8, nbytes)[:int(count) * dtype.itemsize].view(dtype)
        self._pinned[p.value] = arr
        return arr

    def host_release(self, arr: np.ndarray) -> None:
        p = arr.__array_interface__["data"][0]
        if self._pinned.pop(p, None) is not None:
            _check(self.lib.rmq_host_free(self.h, C.c_void_p(p)), "rmq_host_free")

    def host_register(self, arr: np.ndarray) -> None:
        """Page-lock a caller's contiguous array in place (rmq_host_register), so it can serve as
        pinned batch arrays or pinned fetch rows; undone by host_unregister before it is freed."""
        if not arr.flags["C_CONTIGUOUS"] or arr.nbytes == 0:
            raise ValueError("host_register needs a non-empty contiguous array")
        _check(self.lib.rmq_host_register(self.h, C.c_void_p(arr.__array_interface__["data"][0]), arr.nbytes),
               "rmq_host_register")

    def host_unregister(self, arr: np.ndarray) -> None:
        _check(self.lib.rmq_host_unregister(self.h, C.c_void_p(arr.__array_interface__["data"][0])),
               "rmq_host_unregister")

    def append_pinned_async(self, pidx: np.ndarray, lens: np.ndarray, payload: np.ndarray, out: np.ndarray,
                            payload_off: np.ndarray | None = None, payload_bytes: int | None = None) -> int:
        """rmq_append of a batch whose arrays (and `out`, uint64[n]) are page-locked (host_empty):
        one DMA per section, no host copy; the arrays must stay unchanged until the ticket
        completes. Payload ranges are checked on the device (rejected_invalid), like device
        batches."""
        n = len(pidx)
        nb = payload.size if payload_bytes is None else int(payload_bytes)
        b = A.RmqBatch(n, A.RMQ_MEM_PINNED, _ptr(pidx), _ptr(lens), _ptr(payload_off),
                       _ptr(payload) if nb else None, nb)
        t = C.c_uint64()
        _check(self.lib.rmq_append(self.h, C.byref(b), _ptr(out), C.byref(t)), "rmq_append")
        return t.value

    def append_device(self, n: int, d_pidx: int, d_len: int, d_payload: int, payload_bytes: int,
                      d_out: int, d_payload_off: int | None = None) -> int:
        b = self._dbatch
        b.n, b.pidx, b.len, b.payload_off, b.payload, b.payload_bytes = (
            n, d_pidx, d_len, d_payload_off, d_payload, payload_bytes)
        rc = self.lib.rmq_append(self.h, self._dargs[0], d_out, self._dargs[1])
        if rc < 0:
            raise EngineError(rc, "rmq_append")
        return self._dticket.value

    def poll(self, ticket: int, want_commit: bool = False):
        P = self.cfg.num_partitions
        commit = np.empty(P, np.uint64) if want_commit else None
        hw = np.empty(P, np.uint64) if want_commit else None
        rc = _check(self.lib.rmq_poll_commit(self.h, ticket, _ptr(commit), _ptr(hw)), "rmq_poll_commit")
        if rc == A.RMQ_PENDING:
            return None
        self._keep.pop(ticket, None)
        return (commit, hw) if want_commit else True

    def wait(self, ticket: int) -> dict | None:
        """Stats of a completed ticket, or None while it is pending: with a replication transport a
        ticket is applied only by an rmq_sync on every rank (the caller's arrays stay referenced
        until then; their out offsets are not written yet)."""
        st = A.RmqAppendStats()
        rc = _check(self.lib.rmq_ticket_stats(self.h, ticket, C.byref(st)), "rmq_ticket_stats")
        if rc == A.RMQ_PENDING:
            return None
        self._keep.pop(ticket, None)
        return {f: int(getattr(st, f)) for f, _ in A.RmqAppendStats._fields_}

    def append(self, pidx, lens, payload, payload_off=None) -> tuple[np.ndarray, dict]:
        """Synchronous append: offsets and stats of the batch. With a replication transport the
        batch is applied only by a collective rmq_sync, so this raises RMQ_PENDING (keep the
        ticket: append_async + sync + wait). The check comes before anything is queued, so a caller
        that retries after the error never appends the records twice."""
        if self.transport:
            raise EngineError(A.RMQ_PENDING, "rmq_append (transport attached: use append_async, then rmq_sync "
                                             "on every rank applies it)")
        t, out = self.append_async(pidx, lens, payload, payload_off)
        stats = self.wait(t)
        if stats is None:
            raise EngineError(A.RMQ_PENDING, "rmq_append (transport attached: rmq_sync on every rank applies it)")
        return out, stats

    def commit_snapshot(self) -> np.ndarray:
        """Commit index of every partition after everything submitted so far."""
        P = self.cfg.num_partitions
        commit = np.empty(P, np.uint64)
        _check(self.lib.rmq_poll_commit(self.h, 0, _ptr(commit), None), "rmq_poll_commit")
        return commit

    def sync(self) -> None:
        _check(self.lib.rmq_sync(self.h), "rmq_sync")
        self._keep.clear()  # every ticket is complete: its out offsets are in the caller's arrays

    def ack(self, pidx, slot, match) -> None:
        pidx = np.ascontiguousarray(pidx, np.uint32)
        slot = np.ascontiguousarray(slot, np.uint32)
        match = np.ascontiguousarray(match, np.uint64)
        _check(self.lib.rmq_ack(self.h, _ptr(pidx), _ptr(slot), _ptr(match), len(pidx)), "rmq_ack")

    def commit_consumer_offset(self, pidx, consumer, offset) -> tuple[int, np.ndarray]:
        """rmq_commit_consumer_offset: (rc, per-item status); the call's ticket (0 if no item was
        accepted) is in self.last_offset_ticket, for poll_offsets."""
        pidx = np.ascontiguousarray(pidx, np.uint32)
        consumer = np.ascontiguousarray(consumer, np.uint32)
        offset = np.ascontiguousarray(offset, np.uint64)
        status = np.zeros(len(pidx), np.int32)
        t = C.c_uint64()
        rc = self.lib.rmq_commit_consumer_offset(self.h, _ptr(pidx), _ptr(consumer), _ptr(offset),
                                                 len(pidx), _ptr(status), C.byref(t))
        if rc in (A.RMQ_EDEVICE, A.RMQ_ENOMEM):
            raise EngineError(rc, "rmq_commit_consumer_offset")
        self.last_offset_ticket = int(t.value)
        return rc, status

    def poll_offsets(self, ticket: int) -> int:
        """rmq_poll_commit of a consumer-offset ticket: RMQ_OK (the rows are on a quorum),
        RMQ_PENDING, or RMQ_ENOTLEADER (leadership moved first: the commit may be lost)."""
        rc = self.lib.rmq_poll_commit(self.h, ticket, None, None)
        if rc not in (A.RMQ_OK, A.RMQ_PENDING, A.RMQ_ENOTLEADER):
            raise EngineError(rc, "rmq_poll_commit (offsets)")
        return rc

    def fetch(self, pidx, consumer, max_records, out_cap: int | None = None, commit: bool = False,
              out: np.ndarray | None = None, replica: bool = False):
        """rmq_fetch into a host array (sized by a first call when out_cap is None, or the caller's
        uint8 `out`, e.g. page-locked from host_empty: one call, RMQ_ENOSPC if it is too small);
        commit: RMQ_FETCH_COMMIT on every request (the size query commits nothing); replica:
        RMQ_FETCH_REPLICA (this engine's own replica from its replica cursor, leader or follower)."""
        n = len(pidx)
        req = np.zeros((n, 4), np.uint32)
        req[:, 0], req[:, 1], req[:, 2] = pidx, consumer, max_records
        req[:, 3] = A.RMQ_FETCH_REPLICA if replica else 0
        res = np.zeros(n, FETCH_RES_DTYPE)
        if out is not None:
            if commit:
                req[:, 3] |= A.RMQ_FETCH_COMMIT
            used = C.c_uint64()
            rc = self.lib.rmq_fetch(self.h, _ptr(req), n, A.RMQ_MEM_HOST, _ptr(out), out.size, _ptr(res),
                                    C.byref(used))
            if rc not in (A.RMQ_OK, A.RMQ_ENOSPC):
                raise EngineError(rc, "rmq_fetch")
            return rc, res, out, int(used.value)
        if out_cap is None:
            used = C.c_uint64()
            rc = self.lib.rmq_fetch(self.h, _ptr(req), n, A.RMQ_MEM_HOST, None, 0, _ptr(res), C.byref(used))
            if rc not in (A.RMQ_OK, A.RMQ_ENOSPC):
                raise EngineError(rc, "rmq_fetch")
            out_cap = int(used.value)
        if commit:
            req[:, 3] |= A.RMQ_FETCH_COMMIT
        out = np.zeros(max(out_cap, 1), np.uint8)
        used = C.c_uint64()
        rc = self.lib.rmq_fetch(self.h, _ptr(req), n, A.RMQ_MEM_HOST, _ptr(out), out_cap, _ptr(res), C.byref(used))
        if rc not in (A.RMQ_OK, A.RMQ_ENOSPC):
            raise EngineError(rc, "rmq_fetch")
        return rc, res, out[:out_cap], int(used.value)

    def fetch_device(self, pidx, consumer, max_records, d_out: int, out_cap: int, commit: bool = False,
                     req: np.ndarray | None = None, res: np.ndarray | None = None, pinned_rows: bool = False,
                     d_rows: tuple[int, int, int] | None = None):
        """rmq_fetch into a device buffer (16-byte aligned); returns (rc, res, bytes_used). req / res:
        the caller's arrays (pidx / consumer / max_records None leave req's columns as they are);
        pinned_rows: page-locked ones (fetch_rows), read and written by the kernels in place
        (RMQ_FETCH_PINNED_ROWS). d_rows = (n, device request rows, device result rows): rows in
        device memory (RMQ_FETCH_DEVICE_ROWS, flags ignored); res is then None."""
        if d_rows is not None:
            n, d_req, d_res = d_rows
            used = C.c_uint64()
            rc = self.lib.rmq_fetch(self.h, C.c_void_p(d_req), n, A.RMQ_MEM_DEVICE | A.RMQ_FETCH_DEVICE_ROWS,
                                    d_out, out_cap, C.c_void_p(d_res), C.byref(used))
            if rc not in (A.RMQ_OK, A.RMQ_ENOSPC):
                raise EngineError(rc, "rmq_fetch")
            return rc, None, int(used.value)
        n = len(pidx) if pidx is not None else len(req)
        if req is None:
            req = np.zeros((n, 4), np.uint32)
            req[:, 3] = A.RMQ_FETCH_COMMIT if commit else 0
        for col, v in ((0, pidx), (1, consumer), (2, max_records)):
            if v is not None:
                req[:, col] = v
        if res is None:
            res = np.zeros(n, FETCH_RES_DTYPE)
        used = C.c_uint64()
        mem = A.RMQ_MEM_DEVICE | (A.RMQ_FETCH_PINNED_ROWS if pinned_rows else 0)
        rc = self.lib.rmq_fetch(self.h, _ptr_reused(req), n, mem, d_out, out_cap, _ptr_reused(res), C.byref(used))
        if rc not in (A.RMQ_OK, A.RMQ_ENOSPC):
            raise EngineError(rc, "rmq_fetch")
        return rc, res, int(used.value)

    def fetch_async(self, pidx, consumer, max_records, d_out: int | None = None, out_cap: int = 0,
                    out: np.ndarray | None = None, req: np.ndarray | None = None,
                    res: np.ndarray | None = None, pinned_rows: bool = False) -> "FetchTicket":
        """rmq_fetch_async into a device buffer (d_out, 16-byte aligned) or a host array (out): the
        call returns at once; fetch_poll(ticket) gives (rc, res, bytes_used) once it completes. The
        handle keeps the request, result and output arrays alive until then. req ([n, 4] uint32)
        and res (FETCH_RES_DTYPE[n]) may be a caller's arrays reused from call to call; with req
        given, pidx / consumer / max_records None leave those columns as they are (column 3: the
        requests' flags, RMQ_FETCH_COMMIT). pinned_rows: req and res are page-locked (fetch_rows)
        and the kernels read and write them in place (RMQ_FETCH_PINNED_ROWS); req then stays
        unchanged until the ticket completes."""
        n = len(pidx) if pidx is not None else len(req)
        if pinned_rows and (req is None or res is None):
            raise ValueError("pinned_rows needs the caller's page-locked req and res (fetch_rows)")
        if req is None:
            req = np.empty((n, 4), np.uint32)
            req[:, 3] = 0
        for col, v in ((0, pidx), (1, consumer), (2, max_records)):
            if v is not None:
                req[:, col] = v
        if res is None:
            res = np.empty(n, FETCH_RES_DTYPE)
        if d_out is not None:
            mem, ptr = A.RMQ_MEM_DEVICE, C.c_void_p(d_out)
        else:
            out_cap = 0 if out is None else min(int(out_cap) or out.size, out.size)
            mem, ptr = A.RMQ_MEM_HOST, (_ptr(out) if out is not None else None)
        if pinned_rows:
            mem |= A.RMQ_FETCH_PINNED_ROWS
        t = C.c_uint64()
        _check(self.lib.rmq_fetch_async(self.h, _ptr_reused(req), n, mem, ptr, out_cap, _ptr_reused(res), C.byref(t)),
               "rmq_fetch_async")
        tk = FetchTicket(t.value, req, res, out)
        self._fetching[t.value] = tk
        return tk

    def fetch_rows(self, n: int):
        """A page-locked request array ([n, 4] uint32, zeroed) and result array (FETCH_RES_DTYPE[n])
        for fetch_async(..., pinned_rows=True); freed with the engine or by host_release."""
        req = self.host_empty(4 * n, np.uint32).reshape(n, 4)
        req[:] = 0
        return req, self.host_empty(n, FETCH_RES_DTYPE)

    def fetch_poll(self, tk: "FetchTicket", wait: bool = False):
        """(rc, res, bytes_used) of an rmq_fetch_async ticket, or None while it runs."""
        used = C.c_uint64()
        rc = self.lib.rmq_fetch_poll(self.h, tk.ticket, 1 if wait else 0, C.byref(used))
        if rc == A.RMQ_PENDING:
            return None
        self._fetching.pop(tk.ticket, None)
        if rc not in (A.RMQ_OK, A.RMQ_ENOSPC):
            raise EngineError(rc, "rmq_fetch_poll")
        return rc, tk.res, int(used.value)

    def set_segments(self, pidx, segment_bytes) -> None:
        """Ring sizes of partitions pidx[i] (rmq_set_segments: retention at a smaller size first, the
        retained log keeps its offsets and positions)."""
        p = np.ascontiguousarray(pidx, np.uint32)
        sb = np.ascontiguousarray(segment_bytes, np.uint64)
        _check(self.lib.rmq_set_segments(self.h, len(p), p.ctypes.data_as(C.POINTER(C.c_uint32)),
                                         sb.ctypes.data_as(C.POINTER(C.c_uint64))), "rmq_set_segments")

    # ---- read-back
    def states(self, first: int = 0, n: int | None = None) -> np.ndarray:
        """rmq_get_partition_states: the states of partitions [first, first + n) as a structured
        array of rmq_partition_state (one device copy per field)."""
        n = self.cfg.num_partitions - first if n is None else n
        out = np.zeros(n, STATE_DTYPE)
        _check(self.lib.rmq_get_partition_states(self.h, first, n, _ptr(out)), "rmq_get_partition_states")
        return out

    def state(self, pidx: int) -> dict:
        s = A.RmqPartitionState()
        _check(self.lib.rmq_get_partition_state(self.h, pidx, C.byref(s)), "rmq_get_partition_state")
        return state_to_dict(s, self.cfg.replication_factor)

    def read_segment(self, replica: int, pidx: int, ring_off: int = 0, n: int | None = None) -> np.ndarray:
        n = self.state(pidx)["segment_bytes"] - ring_off if n is None else n
        out = np.empty(n, np.uint8)
        _check(self.lib.rmq_read_segment(self.h, replica, pidx, ring_off, n, _ptr(out)), "rmq_read_segment")
        return out

    def read_index(self, pidx: int, m_first: int, count: int) -> np.ndarray:
        out = np.empty((count, 2), np.uint64)
        _check(self.lib.rmq_read_index(self.h, pidx, m_first, count, _ptr(out)), "rmq_read_index")
        return out

    def consumer_table(self, first: int = 0, n: int | None = None) -> np.ndarray:
        """rmq_read_consumer_table: the consumer-offset rows of partitions [first, first + n)."""
        n = self.cfg.num_partitions - first if n is None else n
        out = np.empty((n, self.cfg.max_consumers), np.uint64)
        _check(self.lib.rmq_read_consumer_table(self.h, first, n, _ptr(out)), "rmq_read_consumer_table")
        return out

    def consumer_offsets(self, pidx: int) -> np.ndarray:
        out = np.empty(self.cfg.max_consumers, np.uint64)
        _check(self.lib.rmq_read_consumer_offsets(self.h, pidx, _ptr(out)), "rmq_read_consumer_offsets")
        return out

    # ---- device memory / timing
    def device_alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        _check(self.lib.rmq_device_alloc(self.h, nbytes, C.byref(p)), "rmq_device_alloc")
        return p.value

    def device_free(self, p: int) -> None:
        _check(self.lib.rmq_device_free(self.h, p), "rmq_device_free")

    def h2d(self, dst: int, src: np.ndarray) -> None:
        src = np.ascontiguousarray(src)
        _check(self.lib.rmq_memcpy(self.h, dst, _ptr(src), src.nbytes, 0), "rmq_memcpy")

    def d2h(self, dst: np.ndarray, src: int) -> None:
        _check(self.lib.rmq_memcpy(self.h, _ptr(dst), src, dst.nbytes, 1), "rmq_memcpy")

    def profile(self, enable: int) -> None:
        """rmq_profile_enable: 0 off, 1 on, k >= 2 on with every fetch's kernels run k times."""
        _check(self.lib.rmq_profile_enable(self.h, int(enable)), "rmq_profile_enable")

    def profile_query(self, kernel: int) -> tuple[int, float]:
        n, ms = C.c_uint64(), C.c_double()
        _check(self.lib.rmq_profile_query(self.h, kernel, C.byref(n), C.byref(ms)), "rmq_profile_query")
        return int(n.value), float(ms.value)

    def device_info(self) -> tuple[str, int]:
        buf = C.create_string_buffer(256)
        cu = C.c_uint32()
        _check(self.lib.rmq_device_info(self.h, buf, 256, C.byref(cu)), "rmq_device_info")
        return buf.value.decode(), int(cu.value)


class LocalHub:
    """rmq_local_hub: in-process transport for `world` engines, each driven by its own thread."""

    def __init__(self, world: int, lib_path: str | None = None):
        self.lib = A.load(lib_path) if lib_path else A.load()
        h = C.c_void_p()
        _check(self.lib.rmq_local_hub_create(world, C.byref(h)), "rmq_local_hub_create")
        self.h = h

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.rmq_local_hub_destroy(self.h)
            self.h = None


def rccl_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    _check(A.load().rmq_rccl_unique_id(buf), "rmq_rccl_unique_id")
    return bytes(buf)


def parse_records(buf: np.ndarray) -> list[tuple[int, int, bytes]]:
    """Split FORMAT.md records: [(offset, crc, payload), ...]."""
    out, pos, b = [], 0, buf.tobytes()
    while pos + 16 <= len(b):
        off = int.from_bytes(b[pos:pos + 8], "little")
        ln = int.from_bytes(b[pos + 8:pos + 12], "little")
        crc = int.from_bytes(b[pos + 12:pos + 16], "little")
        out.append((off, crc, b[pos + 16:pos + 16 + ln]))
        pos += 16 + ((ln + 15) & ~15)
    return out
