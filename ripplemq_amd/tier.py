"""Durable segment files below the HBM rings, and replay.

The reference never evicts a record: ``PartitionStateMachine`` keeps every message in its
``messages`` list (``mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java:26,64-69``)
and jraft persists the log under the partition's data path (``PartitionRaftServer.java:53,88-90``).
The engine's replica rings keep a retained window only (FORMAT.md §4): a fetch below it answers
``RMQ_EOFFSET``. This module is the tier that restores the reference's semantics on the host side:

* ``DurableLog.spill()`` moves every committed record not yet durable into per-partition segment
  files with ONE ``rmq_fetch`` for all partitions, led or followed: replica reads
  (``RMQ_FETCH_REPLICA | RMQ_FETCH_COMMIT``) start at each partition's replica cursor (the durable
  end, local to the engine) and end at the replica's commit, so the fetch kernel returns exactly the
  records ``[durable end, commit)`` of this engine's own replica and moves the cursor on the device.
  jraft keeps the whole log on every node (``PartitionRaftServer.java:53,88-90``): a follower's tier
  persists its replica too, so a leader moved to it serves consumers below its rings from its own
  files. A segment file holds the records exactly as the rings do (FORMAT.md
  §1: 16-byte header {offset, length, CRC32C} + payload padded to 16 bytes), named by its first
  offset (``p<pidx>/<first offset>.seg``), rolled at ``segment_file_bytes``.
* ``DurableLog.read(p, off, max)`` serves ``[off, min(off + max, durable end))`` from the files
  (the broker's ``process_batch_read`` falls back to it on ``RMQ_EOFFSET`` after a spill, so a
  consumer below the rings gets what the reference's list would give it).
* ``replay(directory, engine)`` rebuilds a fresh engine's logs from the files: the records are
  re-appended in offset order (the engine computes every CRC again) and the result is checked
  bit for bit against the files: offsets, and the ring bytes of the retained window.
* The rest of a partition's durable state, as jraft keeps it in the partition's log and
  ``raft_meta`` directory (``PartitionRaftServer.java:53,88-90``): every spill also writes the
  partition's consumer-offset row (the reference's offset commits are log entries applied by
  ``PartitionStateMachine.java:71-77``; the tier's own cursor slot stored as 0, the durable end
  being in the ends file) to ``p<pidx>/offsets.bin`` and its term and cursor slot to
  ``p<pidx>/meta.json``, each replaced atomically (write, fsync if asked, rename) when it changed;
  ``replay`` restores both after the records (the term through ``rmq_become_leader``, so only
  appends of the restored term advance the commit). Offsets and terms are durable at spill
  granularity, like the records; a vote is durable before it is answered (``save_vote``, Raft's
  votedFor in raft_meta, ``PartitionRaftServer.java:89``).

Spill must run at least once per retained window of every partition (rings hold ``retain``
batches of their traffic, ``ripplemq_amd/rings.py``); a cursor below a ring's start raises, since
records were lost before they were durable.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import time

import numpy as np

from . import _abi as A
from .engine import EngineError

SEG_SUFFIX = ".seg"
OFFSETS_FILE = "offsets.bin"   # u64 consumer offsets of the partition (rmq_config.max_consumers)
META_FILE = "meta.json"        # {"term", "voted_term", "voted_for", "cursor"}: the partition's raft_meta
ENDS_FILE = "durable_ends.bin" # tier root: u64 pairs {partition, durable end} of the last spill


def load_ends(root: str) -> dict[int, int]:
    """The durable end of every partition the last completed spill recorded (empty if none)."""
    try:
        a = np.fromfile(os.path.join(root, ENDS_FILE), np.uint64).reshape(-1, 2)
    except (FileNotFoundError, ValueError):
        return {}
    return {int(p): int(e) for p, e in a}


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf.view(np.uint8).reshape(-1))
    return np.frombuffer(bytes(buf), np.uint8)


def _scan(buf, first: int, max_records: int, check: bool, positions: bool):
    """rmq_scan_records (the engine library's native walk of back-to-back FORMAT.md §1 records)."""
    a = _as_u8(buf)
    pos = np.zeros(max_records + 1, np.uint64) if positions else None
    n, nb = C.c_uint64(), C.c_uint64()
    rc = A.load().rmq_scan_records(a.ctypes.data if a.size else None, a.size, first, max_records,
                                   A.RMQ_SCAN_CHECK if check else 0,
                                   pos.ctypes.data if pos is not None else None, C.byref(n), C.byref(nb))
    if rc:
        raise EngineError(rc, "rmq_scan_records")
    k = int(n.value)
    return k, int(nb.value), (pos[:k + 1].astype(np.int64) if pos is not None else None)


def record_positions(buf: np.ndarray, count: int | None = None, first: int | None = None) -> np.ndarray:
    """Byte positions of the FORMAT.md §1 records laid back to back in ``buf`` (plus the end); the
    header offsets must run first, first + 1, ... (first: the first header's)."""
    a = _as_u8(buf)
    if first is None:
        first = int(a[:8].view(np.uint64)[0]) if a.size >= 16 else 0
    cap = a.size // 16 if count is None else int(count)
    return _scan(a, first, cap, False, True)[2]


def whole_records(b, first: int, durable_end: int | None = None) -> tuple[int, int]:
    """(records, bytes) of the longest prefix of ``b`` made of whole FORMAT.md §1 records whose
    header offsets run first, first + 1, ... and whose CRC32C and zero padding check out: a crash in
    the middle of a segment write leaves a torn last record (cut short, garbage, or zero-filled by
    the file system), which this excludes. A zero-filled record at offset `first` (header offset 0,
    length 0, CRC 0) is also a valid empty message: past `durable_end` (the end the last completed
    spill recorded) an all-zero record counts as torn."""
    a = _as_u8(b)
    k, nb, pos = _scan(a, first, a.size // 16, True, True)
    if durable_end is not None:
        for i in range(k):
            if first + i >= durable_end and not a[pos[i]:pos[i + 1]].any():
                return i, int(pos[i])
    if nb + 16 <= a.size:
        # a torn tail ends the file; whole records AFTER the bad one mean a record inside the log
        # was corrupted (a flipped byte), which no cut may hide
        ln = int(a[nb + 8:nb + 12].view(np.uint32)[0])
        nxt = nb + 16 + ((ln + 15) & ~15)
        if nxt + 16 <= a.size and _scan(a[nxt:], first + k + 1, 1, True, False)[0]:
            raise EngineError(A.RMQ_EINVAL, f"record {first + k} is corrupted inside the segment")
    return k, nb


class _PartitionFiles:
    """One partition's segment files: record k (offset base + k) at logical byte pos[k] of the
    concatenated files; segment s covers logical bytes [seg_pos[s], seg_pos[s + 1])."""

    def __init__(self, root: str, p: int, segment_file_bytes: int, durable: int = 0):
        self.dir = os.path.join(root, f"p{p:06d}")
        self._row = None     # the consumer-offset row / meta last written (no re-read per spill)
        self._meta = None
        self._fd = -1        # the last segment file, open for appends (spill)
        os.makedirs(self.dir, exist_ok=True)
        self.limit = segment_file_bytes
        self.base = 0
        self._pos = np.zeros(1024, np.int64)  # record positions with room to grow (pos: the live part)
        self._n = 1
        self.seg_first: list[int] = []   # first offset of every segment file
        self.seg_pos: list[int] = []     # its first logical byte
        self._owner = None   # the DurableLog whose spills hold positions not merged here yet
        self._li = -1        #   and this partition's index there
        names = sorted(int(f[:-len(SEG_SUFFIX)]) for f in os.listdir(self.dir) if f.endswith(SEG_SUFFIX))
        cat, acc = [], 0
        for i, first in enumerate(names):  # reopen: walk the headers of every file, in offset order
            data = np.fromfile(self._path(first), np.uint8)
            n, whole = whole_records(data, first, durable)
            if whole != data.size:
                # a torn tail (the spill that wrote it never advanced the durable cursor, so the next
                # spill fetches those records again): cut the file back to its last whole record
                if i != len(names) - 1:
                    raise EngineError(A.RMQ_EINVAL, f"{self.dir}: segment {first} is torn and not the last one")
                os.truncate(self._path(first), whole)
                data = data[:whole]
            if n == 0:
                os.remove(self._path(first))
                continue
            rp = record_positions(data, n, first)
            if not self.seg_first:
                self.base = first
            elif first != self.base + sum(len(x) for x in cat):
                raise EngineError(A.RMQ_EINVAL, f"{self.dir}: segment {first} does not continue the log")
            self.seg_first.append(first)
            self.seg_pos.append(acc)
            cat.append(rp[:-1] + acc)
            acc += int(rp[-1])
        if cat:
            self._set_pos(np.concatenate(cat + [np.asarray([acc], np.int64)]))

    @property
    def pos(self) -> np.ndarray:
        """Logical byte position of every durable record, then the end."""
        if self._owner is not None:
            self._owner._merge(self._li)
        return self._pos[:self._n]

    def _set_pos(self, v: np.ndarray) -> None:
        if len(v) > len(self._pos):
            self._pos = np.zeros(max(len(v), 2 * len(self._pos)), np.int64)
        self._pos[:len(v)] = v
        self._n = len(v)

    def _path(self, first: int) -> str:
        return os.path.join(self.dir, f"{first:020d}{SEG_SUFFIX}")

    def _replace(self, name: str, data: bytes, fsync: bool) -> None:
        tmp = os.path.join(self.dir, name + ".tmp")
        with open(tmp, "wb") as f:
            f.write(data)
            if fsync:
                f.flush()
                os.fsync(f.fileno())
        os.replace(tmp, os.path.join(self.dir, name))

    def save_state(self, offsets: np.ndarray, term: int, cursor: int, fsync: bool, vote=(0, A.RMQ_NO_VOTE),
                   led: int = 1) -> None:
        """The partition's consumer-offset row, term and vote (jraft's raft_meta term / votedFor,
        PartitionRaftServer.java:89), each rewritten only when it changed. The
        tier's own cursor slot is stored as 0 (the durable end is in the ends file and moves with
        every spill: the row then changes only when consumers commit)."""
        row = np.array(offsets, np.uint64)
        if 0 <= cursor < len(row):
            row[cursor] = 0
        row = row.tobytes()
        if self._row is None:
            self._row = self.load_offsets_bytes()
        if row != self._row:
            self._replace(OFFSETS_FILE, row, fsync)
            self._row = row
        self.save_meta(term, vote, cursor, fsync, led)

    def save_meta(self, term: int, vote, cursor: int, fsync: bool, led: int = 1) -> None:
        """meta.json (term, vote, whether this replica led the vote's term, cursor) when it changed:
        written to a temporary file and renamed."""
        meta = {"term": int(term), "voted_term": int(vote[0]), "voted_for": int(vote[1]), "led": int(led),
                "cursor": int(cursor)}
        if self._meta is None:
            self._meta = self.load_meta()
        if self._meta != meta:
            self._replace(META_FILE, json.dumps(meta).encode(), fsync)
            self._meta = meta

    def load_offsets_bytes(self) -> bytes:
        try:
            with open(os.path.join(self.dir, OFFSETS_FILE), "rb") as f:
                return f.read()
        except FileNotFoundError:
            return b""

    def load_meta(self) -> dict:
        try:
            with open(os.path.join(self.dir, META_FILE)) as f:
                return json.load(f)
        except FileNotFoundError:
            return {}

    @property
    def end(self) -> int:
        """Offset after the last durable record."""
        return self.base + len(self.pos) - 1

    def append_fd(self, first: int) -> tuple[int, int]:
        """(fd, logical bytes so far) for a spill that appends records from offset `first`: the last
        segment file, open for appends, or a new one when it reached the size limit."""
        if not self.seg_first:
            self.base = first
        elif first != self.end:
            raise EngineError(A.RMQ_EINVAL, f"{self.dir}: spill of offset {first} does not continue {self.end}")
        total = int(self.pos[-1])
        if not self.seg_first or total - self.seg_pos[-1] >= self.limit:
            self.close()
            self.seg_first.append(first)
            self.seg_pos.append(total)
        if self._fd < 0:
            self._fd = os.open(self._path(self.seg_first[-1]), os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        return self._fd, total

    def add_positions(self, rp: np.ndarray, total: int) -> None:
        """The positions of records appended at logical byte `total` (rp: inside their run, then its end)."""
        n0 = self._n - 1  # the end entry is overwritten by the first new record's position
        if n0 + len(rp) > len(self._pos):
            grown = np.zeros(max(n0 + len(rp), 2 * len(self._pos)), np.int64)
            grown[:self._n] = self._pos[:self._n]
            self._pos = grown
        self._pos[n0:n0 + len(rp)] = rp
        self._pos[n0:n0 + len(rp)] += total
        self._n = n0 + len(rp)

    def close(self) -> None:
        if self._fd >= 0:
            os.close(self._fd)
            self._fd = -1

    def read_bytes(self, a: int, b: int) -> bytes:
        """Logical bytes [a, b) across the segment files."""
        out = []
        for s, first in enumerate(self.seg_first):
            lo = self.seg_pos[s]
            hi = self.seg_pos[s + 1] if s + 1 < len(self.seg_pos) else int(self.pos[-1])
            x, y = max(a, lo), min(b, hi)
            if x < y:
                with open(self._path(first), "rb") as f:
                    f.seek(x - lo)
                    out.append(f.read(y - x))
        return b"".join(out)

    def read_records(self, off: int, end: int) -> bytes:
        """The record images of offsets [off, end) (both within [base, self.end])."""
        return self.read_bytes(int(self.pos[off - self.base]), int(self.pos[end - self.base]))


def split_records(data: bytes) -> list[tuple[int, int, bytes]]:
    """[(offset, crc, payload)] of back-to-back FORMAT.md §1 records."""
    out, pos = [], 0
    while pos + 16 <= len(data):
        off = int.from_bytes(data[pos:pos + 8], "little")
        ln = int.from_bytes(data[pos + 8:pos + 12], "little")
        crc = int.from_bytes(data[pos + 12:pos + 16], "little")
        out.append((off, crc, data[pos + 16:pos + 16 + ln]))
        pos += 16 + ((ln + 15) & ~15)
    return out


class DurableLog:
    """Segment files of the partitions ``partitions`` of one engine (every partition it holds a
    replica of, led or followed), fed by spill from the engine's own replica."""

    def __init__(self, engine, directory: str, partitions, cursor: int, *,
                 segment_file_bytes: int = 64 << 20, fsync: bool = False, start=None):
        self.engine = engine
        self.dir = directory
        self.cursor = int(cursor)
        self.fsync = fsync
        ends = load_ends(directory)
        self.parts = {int(p): _PartitionFiles(directory, int(p), segment_file_bytes, ends.get(int(p), 0))
                      for p in partitions}
        self._saved = None  # [partition of parts][row, term, voted term, voted for] as last saved
        self._buf = None    # the spill's fetch output (reused)
        # every partition's spill state as arrays (a spill of thousands of partitions runs no
        # per-partition Python): durable end, logical bytes, first byte of the open segment file
        # and its descriptor (-1: none open); the record positions of each spill are kept per spill
        # and merged into a partition's files object when it is read
        self._files = list(self.parts.values())
        self._chunks = []   # per spill: (local indices, run starts in pos, counts, bytes before, pos)
        self._merged = np.zeros(len(self._files), np.int64)  # chunks merged into each files object
        for k, f in enumerate(self._files):
            f._owner, f._li = self, k
        self._end = np.fromiter((f.end for f in self._files), np.int64, len(self._files))
        self._total = np.fromiter((int(f.pos[-1]) for f in self._files), np.int64, len(self._files))
        self._segbase = np.fromiter((f.seg_pos[-1] if f.seg_first else -1 for f in self._files), np.int64,
                                    len(self._files))
        self._fd = np.full(len(self._files), -1, np.int64)
        self._limit = int(segment_file_bytes)
        self.phase_s: dict[str, float] = {}
        # `start` (one offset per partition, in `partitions` order): a tier attached to an engine
        # that already holds records begins a partition without files at that offset (its log start:
        # the records below it were never durable and are gone from the ring)
        if start is not None:
            fresh = np.fromiter((not f.seg_first for f in self._files), bool, len(self._files))
            st = np.asarray(start, np.int64).reshape(-1)
            if st.size != len(self._files):
                raise ValueError("start: one offset per partition")
            self._end[fresh] = np.maximum(self._end[fresh], st[fresh])
        # a reopened tier continues where its files end: the replica cursors name that offset
        # (`cursor` only keys the replica reads' position cache; no consumer slot is used)
        pidx = np.fromiter(self.parts, np.uint32, len(self.parts))
        if len(pidx):
            self.engine.set_replica_cursor(pidx, self._end.astype(np.uint64))

    def end(self, p: int) -> int:
        return self.parts[p].end

    def save_vote(self, p: int, term: int, voted_for: int) -> None:
        """Raft's votedFor (and currentTerm) of partition p, durable BEFORE the vote is answered
        (jraft's raft_meta, PartitionRaftServer.java:89): meta.json is replaced (fsync'd when the tier
        fsyncs) so that a replica that restarts cannot vote twice in one term."""
        f = self.parts[int(p)]
        f.save_meta(term, (term, voted_for), self.cursor, self.fsync, led=0)

    def _merge(self, k: int) -> None:
        """The record positions of partition k's spills not merged into its files object yet."""
        m = int(self._merged[k])
        if m == len(self._chunks):
            return
        self._merged[k] = len(self._chunks)
        f = self._files[k]
        f._owner = None  # (add_positions reads its own arrays)
        try:
            for li, starts, counts, before, pos in self._chunks[m:]:
                j = int(np.searchsorted(li, k))
                if j < len(li) and li[j] == k:
                    s0, c = int(starts[j]), int(counts[j])
                    f.add_positions(pos[s0:s0 + c + 1], int(before[j]))
        finally:
            f._owner = self

    def close(self) -> None:
        """Close the open segment files (spill reopens them)."""
        for f in self.parts.values():
            f.close()
        self._fd[:] = -1

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def spill(self) -> int:
        """Make every committed record durable; returns the number of records written. The host
        time of its phases adds up in self.phase_s (fetch, files, commit, state)."""
        t0 = time.perf_counter()
        pidx = np.fromiter(self.parts, np.uint32, len(self.parts))
        if not len(pidx):
            return 0
        cons = np.full(len(pidx), self.cursor, np.uint32)
        mx = np.full(len(pidx), 0xFFFFFFFF, np.uint32)
        # one fetch into a reused buffer (page-locked when the engine offers it), grown when short
        while True:
            if self._buf is not None:
                rc, res, buf, used = self.engine.fetch(pidx, cons, mx, out=self._buf, commit=True, replica=True)
                if rc == A.RMQ_OK:
                    break
                # (RMQ_ENOSPC: the requests that fitted moved their cursors; every one reads again)
                self.engine.set_replica_cursor(pidx, self._end.astype(np.uint64))
            else:
                used = 1 << 20
            need = max(2 * int(used), 1 << 20)
            if hasattr(self.engine, "host_empty"):
                if self._buf is not None:
                    self.engine.host_release(self._buf)
                self._buf = self.engine.host_empty(need, np.uint8)
            else:
                self._buf = np.zeros(need, np.uint8)
        t1 = time.perf_counter()
        status = res["status"].astype(np.int64)
        bad = np.flatnonzero(status != A.RMQ_OK)
        if len(bad):
            p, st = int(pidx[bad[0]]), int(status[bad[0]])
            raise EngineError(st, f"spill of partition {p} (records lost before they were durable)"
                              if st == A.RMQ_EOFFSET else f"spill of partition {p}")
        sel = np.flatnonzero((status == A.RMQ_OK) & (res["count"] > 0))
        moved = 0
        if len(sel):
            ps = pidx[sel]
            first = np.ascontiguousarray(res["start_offset"][sel], np.uint64)
            count = np.ascontiguousarray(res["count"][sel], np.uint64)
            opos = np.ascontiguousarray(res["out_pos"][sel], np.uint64)
            nbytes = np.ascontiguousarray(res["bytes"][sel], np.uint64)
            # (pidx lists the partitions in local order: sel are their local indices, ascending)
            gap = np.flatnonzero((self._segbase[sel] >= 0) & (first.astype(np.int64) != self._end[sel]))
            if len(gap):
                k = int(sel[gap[0]])
                raise EngineError(A.RMQ_EINVAL, f"{self._files[k].dir}: spill of offset {int(first[gap[0]])} "
                                                f"does not continue {int(self._end[k])}")
            # a new segment file where none is open or the open one reached the size limit (rare)
            roll = (self._fd[sel] < 0) | ((self._segbase[sel] >= 0) &
                                          (self._total[sel] - self._segbase[sel] >= self._limit))
            for j in np.flatnonzero(roll).tolist():
                k = int(sel[j])
                f = self._files[k]
                fd, total = f.append_fd(int(first[j]))  # (a partition's first file starts its log)
                self._fd[k], self._segbase[k], self._end[k], self._total[k] = fd, f.seg_pos[-1], f.end, total
            fds = np.ascontiguousarray(self._fd[sel], np.int32)
            before = self._total[sel].copy()
            pos = np.empty(int(count.sum()) + len(sel), np.uint64)
            data = np.ascontiguousarray(buf.view(np.uint8).reshape(-1))
            rc = A.load().rmq_tier_append(len(sel), _ptr(fds), _ptr(first), _ptr(count), _ptr(opos), _ptr(nbytes),
                                          data.ctypes.data, _ptr(pos), 16, 1 if self.fsync else 0)
            if rc:
                # some runs may already be (partly) in their files: cut every file back to its size
                # before the call, so the records the next spill writes again are not doubled. The
                # replica cursors moved with the fetch: put them back to the durable ends too.
                for j in range(len(sel)):
                    os.ftruncate(int(fds[j]), int(before[j] - self._segbase[sel[j]]))
                self.engine.set_replica_cursor(ps, self._end[sel].astype(np.uint64))
                raise EngineError(rc, "spill: segment append (a run does not hold its records, or an I/O error)")
            ends = np.cumsum(count.astype(np.int64) + 1)
            self._chunks.append((sel.astype(np.int64), ends - count.astype(np.int64) - 1, count.astype(np.int64),
                                 before, pos.view(np.int64)))
            self._end[sel] += count.astype(np.int64)
            self._total[sel] += nbytes.astype(np.int64)
            moved = int(count.sum())
            t2 = time.perf_counter()
        else:
            t2 = time.perf_counter()
        t3 = time.perf_counter()
        # offsets and term of the partitions led here (one bulk read of each), then the durable ends
        # of every partition in one file: a reopen trusts the records below them
        rows = self.engine.consumer_table()[pidx]
        t3a = time.perf_counter()
        sts = self.engine.states()[pidx]
        t3b = time.perf_counter()
        if 0 <= self.cursor < rows.shape[1]:
            rows[:, self.cursor] = 0  # (the tier's own slot: the durable end, in the ends file)
        key = np.concatenate([rows, sts["term"][:, None], sts["voted_term"][:, None],
                              sts["voted_for"][:, None].astype(np.uint64), sts["led"][:, None].astype(np.uint64)],
                             axis=1)
        # only the partitions whose row, term or vote changed since the last save (most spills: none);
        # every partition held here, led or followed (a follower's term and vote are its raft_meta)
        changed = np.ones(len(pidx), bool)
        if self._saved is not None:
            changed &= (key != self._saved).any(axis=1)
        for k in np.flatnonzero(changed).tolist():
            p = int(pidx[k])
            self.parts[p].save_state(rows[k], int(sts["term"][k]), self.cursor, self.fsync,
                                     vote=(int(sts["voted_term"][k]), int(sts["voted_for"][k])),
                                     led=int(sts["led"][k]))
        if self._saved is None:
            self._saved = key.copy()
        else:
            self._saved[changed] = key[changed]
        t3c = time.perf_counter()
        ends = np.empty((len(self.parts), 2), np.uint64)
        ends[:, 0] = pidx
        ends[:, 1] = self._end
        tmp = os.path.join(self.dir, ENDS_FILE + ".tmp")
        with open(tmp, "wb") as f:
            f.write(ends.tobytes())
            if self.fsync:
                f.flush()
                os.fsync(f.fileno())
        os.replace(tmp, os.path.join(self.dir, ENDS_FILE))
        t4 = time.perf_counter()
        for k, v in (("fetch", t1 - t0), ("files", t2 - t1), ("commit", t3 - t2), ("table", t3a - t3),
                     ("states", t3b - t3a), ("save", t3c - t3b), ("ends", t4 - t3c)):
            self.phase_s[k] = self.phase_s.get(k, 0.0) + v
        return moved

    def read(self, p: int, off: int, max_messages: int) -> list[tuple[int, int, bytes]]:
        """Records [off, min(off + max, durable end)) of partition p from the files."""
        return split_records(self.read_images(p, off, max_messages)[1])

    def read_images(self, p: int, off: int, max_messages: int) -> tuple[int, bytes]:
        """(count, record images) of [off, min(off + max, durable end)): the FORMAT.md §1 bytes as
        rmq_fetch returns them, one read per segment file touched (a broker forwarding record
        images, as the fetch output, needs no per-record split)."""
        f = self.parts[p]
        end = min(off + max(int(max_messages), 0), f.end)
        if off < f.base or off >= end:
            return 0, b""
        return end - off, f.read_records(off, end)


def replay(directory: str, engine, partitions, *, batch_records: int = 65536) -> dict:
    """Rebuild a fresh engine's logs from segment files: every record is appended again in offset
    order (the engine recomputes its CRC32C) and must get the offset the file holds; afterwards
    the retained window of every partition's lowest local ring must equal the files' bytes for it.
    Then each partition's term (rmq_become_leader) and consumer-offset row come back from its
    meta and offsets files. Returns {"records": n, "partitions": k, "terms": t, "offset_rows": o}."""
    ends = load_ends(directory)
    files = {int(p): _PartitionFiles(directory, int(p), 1 << 62, ends.get(int(p), 0)) for p in partitions}
    recs = {}
    for p, f in files.items():
        if f.end == f.base:
            continue
        st = engine.state(p)
        if st["log_end_offset"] != f.base:
            raise EngineError(A.RMQ_EINVAL, f"replay of partition {p}: log ends at {st['log_end_offset']}, "
                                            f"files start at {f.base}")
        recs[p] = split_records(f.read_records(f.base, f.end))
    # interleave the partitions into batches (any order across partitions keeps per-partition order)
    queue = [(p, k) for p, r in recs.items() for k in range(len(r))]
    queue.sort(key=lambda x: (x[1], x[0]))
    total = 0
    for s in range(0, len(queue), batch_records):
        chunk = queue[s:s + batch_records]
        pidx = np.fromiter((p for p, _ in chunk), np.uint32, len(chunk))
        pays = [recs[p][k][2] for p, k in chunk]
        lens = np.fromiter((len(x) for x in pays), np.uint32, len(chunk))
        payload = np.frombuffer(b"".join(pays) + bytes(16), np.uint8)
        offs, stats = engine.append(pidx, lens, payload)
        want = np.fromiter((recs[p][k][0] for p, k in chunk), np.uint64, len(chunk))
        if stats["appended"] != len(chunk) or not np.array_equal(offs, want):
            raise EngineError(A.RMQ_EINVAL, f"replay: batch at {s} got other offsets than the files hold")
        total += len(chunk)
    if hasattr(engine, "sync"):
        engine.sync()
    for p, f in files.items():
        if p not in recs:
            continue
        st = engine.state(p)
        lo_off = st["log_start_offset"]
        data = f.read_records(lo_off, f.end)
        S = st["segment_bytes"]
        a = st["log_start_pos"] % S
        n = st["log_end_pos"] - st["log_start_pos"]
        r0 = st["leader_slot"]  # the leader's own replica is local
        ring = engine.read_segment(r0, p, a, min(n, S - a)).tobytes()
        if n > S - a:
            ring += engine.read_segment(r0, p, 0, n - (S - a)).tobytes()
        if ring != data:
            raise EngineError(A.RMQ_EINVAL, f"replay of partition {p}: ring bytes differ from the files "
                                            f"(a CRC or payload changed)")
    terms = rows = 0
    for p, f in files.items():
        meta = f.load_meta()
        term = int(meta.get("term", 0))
        vt, vf = int(meta.get("voted_term", 0)), int(meta.get("voted_for", A.RMQ_NO_VOTE))
        led = int(meta.get("led", 1))  # (a meta without the flag came from a leader's spill)
        if led and term > engine.state(p)["term"]:
            engine.become_leader(p, term)
            terms += 1
        if vt > engine.state(p)["voted_term"]:  # a vote newer than any term it led (raft_meta votedFor):
            engine.set_vote(p, vt, vf)          # restored as a vote, never as a leadership
            terms += 0 if led else 1
        raw = f.load_offsets_bytes()
        if raw:
            offs = np.frombuffer(raw, np.uint64).copy()
            n = min(len(offs), engine.cfg.max_consumers)
            rc, st = engine.commit_consumer_offset(np.full(n, p, np.uint32), np.arange(n, dtype=np.uint32), offs[:n])
            if rc:
                raise EngineError(rc, f"replay of partition {p}: consumer offsets")
            rows += 1
    return {"records": total, "partitions": len(recs), "terms": terms, "offset_rows": rows}
