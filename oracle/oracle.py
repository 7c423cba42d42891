"""ctypes handle over the C oracle (oracle/libripple_oracle.so) — TEST INFRASTRUCTURE ONLY.

Same method names and return shapes as ripplemq_amd.engine.Engine so a parity test can run one
scenario through both and compare everything. Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; the product package never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from ripplemq_amd import _abi as A
from ripplemq_amd.engine import FETCH_RES_DTYPE, STATE_DTYPE, EngineConfig, EngineError, state_to_dict

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libripple_oracle.so")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
    sigs = {
        "ro_crc32c_bitwise": (u32, [vp, C.c_size_t]),
        "ro_crc32c": (u32, [vp, C.c_size_t]),
        "ro_crc32c_hw_available": (C.c_int, []),
        "ro_create": (vp, [C.POINTER(A.RmqConfig)]),
        "ro_destroy": (None, [vp]),
        "ro_set_replicas": (C.c_int, [vp, u32, vp, u32, u32]),
        "ro_become_leader": (C.c_int, [vp, u32, u64]),
        "ro_append": (C.c_int, [vp, u32, vp, vp, vp, vp, u64, vp, C.POINTER(A.RmqAppendStats)]),
        "ro_ack": (C.c_int, [vp, vp, vp, vp, u32]),
        "ro_commit_consumer_offset": (C.c_int, [vp, vp, vp, vp, u32, vp]),
        "ro_fetch": (C.c_int, [vp, vp, u32, vp, u64, vp, C.POINTER(u64)]),
        "ro_set_replica_cursor": (C.c_int, [vp, u32, vp, vp]),
        "ro_get_partition_state": (C.c_int, [vp, u32, C.POINTER(A.RmqPartitionState)]),
        "ro_get_partition_states": (C.c_int, [vp, u32, u32, vp]),
        "ro_commit_notice": (C.c_int, [vp, u32, vp]),
        "ro_apply_notice": (C.c_int, [vp, u32, vp, u32]),
        "ro_offset_quorum": (C.c_int, [vp, u32, C.POINTER(u64), C.POINTER(u64)]),
        "ro_read_segment": (C.c_int, [vp, u32, u32, u64, u64, vp]),
        "ro_read_index": (C.c_int, [vp, u32, u64, u64, vp]),
        "ro_read_consumer_offsets": (C.c_int, [vp, u32, vp]),
        "ro_record_pos": (C.c_int, [vp, u32, u64, C.POINTER(u64)]),
        "ro_append_sharded": (C.c_int, [vp, u32, vp, vp, vp, u32, C.c_int, C.POINTER(u32)]),
        "ro_reserve": (C.c_int, [vp, vp]),
        "ro_set_world": (C.c_int, [vp, u32]),
        "ro_set_key": (C.c_int, [vp, u32, u64]),
        "ro_round_region": (C.c_int, [vp, u32, vp, u64, C.POINTER(u64)]),
        "ro_end_round": (None, [vp]),
        "ro_ingest": (C.c_int, [vp, u32, vp, u64, vp]),
        "ro_apply_acks": (C.c_int, [vp, u32, vp, u32, u64]),
        "ro_round_no": (u64, [vp]),
        "ro_catchup_reserve": (u64, [C.POINTER(A.RmqConfig)]),
        "ro_pair_entries": (u32, [vp, u32, u32]),
        "ro_counters": (None, [vp, vp]),
        "ro_set_segments": (C.c_int, [vp, u32, vp, vp]),
        "ro_vote": (C.c_int, [vp, u32, u64, u32, u64, u64, C.POINTER(u32)]),
        "ro_set_vote": (C.c_int, [vp, u32, u64, u32]),
        "ro_leader_silent": (C.c_int, [vp, u32, vp, u32, C.POINTER(u32)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def crc32c(data: bytes, bitwise: bool = False) -> int:
    lib = load()
    buf = (C.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
    fn = lib.ro_crc32c_bitwise if bitwise else lib.ro_crc32c
    return int(fn(buf, len(data)))


def _p(a):
    return None if a is None else a.ctypes.data


class OracleEngine:
    """Sequential CPU restatement with the Engine's Python surface."""

    def __init__(self, cfg: EngineConfig):
        self.lib = load()
        self.cfg = cfg
        c = cfg.to_c()
        self.h = self.lib.ro_create(C.byref(c))
        if not self.h:
            raise ValueError("invalid oracle config")
        self.last_offset_ticket = 0
        self._tseq = 0
        self._tickets: dict[int, list[tuple[int, int]]] = {}

    def close(self):
        if self.h:
            self.lib.ro_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_replicas(self, pidx, ranks, leader_slot):
        r = (C.c_uint32 * len(ranks))(*ranks)
        rc = self.lib.ro_set_replicas(self.h, pidx, r, len(ranks), leader_slot)
        if rc:
            raise EngineError(rc, "oracle")

    def set_placement(self, pidx, keys, ranks, leader_slot):
        ranks = np.asarray(ranks).reshape(len(pidx), self.cfg.replication_factor)
        for i, p in enumerate(pidx):
            self.set_replicas(int(p), [int(x) for x in ranks[i]], int(leader_slot[i]))
            if keys is not None:
                self.lib.ro_set_key(self.h, int(p), int(keys[i]))

    # ---- replication rounds (FORMAT.md §9)
    def set_world(self, world):
        if self.lib.ro_set_world(self.h, world):
            raise EngineError(A.RMQ_EINVAL, "oracle")

    def round_region(self, dst) -> np.ndarray:
        n = C.c_uint64()
        self.lib.ro_round_region(self.h, dst, None, 0, C.byref(n))
        out = np.zeros(max(int(n.value), 1), np.uint8)
        rc = self.lib.ro_round_region(self.h, dst, _p(out), out.size, C.byref(n))
        if rc:
            raise EngineError(rc, "oracle")
        return out[:int(n.value)]

    def end_round(self):
        self.lib.ro_end_round(self.h)

    def pair_entries(self, src, dst) -> int:
        return int(self.lib.ro_pair_entries(self.h, src, dst))

    def ingest(self, src, region) -> np.ndarray:
        """FORMAT.md §9 acks, [n][2] {log end offset | status << 62, log end position}."""
        region = np.ascontiguousarray(region, np.uint8)
        n = self.pair_entries(src, self.cfg.rank)
        acks = np.zeros((max(n, 1), 2), np.uint64)
        rc = self.lib.ro_ingest(self.h, src, _p(region) if region.size else None, region.size, _p(acks))
        if rc:
            raise EngineError(rc, "oracle ingest")
        return acks[:n]

    def commit_notice(self, dst) -> np.ndarray:
        """FORMAT.md §9 v4 commit notices for the pair (me -> dst): [n][2] {commit, term}."""
        n = self.pair_entries(self.cfg.rank, dst)
        out = np.zeros((max(n, 1), 2), np.uint64)
        rc = self.lib.ro_commit_notice(self.h, dst, _p(out))
        if rc:
            raise EngineError(rc, "oracle commit_notice")
        return out[:n]

    def apply_notice(self, src, notices):
        notices = np.ascontiguousarray(notices, np.uint64).reshape(-1, 2)
        rc = self.lib.ro_apply_notice(self.h, src, _p(notices) if notices.size else None, len(notices))
        if rc:
            raise EngineError(rc, "oracle apply_notice")

    def apply_acks(self, dst, acks, round_no):
        acks = np.ascontiguousarray(acks, np.uint64).reshape(-1, 2)
        rc = self.lib.ro_apply_acks(self.h, dst, _p(acks) if acks.size else None, len(acks), round_no)
        if rc:
            raise EngineError(rc, "oracle apply_acks")

    def round_no(self) -> int:
        return int(self.lib.ro_round_no(self.h))

    def catchup_reserve(self) -> int:
        c = self.cfg.to_c()
        return int(self.lib.ro_catchup_reserve(C.byref(c)))

    def counters(self) -> np.ndarray:
        """[0] records ingested, [1] entries refused (CRC), [2] refused (log / term / missed),
        [3] bytes ingested, [4] catch-up entries sent, [5] detached entry plans."""
        out = np.zeros(6, np.uint64)
        self.lib.ro_counters(self.h, _p(out))
        return out

    def become_leader(self, pidx, term):
        rc = self.lib.ro_become_leader(self.h, pidx, term)
        if rc:
            raise EngineError(rc, "oracle")

    def vote(self, pidx, term, candidate, cand_last_log_term, cand_log_end) -> bool:
        g = C.c_uint32(0)
        rc = self.lib.ro_vote(self.h, pidx, term, candidate, cand_last_log_term, cand_log_end, C.byref(g))
        if rc:
            raise EngineError(rc, "oracle")
        return bool(g.value)

    def set_vote(self, pidx, term, voted_for):
        rc = self.lib.ro_set_vote(self.h, pidx, term, voted_for)
        if rc:
            raise EngineError(rc, "oracle")

    def leader_silent(self, silent_rounds: int, timeout_ms: int = 0) -> np.ndarray:
        """Followed partitions whose leader was silent for silent_rounds rounds (the oracle keeps no
        wall clock: timeout_ms is not modelled)."""
        n = C.c_uint32(0)
        self.lib.ro_leader_silent(self.h, silent_rounds, None, 0, C.byref(n))
        out = np.zeros(max(n.value, 1), np.uint32)
        self.lib.ro_leader_silent(self.h, silent_rounds, _p(out), n.value, C.byref(n))
        return out[:n.value]

    def append(self, pidx, lens, payload, payload_off=None):
        pidx = np.ascontiguousarray(pidx, np.uint32)
        lens = np.ascontiguousarray(lens, np.uint32)
        payload = np.ascontiguousarray(payload, np.uint8)
        if payload_off is not None:
            payload_off = np.ascontiguousarray(payload_off, np.uint64)
        out = np.empty(len(pidx), np.uint64)
        st = A.RmqAppendStats()
        rc = self.lib.ro_append(self.h, len(pidx), _p(pidx), _p(lens), _p(payload_off),
                                _p(payload) if payload.size else None, payload.size, _p(out), C.byref(st))
        if rc:
            raise EngineError(rc, "oracle")
        return out, {f: int(getattr(st, f)) for f, _ in A.RmqAppendStats._fields_}

    def append_sharded(self, batches, threads, pin=True):
        """ro_append_sharded over a list of workload Batches (bench.py's multi-core CPU baseline).
        Returns [(out_offsets, stats)] per batch, like append()."""
        nb = len(batches)
        keep, outs = [], []
        arr = (A.RmqBatch * max(nb, 1))()
        for k, b in enumerate(batches):
            pidx = np.ascontiguousarray(b.pidx, np.uint32)
            lens = np.ascontiguousarray(b.lens, np.uint32)
            pay = np.ascontiguousarray(b.payload, np.uint8)
            keep += [pidx, lens, pay]
            arr[k] = A.RmqBatch(len(pidx), A.RMQ_MEM_HOST, _p(pidx), _p(lens), None,
                                _p(pay) if pay.size else None, pay.size)
            outs.append(np.empty(len(pidx), np.uint64))
        optr = (C.c_void_p * max(nb, 1))(*[o.ctypes.data for o in outs])
        st = (A.RmqAppendStats * max(nb, 1))()
        done = C.c_uint32()
        rc = self.lib.ro_append_sharded(self.h, nb, arr, optr, st, threads, int(pin), C.byref(done))
        if rc:
            raise EngineError(rc, "oracle")
        return [(outs[k], {f: int(getattr(st[k], f)) for f, _ in A.RmqAppendStats._fields_}) for k in range(nb)]

    def reserve(self, bytes_per_partition):
        b = np.ascontiguousarray(bytes_per_partition, np.uint64)
        rc = self.lib.ro_reserve(self.h, _p(b))
        if rc:
            raise EngineError(rc, "oracle")

    def ack(self, pidx, slot, match):
        pidx = np.ascontiguousarray(pidx, np.uint32)
        slot = np.ascontiguousarray(slot, np.uint32)
        match = np.ascontiguousarray(match, np.uint64)
        rc = self.lib.ro_ack(self.h, _p(pidx), _p(slot), _p(match), len(pidx))
        if rc:
            raise EngineError(rc, "oracle")

    def commit_consumer_offset(self, pidx, consumer, offset):
        pidx = np.ascontiguousarray(pidx, np.uint32)
        consumer = np.ascontiguousarray(consumer, np.uint32)
        offset = np.ascontiguousarray(offset, np.uint64)
        status = np.zeros(len(pidx), np.int32)
        rc = self.lib.ro_commit_consumer_offset(self.h, _p(pidx), _p(consumer), _p(offset), len(pidx), _p(status))
        # the engine's consumer-offset ticket: the accepted partitions at their new row versions
        parts = sorted(set(int(x) for x in pidx[status == 0]))
        self.last_offset_ticket = 0
        if parts:
            self._tseq += 1
            self.last_offset_ticket = A.RMQ_TICKET_OFFSETS | self._tseq
            self._tickets[self.last_offset_ticket] = [(p, self.offset_quorum(p)[0]) for p in parts]
        return rc, status

    def offset_quorum(self, p) -> tuple[int, int]:
        """(row version, newest version a quorum holds) of partition p (FORMAT.md §8)."""
        v, q = C.c_uint64(), C.c_uint64()
        rc = self.lib.ro_offset_quorum(self.h, int(p), C.byref(v), C.byref(q))
        if rc:
            raise EngineError(rc, "oracle offset_quorum")
        return int(v.value), int(q.value)

    def poll_offsets(self, ticket) -> int:
        """As rmq_poll_commit of a consumer-offset ticket: RMQ_OK once every partition's row is on a
        quorum at the ticket's version, RMQ_ENOTLEADER if leadership moved first, else RMQ_PENDING."""
        want = self._tickets[ticket]
        done = all(self.offset_quorum(p)[1] >= v for p, v in want)
        lost = not done and any(self.offset_quorum(p)[1] < v and not self.state(p)["is_leader"] for p, v in want)
        if not done and not lost:
            return A.RMQ_PENDING
        del self._tickets[ticket]
        return A.RMQ_OK if done else A.RMQ_ENOTLEADER

    def set_replica_cursor(self, pidx, offset):
        pidx = np.ascontiguousarray(pidx, np.uint32)
        offset = np.ascontiguousarray(offset, np.uint64)
        rc = self.lib.ro_set_replica_cursor(self.h, len(pidx), _p(pidx), _p(offset))
        if rc:
            raise EngineError(rc, "oracle set_replica_cursor")

    def fetch(self, pidx, consumer, max_records, out_cap=None, commit=False, out=None, replica=False):
        n = len(pidx)
        req = np.zeros((n, 4), np.uint32)
        req[:, 0], req[:, 1], req[:, 2] = pidx, consumer, max_records
        req[:, 3] = A.RMQ_FETCH_REPLICA if replica else 0
        res = np.zeros(n, FETCH_RES_DTYPE)
        used = C.c_uint64()
        if out is not None:  # the caller's buffer (as Engine.fetch)
            if commit:
                req[:, 3] |= A.RMQ_FETCH_COMMIT
            rc = self.lib.ro_fetch(self.h, _p(req), n, _p(out), out.size, _p(res), C.byref(used))
            return rc, res, out, int(used.value)
        if out_cap is None:  # the size query commits nothing
            self.lib.ro_fetch(self.h, _p(req), n, None, 0, _p(res), C.byref(used))
            out_cap = int(used.value)
        if commit:
            req[:, 3] |= A.RMQ_FETCH_COMMIT
        out = np.zeros(max(out_cap, 1), np.uint8)
        rc = self.lib.ro_fetch(self.h, _p(req), n, _p(out), out_cap, _p(res), C.byref(used))
        return rc, res, out[:out_cap], int(used.value)

    def state(self, pidx):
        s = A.RmqPartitionState()
        rc = self.lib.ro_get_partition_state(self.h, pidx, C.byref(s))
        if rc:
            raise EngineError(rc, "oracle")
        return state_to_dict(s, self.cfg.replication_factor)

    def states(self, first=0, n=None):
        n = self.cfg.num_partitions - first if n is None else n
        out = np.zeros(n, STATE_DTYPE)
        rc = self.lib.ro_get_partition_states(self.h, first, n, _p(out))
        if rc:
            raise EngineError(rc, "oracle")
        return out

    def commit_snapshot(self):
        return np.array([self.state(p)["commit"] for p in range(self.cfg.num_partitions)], np.uint64)

    def set_segments(self, pidx, segment_bytes):
        p = np.ascontiguousarray(pidx, np.uint32)
        sb = np.ascontiguousarray(segment_bytes, np.uint64)
        rc = self.lib.ro_set_segments(self.h, len(p), _p(p), _p(sb))
        if rc:
            raise EngineError(rc, "oracle")

    def read_segment(self, replica, pidx, ring_off=0, n=None):
        n = self.state(pidx)["segment_bytes"] - ring_off if n is None else n
        out = np.empty(n, np.uint8)
        rc = self.lib.ro_read_segment(self.h, replica, pidx, ring_off, n, _p(out))
        if rc:
            raise EngineError(rc, "oracle")
        return out

    def read_index(self, pidx, m_first, count):
        out = np.empty((count, 2), np.uint64)
        rc = self.lib.ro_read_index(self.h, pidx, m_first, count, _p(out))
        if rc:
            raise EngineError(rc, "oracle")
        return out

    def consumer_table(self, first=0, n=None):
        n = self.cfg.num_partitions - first if n is None else n
        return np.stack([self.consumer_offsets(first + i) for i in range(n)]) if n else \
            np.zeros((0, self.cfg.max_consumers), np.uint64)

    def consumer_offsets(self, pidx):
        out = np.empty(self.cfg.max_consumers, np.uint64)
        self.lib.ro_read_consumer_offsets(self.h, pidx, _p(out))
        return out

    def record_pos(self, pidx, offset):
        v = C.c_uint64()
        rc = self.lib.ro_record_pos(self.h, pidx, offset, C.byref(v))
        if rc:
            raise EngineError(rc, "oracle")
        return int(v.value)
