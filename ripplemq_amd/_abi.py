"""ctypes mirror of include/ripplemq_engine.h (the C-ABI drop-in boundary).

Only plain pointers and sizes cross the boundary. This module loads the in-tree
``libripplemq_engine.so`` and declares the argument/return types of every exported symbol.
It never falls back to anything: if the library is missing, loading raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HEADER = os.path.join(REPO, "include", "ripplemq_engine.h")
LIB_PATH = os.environ.get("RMQ_LIB") or os.path.join(HERE, "libripplemq_engine.so")

RMQ_ABI_VERSION = 10
RMQ_FETCH_COMMIT = 1
RMQ_FETCH_REPLICA = 2
RMQ_FETCH_PINNED_ROWS = 0x100
RMQ_FETCH_DEVICE_ROWS = 0x200
RMQ_MAX_RF = 8
RMQ_ALL_PARTITIONS = 0xFFFFFFFF
RMQ_OFFSET_NONE = 0xFFFFFFFFFFFFFFFF
RMQ_RECORD_HEADER_BYTES = 16
RMQ_TICKET_OFFSETS = 1 << 63
RMQ_SCAN_CHECK = 1

RMQ_OK = 0
RMQ_PENDING = 1
RMQ_ENOTLEADER = -1
RMQ_ENOPART = -2
RMQ_EINVAL = -3
RMQ_ENOSPC = -4
RMQ_EDEVICE = -5
RMQ_EOFFSET = -6
RMQ_ENOMEM = -7
RMQ_ESTALE = -8
RMQ_ETERM = -9
RMQ_NO_VOTE = 0xFFFFFFFF

RMQ_MEM_HOST = 0
RMQ_MEM_DEVICE = 1
RMQ_MEM_PINNED = 2

STATUS_NAMES = {
    RMQ_OK: "RMQ_OK", RMQ_PENDING: "RMQ_PENDING", RMQ_ENOTLEADER: "RMQ_ENOTLEADER",
    RMQ_ENOPART: "RMQ_ENOPART", RMQ_EINVAL: "RMQ_EINVAL", RMQ_ENOSPC: "RMQ_ENOSPC",
    RMQ_EDEVICE: "RMQ_EDEVICE", RMQ_EOFFSET: "RMQ_EOFFSET", RMQ_ENOMEM: "RMQ_ENOMEM",
    RMQ_ESTALE: "RMQ_ESTALE", RMQ_ETERM: "RMQ_ETERM",
}

u32 = C.c_uint32
u64 = C.c_uint64
i32 = C.c_int32
vp = C.c_void_p


class RmqConfig(C.Structure):
    _fields_ = [
        ("num_partitions", u32), ("replication_factor", u32), ("segment_bytes", u64),
        ("index_interval", u32), ("max_consumers", u32), ("max_batch_records", u32),
        ("pipeline_depth", u32), ("max_batch_bytes", u64), ("device", i32), ("rank", u32),
        ("pool_bytes", u64),
    ]


class RmqBatch(C.Structure):
    _fields_ = [
        ("n", u32), ("mem", u32), ("pidx", vp), ("len", vp), ("payload_off", vp),
        ("payload", vp), ("payload_bytes", u64),
    ]


class RmqFetchReq(C.Structure):
    _fields_ = [("pidx", u32), ("consumer", u32), ("max_records", u32), ("reserved", u32)]


class RmqFetchRes(C.Structure):
    _fields_ = [
        ("start_offset", u64), ("out_pos", u64), ("count", u32), ("bytes", u32),
        ("status", i32), ("reserved", u32),
    ]


class RmqPartitionState(C.Structure):
    _fields_ = [
        ("log_end_offset", u64), ("log_end_pos", u64), ("log_start_offset", u64),
        ("log_start_pos", u64), ("commit", u64), ("high_watermark", u64), ("term", u64),
        ("term_start", u64), ("match", u64 * RMQ_MAX_RF), ("replica_rank", u32 * RMQ_MAX_RF),
        ("leader_slot", u32), ("is_leader", u32), ("segment_bytes", u64), ("leader_commit", u64),
        ("last_log_term", u64), ("voted_term", u64), ("voted_for", u32), ("led", u32), ("heard_round", u64),
    ]


class RmqReplStats(C.Structure):
    _fields_ = [
        ("world", u32), ("rank", u32), ("out_entries", u32), ("in_entries", u32), ("rounds", u64),
        ("bytes_sent", u64), ("bytes_received", u64), ("records_ingested", u64), ("refused_crc", u64),
        ("refused_log", u64), ("bytes_ingested", u64), ("catchup_entries", u64), ("detached_plans", u64),
        ("general_plans", u64), ("host_waits", u64), ("host_wait_ns", u64),
    ]


class RmqAppendStats(C.Structure):
    _fields_ = [
        ("records", u32), ("appended", u32), ("rejected_not_leader", u32),
        ("rejected_no_partition", u32), ("rejected_no_space", u32), ("rejected_invalid", u32),
    ]


def header_symbols(path: str = HEADER) -> list[str]:
    """Every function the public header declares (the drop-in surface)."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rmq_\w+)\s*\(", text, re.M)))


_SIGS = {
    "rmq_abi_version": (u32, []),
    "rmq_strerror": (C.c_char_p, [C.c_int]),
    "rmq_config_default": (None, [C.POINTER(RmqConfig), u32, u32]),
    "rmq_create": (C.c_int, [C.POINTER(RmqConfig), C.POINTER(vp)]),
    "rmq_destroy": (None, [vp]),
    "rmq_set_replicas": (C.c_int, [vp, u32, C.POINTER(u32), u32, u32]),
    "rmq_become_leader": (C.c_int, [vp, u32, u64]),
    "rmq_vote": (C.c_int, [vp, u32, u64, u32, u64, u64, C.POINTER(u32)]),
    "rmq_set_vote": (C.c_int, [vp, u32, u64, u32]),
    "rmq_leader_silent": (C.c_int, [vp, u32, u32, vp, u32, C.POINTER(u32)]),
    "rmq_set_segments": (C.c_int, [vp, u32, C.POINTER(u32), C.POINTER(u64)]),
    "rmq_append": (C.c_int, [vp, C.POINTER(RmqBatch), vp, C.POINTER(u64)]),
    "rmq_ack": (C.c_int, [vp, vp, vp, vp, u32]),
    "rmq_poll_commit": (C.c_int, [vp, u64, vp, vp]),
    "rmq_ticket_stats": (C.c_int, [vp, u64, C.POINTER(RmqAppendStats)]),
    "rmq_sync": (C.c_int, [vp]),
    "rmq_commit_consumer_offset": (C.c_int, [vp, vp, vp, vp, u32, vp, C.POINTER(u64)]),
    "rmq_set_replica_cursor": (C.c_int, [vp, u32, vp, vp]),
    "rmq_fetch": (C.c_int, [vp, vp, u32, u32, vp, u64, vp, C.POINTER(u64)]),
    "rmq_fetch_async": (C.c_int, [vp, vp, u32, u32, vp, u64, vp, C.POINTER(u64)]),
    "rmq_fetch_poll": (C.c_int, [vp, u64, u32, C.POINTER(u64)]),
    "rmq_get_partition_state": (C.c_int, [vp, u32, C.POINTER(RmqPartitionState)]),
    "rmq_get_partition_states": (C.c_int, [vp, u32, u32, vp]),
    "rmq_read_segment": (C.c_int, [vp, u32, u32, u64, u64, vp]),
    "rmq_read_index": (C.c_int, [vp, u32, u64, u64, vp]),
    "rmq_read_consumer_offsets": (C.c_int, [vp, u32, vp]),
    "rmq_read_consumer_table": (C.c_int, [vp, u32, u32, vp]),
    "rmq_device_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
    "rmq_device_free": (C.c_int, [vp, vp]),
    "rmq_memcpy": (C.c_int, [vp, vp, vp, u64, C.c_int]),
    "rmq_host_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
    "rmq_host_free": (C.c_int, [vp, vp]),
    "rmq_host_register": (C.c_int, [vp, vp, u64]),
    "rmq_host_unregister": (C.c_int, [vp, vp]),
    "rmq_profile_enable": (C.c_int, [vp, C.c_int]),
    "rmq_profile_query": (C.c_int, [vp, C.c_int, C.POINTER(u64), C.POINTER(C.c_double)]),
    "rmq_device_info": (C.c_int, [vp, C.c_char_p, u32, C.POINTER(u32)]),
    "rmq_set_placement": (C.c_int, [vp, u32, vp, vp, vp, vp]),
    "rmq_rccl_unique_id": (C.c_int, [vp]),
    "rmq_attach_rccl": (C.c_int, [vp, vp, u32]),
    "rmq_local_hub_create": (C.c_int, [u32, C.POINTER(vp)]),
    "rmq_local_hub_destroy": (None, [vp]),
    "rmq_attach_local": (C.c_int, [vp, vp]),
    "rmq_replication_stats": (C.c_int, [vp, C.POINTER(RmqReplStats)]),
    "rmq_read_outbox": (C.c_int, [vp, u32, vp, u64, C.POINTER(u64)]),
    "rmq_fault_drop_rounds": (C.c_int, [vp, u32]),
    "rmq_fault_corrupt": (C.c_int, [vp, u32, C.c_int64]),
    "rmq_fault_isolate": (C.c_int, [vp, u32, u32]),
    "rmq_fault_cut": (C.c_int, [vp, u32, u32]),
    "rmq_scan_records": (C.c_int, [vp, u64, u64, u64, u32, vp, C.POINTER(u64), C.POINTER(u64)]),
    "rmq_tier_append": (C.c_int, [u32, vp, vp, vp, vp, vp, vp, vp, u32, C.c_int]),
}

_lib = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load the engine library (raises OSError if it was not built)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"ripplemq engine library not built: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rmq_abi_version() != RMQ_ABI_VERSION:
        raise OSError("ripplemq ABI version mismatch")
    if path == LIB_PATH:
        _lib = lib
    return lib
