"""ripplemq_amd — MI355X-native engine for RippleMQ's Partition-Raft append / commit / fetch path.

The product is the C-ABI library ``libripplemq_engine.so`` (include/ripplemq_engine.h, HIP kernels
in csrc/). This package is host glue: ctypes bindings (``_abi``), a numpy handle (``engine``), the
reference-shaped state-machine facade (``state_machine``) and synthetic workloads (``workload``).
"""
from .engine import Engine, EngineConfig, EngineError, parse_records  # noqa: F401

__all__ = ["Engine", "EngineConfig", "EngineError", "parse_records"]
