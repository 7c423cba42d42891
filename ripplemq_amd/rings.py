"""Ring sizing for the shared segment pool (rmq_config.pool_bytes + rmq_set_segments, FORMAT.md §2).

The reference keeps one unbounded log per partition (PartitionStateMachine's in-memory list,
mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java); here every (replica, partition)
log is a power-of-two ring carved out of one pool per replica region, so HBM goes where the traffic
is. A broker sizes each partition's ring from its measured append traffic:

    ring(p) = pow2ceil(max(min_bytes,
                           retain_batches * mean bytes of p per batch,
                           2 * (largest batch bytes of p + index interval)))   # no-space rule, §4

capped at max_bytes. `pool_layout` then gives the pool size for an engine created with
segment_bytes = the first-ring size (every partition starts in such a block at p * segment_bytes)
that grows the larger rings with one rmq_set_segments call, largest first (the pool's bump
allocator then aligns each block without gaps after the first).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def pow2ceil(x: np.ndarray) -> np.ndarray:
    x = np.maximum(np.asarray(x, np.float64), 1.0)
    return (2.0 ** np.ceil(np.log2(x))).astype(np.uint64)


def partition_traffic(batches, num_partitions: int) -> tuple[np.ndarray, np.ndarray]:
    """(mean, max) FORMAT.md record bytes (16-byte header + payload padded to 16) per partition per
    batch over `batches` (objects with .pidx and .lens); out-of-range partition ids are ignored."""
    acc = np.zeros((len(batches), num_partitions), np.float64)
    for i, b in enumerate(batches):
        ok = b.pidx < num_partitions
        rb = 16 + (b.lens[ok].astype(np.int64) + 15) // 16 * 16
        acc[i] = np.bincount(b.pidx[ok], weights=rb, minlength=num_partitions)
    return acc.mean(axis=0), acc.max(axis=0)


def ring_sizes(mean: np.ndarray, peak: np.ndarray, retain_batches: float, min_bytes: int,
               index_interval: int, max_bytes: int = 1 << 40) -> np.ndarray:
    need = np.maximum(retain_batches * np.asarray(mean, np.float64),
                      2.0 * (np.asarray(peak, np.float64) + index_interval))
    return np.minimum(np.maximum(pow2ceil(need), np.uint64(min_bytes)), np.uint64(max_bytes))


@dataclass
class PoolLayout:
    segment_bytes: int       # every partition's first ring (rmq_config.segment_bytes)
    pool_bytes: int          # per replica region (rmq_config.pool_bytes)
    grown: np.ndarray        # u32 partition ids to grow, largest ring first
    grown_bytes: np.ndarray  # u64 their ring bytes (rmq_set_segments arguments)
    free_bytes: int          # min blocks left behind by the grown partitions (not coalesced)


def pool_layout(sizes: np.ndarray, min_bytes: int | None = None) -> PoolLayout:
    """Layout for rings of at least `sizes` bytes; with min_bytes None, the first-ring size (one of
    the sizes) that needs the smallest pool (partitions below it keep the larger first ring)."""
    sizes = np.asarray(sizes, np.uint64)
    if min_bytes is None:
        outs = [pool_layout(np.maximum(sizes, c), int(c)) for c in np.unique(sizes)]
        return min(outs, key=lambda o: o.pool_bytes)
    P = sizes.size
    grown = np.flatnonzero(sizes > min_bytes)
    grown = grown[np.argsort(-sizes[grown].astype(np.int64), kind="stable")].astype(np.uint32)
    bump = P * int(min_bytes)
    for s in sizes[grown].tolist():
        bump = (bump + s - 1) // s * s + s
    return PoolLayout(segment_bytes=int(min_bytes), pool_bytes=max(bump, P * int(min_bytes)), grown=grown,
                      grown_bytes=sizes[grown].astype(np.uint64), free_bytes=int(grown.size) * int(min_bytes))
