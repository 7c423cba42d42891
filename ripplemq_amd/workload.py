"""Deterministic synthetic record streams for the BASELINE.json configurations.

Partition selection modes:
  rr       pid = counter % P — RoundRobinSelector.selectPartition's abs(counter++) % n
           (mq-common/src/main/java/partition/selector/RoundRobinSelector.java:26), the counter
           continuing across batches;
  uniform  pid uniform over [0, P);
  zipf     rank ~ Zipf(s) over P ranks, pid = a fixed random permutation of the ranks.
Payload sizes: fixed L, or log-uniform in [lo, hi]. Payload bytes are random.
Seed = 0x52495050 ("RIPP") + config index; batch b of a stream uses stream key (seed, b).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SEED = 0x52495050


@dataclass(frozen=True)
class StreamSpec:
    partitions: int
    records: int            # per batch
    mode: str = "uniform"   # rr | uniform | zipf
    zipf_s: float = 1.1
    size: int | tuple[int, int] = 100
    config_index: int = 1
    invalid_frac: float = 0.0  # fraction of records aimed at pidx >= P (rejection paths)


@dataclass
class Batch:
    pidx: np.ndarray     # u32 [n]
    lens: np.ndarray     # u32 [n]
    payload: np.ndarray  # u8 [sum(lens)] packed

    @property
    def n(self) -> int:
        return len(self.pidx)

    def payload_offsets(self) -> np.ndarray:
        off = np.zeros(self.n, np.uint64)
        if self.n:
            np.cumsum(self.lens[:-1], dtype=np.uint64, out=off[1:])
        return off


def _rng(spec: StreamSpec, b: int) -> np.random.Generator:
    return np.random.Generator(np.random.Philox(key=[SEED + spec.config_index, b]))


_ZIPF_CACHE: dict = {}


def _zipf_table(spec: StreamSpec):
    key = (spec.partitions, spec.zipf_s, spec.config_index)
    if key not in _ZIPF_CACHE:
        g = np.random.Generator(np.random.Philox(key=[SEED + spec.config_index, 0xFFFFFFFF]))
        w = 1.0 / np.arange(1, spec.partitions + 1, dtype=np.float64) ** spec.zipf_s
        cdf = np.cumsum(w)
        cdf /= cdf[-1]
        perm = g.permutation(spec.partitions).astype(np.uint32)
        _ZIPF_CACHE[key] = (cdf, perm)
    return _ZIPF_CACHE[key]


def make_batch(spec: StreamSpec, b: int) -> Batch:
    g = _rng(spec, b)
    n, P = spec.records, spec.partitions
    if spec.mode == "rr":
        pidx = ((np.arange(n, dtype=np.uint64) + np.uint64(b) * np.uint64(n)) % np.uint64(P)).astype(np.uint32)
    elif spec.mode == "uniform":
        pidx = g.integers(0, P, n, dtype=np.uint32)
    elif spec.mode == "zipf":
        cdf, perm = _zipf_table(spec)
        ranks = np.searchsorted(cdf, g.random(n), side="right")
        pidx = perm[np.minimum(ranks, P - 1)]
    else:
        raise ValueError(spec.mode)
    if spec.invalid_frac > 0:
        bad = g.random(n) < spec.invalid_frac
        pidx = np.where(bad, P + g.integers(0, 7, n, dtype=np.uint32), pidx).astype(np.uint32)
    if isinstance(spec.size, tuple):
        lo, hi = spec.size
        # log-uniform over [lo, hi] (shifted by one so that lo = 0 is allowed)
        lens = np.exp(g.uniform(np.log(lo + 1), np.log(hi + 2), n)) - 1
        lens = np.clip(lens.astype(np.int64), lo, hi).astype(np.uint32)
    else:
        lens = np.full(n, spec.size, np.uint32)
    payload = g.integers(0, 256, int(lens.sum(dtype=np.uint64)), dtype=np.uint8)
    return Batch(pidx.astype(np.uint32), lens, payload)


def record_bytes(lens: np.ndarray) -> int:
    """Sum of FORMAT.md record sizes (16-byte header + payload padded to 16)."""
    return int((16 + ((lens.astype(np.uint64) + 15) & ~np.uint64(15))).sum())


# BASELINE.json configs[1..4] as stream specs (configs[0] is the Java docker plumbing run).
CONFIGS = {
    "A": StreamSpec(partitions=256, records=65536, mode="rr", size=100, config_index=1),
    "B": StreamSpec(partitions=4096, records=65536, mode="zipf", zipf_s=1.1, size=100, config_index=2),
    "C": StreamSpec(partitions=4096, records=65536, mode="uniform", size=100, config_index=3),
    "D": StreamSpec(partitions=4096, records=4096, mode="uniform", size=(64, 16384), config_index=4),
}
