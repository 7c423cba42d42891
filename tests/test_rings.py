"""Ring sizing for the shared pool (ripplemq_amd/rings.py): sizes obey the no-space rule of the
traffic they were sized from, and the pool layout holds every ring under the engine's allocator
(restated here: power-of-two blocks aligned to their size, free lists per size, bump pointer —
engine_internal.hpp SegPool)."""
import numpy as np

from ripplemq_amd.rings import partition_traffic, pool_layout, ring_sizes
from ripplemq_amd.workload import CONFIGS, StreamSpec, make_batch


class _Pool:  # the engine's SegPool allocation order
    def __init__(self, size):
        self.size, self.bump, self.free = size, 0, {k: [] for k in range(64)}

    def give(self, off, end):
        while off < end:
            lg = (off & -off).bit_length() - 1 if off else 63
            while (1 << lg) > end - off:
                lg -= 1
            self.free[lg].append(off)
            off += 1 << lg

    def alloc(self, lg):
        for k in range(lg, 64):
            if self.free[k]:
                o = self.free[k].pop()
                for q in range(k, lg, -1):
                    self.free[q - 1].append(o + (1 << (q - 1)))
                return o
        a = (self.bump + (1 << lg) - 1) & ~((1 << lg) - 1)
        if a + (1 << lg) > self.size:
            return None
        self.give(self.bump, a)
        self.bump = a + (1 << lg)
        return a


def _place(sizes, lay):
    pool = _Pool(lay.pool_bytes)
    lg0 = lay.segment_bytes.bit_length() - 1
    blocks = [pool.alloc(lg0) for _ in range(sizes.size)]
    assert None not in blocks
    for p, s in zip(lay.grown.tolist(), lay.grown_bytes.tolist()):
        o = pool.alloc(int(s).bit_length() - 1)
        assert o is not None, "pool too small for the layout"
        pool.free[lg0].append(blocks[p])
        blocks[p] = o
    ends = sorted((b, b + int(max(s, lay.segment_bytes))) for b, s in zip(blocks, sizes.tolist()))
    assert all(e0 <= b1 for (_, e0), (b1, _) in zip(ends, ends[1:])), "overlapping rings"
    assert ends[-1][1] <= lay.pool_bytes


def test_zipf_sizes_and_layout():
    spec = StreamSpec(512, 8192, "zipf", zipf_s=1.1, size=100, config_index=2)
    batches = [make_batch(spec, q) for q in range(12)]
    mean, peak = partition_traffic(batches, spec.partitions)
    sizes = ring_sizes(mean, peak, 64, 64 << 10, 1024)
    assert np.all(sizes & (sizes - 1) == 0) and sizes.min() >= 64 << 10
    assert np.all(peak + 1024 <= sizes)                      # every batch fits (no-space rule)
    assert np.all(sizes >= np.minimum(64 * mean, sizes))
    hot = int(np.argmax(mean))
    assert sizes[hot] >= 16 * sizes.min()
    lay = pool_layout(sizes)
    assert lay.pool_bytes < 2 * int(np.maximum(sizes, lay.segment_bytes).sum())
    _place(np.maximum(sizes, lay.segment_bytes), lay)


def test_layout_with_fixed_floor_and_uniform_sizes():
    g = np.random.default_rng(5)
    sizes = (1 << g.integers(12, 22, 300)).astype(np.uint64)
    lay = pool_layout(sizes, 4096)
    assert lay.segment_bytes == 4096 and list(lay.grown_bytes) == sorted(lay.grown_bytes, reverse=True)
    _place(sizes, lay)
    flat = pool_layout(np.full(64, 1 << 20, np.uint64))
    assert flat.grown.size == 0 and flat.pool_bytes == 64 << 20


def test_bench_configs_fit_one_gpu():
    # config D's shape (RF 5, 4096 partitions, 64 B..16 KB) and config B (Zipf) in a few GiB
    for name, rf, nb in (("B", 3, 6), ("D", 5, 6)):
        spec = CONFIGS[name]
        batches = [make_batch(spec, q) for q in range(nb)]
        mean, peak = partition_traffic(batches, spec.partitions)
        lay = pool_layout(ring_sizes(mean, peak, 64, 64 << 10, 1024))
        assert rf * lay.pool_bytes < 16 << 30, (name, lay.pool_bytes)
