"""Synthetic streams: determinism and the RoundRobinSelector / Zipf shapes the configs ask for."""
import numpy as np

from ripplemq_amd.workload import CONFIGS, StreamSpec, make_batch, record_bytes


def test_deterministic():
    s = StreamSpec(64, 1000, "zipf", size=(10, 500), config_index=3)
    a, b = make_batch(s, 7), make_batch(s, 7)
    assert np.array_equal(a.pidx, b.pidx) and np.array_equal(a.lens, b.lens) and np.array_equal(a.payload, b.payload)
    c = make_batch(s, 8)
    assert not np.array_equal(a.payload[:100], c.payload[:100])


def test_round_robin_counter_continues_across_batches():
    # RoundRobinSelector: partitions[abs(counter++) % n] with one counter per topic
    s = StreamSpec(7, 10, "rr")
    got = np.concatenate([make_batch(s, b).pidx for b in range(3)])
    assert list(got) == [i % 7 for i in range(30)]


def test_zipf_skew():
    s = CONFIGS["B"]
    b = make_batch(StreamSpec(s.partitions, 200_000, "zipf", zipf_s=1.1, config_index=2), 0)
    cnt = np.bincount(b.pidx, minlength=s.partitions)
    top = np.sort(cnt)[::-1]
    assert 0.10 < top[0] / cnt.sum() < 0.25      # hottest partition ~16 %
    assert (cnt > 0).sum() > 1000


def test_sizes_and_record_bytes():
    b = make_batch(StreamSpec(4, 5000, "uniform", size=(64, 16384)), 0)
    assert b.lens.min() >= 64 and b.lens.max() <= 16384
    assert record_bytes(np.array([100, 1, 0])) == 128 + 32 + 16
    assert b.payload.size == int(b.lens.sum())
