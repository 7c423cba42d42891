#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the C oracle (run from the repo root).

Each fixture holds the INPUTS (batches, consumer ops, fetch requests) and the EXPECTED outputs
(out offsets, stats, per-partition state, SHA-256 of every replica ring, live sparse-index
entries, fetch results and fetched bytes). The oracle is pinned independently by the RFC 3720
CRC32C vectors and by tests/refmodel.py; these fixtures pin it (and the GPU engine) against
drift. Regenerate only on an intentional FORMAT.md change.
"""
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from oracle.oracle import OracleEngine  # noqa: E402
from ripplemq_amd.engine import EngineConfig  # noqa: E402
from ripplemq_amd.workload import StreamSpec, make_batch  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

SCENARIOS = {
    # BASELINE configs at fixture scale: A (rr, 256 p), B (Zipf, 4096 p), D (RF 5, 64 B..16 KB)
    "rr_256p": dict(cfg=dict(num_partitions=256, replication_factor=3, segment_bytes=1 << 18,
                             index_interval=1024, max_batch_records=4096),
                    spec=StreamSpec(256, 1024, "rr", size=100, config_index=1), batches=3),
    "zipf_4096p": dict(cfg=dict(num_partitions=4096, replication_factor=3, segment_bytes=1 << 19,
                                index_interval=1024, max_batch_records=4096),
                       spec=StreamSpec(4096, 2048, "zipf", size=100, config_index=2), batches=2),
    "mixed_rf5": dict(cfg=dict(num_partitions=64, replication_factor=5, segment_bytes=1 << 22,
                               index_interval=1024, max_batch_records=4096, max_batch_bytes=8 << 20),
                      spec=StreamSpec(64, 64, "uniform", size=(64, 16384), config_index=4), batches=2),
}


def run(eng, fx):
    """Replay a fixture's inputs on an engine-like object; return the observed outputs."""
    cfg = fx["cfg"]
    P, RF, I = cfg.num_partitions, cfg.replication_factor, cfg.index_interval
    obs = {}
    for b in range(fx["batches"]):
        off, st = eng.append(fx[f"pidx{b}"], fx[f"lens{b}"], fx[f"payload{b}"])
        obs[f"offsets{b}"] = off
        obs[f"stats{b}"] = np.array([st[k] for k in sorted(st) if k != "rejected_invalid"], np.uint64)
        rc, status = eng.commit_consumer_offset(fx[f"cc_p{b}"], fx[f"cc_c{b}"], fx[f"cc_o{b}"])
        obs[f"cc_status{b}"] = status
        rc, res, buf, used = eng.fetch(fx[f"f_p{b}"], fx[f"f_c{b}"], fx[f"f_m{b}"])
        obs[f"fetch_res{b}"] = res.view(np.uint8).copy()
        obs[f"fetch_sha{b}"] = np.frombuffer(hashlib.sha256(buf[:used].tobytes()).digest(), np.uint8)
    states, rings, idx = [], [], []
    for p in range(P):
        s = eng.state(p)
        states.append([s[k] for k in ("log_end_offset", "log_end_pos", "log_start_offset", "log_start_pos",
                                      "commit", "high_watermark", "term", "term_start")] + s["match"])
        for r in range(RF):
            rings.append(np.frombuffer(hashlib.sha256(eng.read_segment(r, p).tobytes()).digest(), np.uint8))
        m_lo, m_hi = -(-s["log_start_pos"] // I), s["log_end_pos"] // I
        h = hashlib.sha256(eng.read_index(p, m_lo, m_hi - m_lo + 1).tobytes()).digest()
        idx.append(np.frombuffer(h, np.uint8))
    obs["states"] = np.array(states, np.uint64)
    obs["ring_sha"] = np.stack(rings)
    obs["index_sha"] = np.stack(idx)
    return obs


def make_inputs(name, sc):
    fx = {"cfg": EngineConfig(**sc["cfg"]), "batches": sc["batches"]}
    spec = sc["spec"]
    g = np.random.default_rng(sum(map(ord, name)))
    P = spec.partitions
    for b in range(sc["batches"]):
        batch = make_batch(spec, b)
        fx[f"pidx{b}"], fx[f"lens{b}"], fx[f"payload{b}"] = batch.pidx, batch.lens, batch.payload
        n = 64
        fx[f"cc_p{b}"] = g.integers(0, P + 1, n).astype(np.uint32)
        fx[f"cc_c{b}"] = g.integers(0, 9, n).astype(np.uint32)
        fx[f"cc_o{b}"] = g.integers(0, 12, n).astype(np.uint64)
        fx[f"f_p{b}"] = g.integers(0, P + 1, n).astype(np.uint32)
        fx[f"f_c{b}"] = g.integers(0, 9, n).astype(np.uint32)
        fx[f"f_m{b}"] = g.integers(0, 20, n).astype(np.uint32)
    return fx


def save(name, fx, obs):
    arrays = {k: v for k, v in fx.items() if isinstance(v, np.ndarray)}
    arrays["cfg"] = np.array([fx["cfg"].num_partitions, fx["cfg"].replication_factor, fx["cfg"].segment_bytes,
                              fx["cfg"].index_interval, fx["cfg"].max_batch_records, fx["cfg"].max_batch_bytes],
                             np.uint64)
    arrays["batches"] = np.array(fx["batches"])
    arrays.update({"exp_" + k: v for k, v in obs.items()})
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrays)


def load(name):
    z = np.load(os.path.join(OUT, f"{name}.npz"), allow_pickle=False)
    c = z["cfg"]
    fx = {k: z[k] for k in z.files if not k.startswith("exp_")}
    fx["cfg"] = EngineConfig(num_partitions=int(c[0]), replication_factor=int(c[1]), segment_bytes=int(c[2]),
                             index_interval=int(c[3]), max_batch_records=int(c[4]), max_batch_bytes=int(c[5]))
    fx["batches"] = int(z["batches"])
    exp = {k[4:]: z[k] for k in z.files if k.startswith("exp_")}
    return fx, exp


if __name__ == "__main__":
    for name, sc in SCENARIOS.items():
        fx = make_inputs(name, sc)
        with OracleEngine(fx["cfg"]) as ora:
            obs = run(ora, fx)
        for b in range(fx["batches"]):  # stats keys sorted: appended first
            assert obs[f"stats{b}"][0] > 0, f"{name}: batch {b} appended nothing (degenerate fixture)"
        save(name, fx, obs)
        print(name, os.path.getsize(os.path.join(OUT, f"{name}.npz")), "bytes")
