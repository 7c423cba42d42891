"""Diagnostic: wall time of synchronous page-locked fetch calls after an offset commit, with and
without a sync before the call, back to back, and after a sync (one JSON line). Found the ~8 ms
outliers of a blocking event wait."""
import json, sys, time
import numpy as np
sys.path.insert(0, ".")
from ripplemq_amd.engine import Engine, EngineConfig
from ripplemq_amd.workload import CONFIGS, make_batch
spec = CONFIGS["B"]; P, C = spec.partitions, 4
eng = Engine(EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 20, index_interval=1024,
                          max_consumers=8, max_batch_records=spec.records, max_batch_bytes=16 << 20, pipeline_depth=4))
for k in range(16):
    b = make_batch(spec, k); eng.append_async(b.pidx, b.lens, b.payload)
eng.sync()
pp = np.repeat(np.arange(P, dtype=np.uint32), C); cc = np.tile(np.arange(C, dtype=np.uint32), P)
hw = eng.states()["high_watermark"].astype(np.int64)
cap = P * C * 10 * 128 + 4096
d_out = eng.device_alloc(cap)
rq, rs = eng.fetch_rows(P * C); rq[:, 0], rq[:, 1], rq[:, 2] = pp, cc, 10
g = np.random.default_rng(1)
out = {}
def one(pre):
    off = (np.repeat(hw, C) - (g.random(P * C) * 100).astype(np.int64)).clip(0).astype(np.uint64)
    eng.commit_consumer_offset(pp, cc, off)
    if pre == "sync": eng.sync()
    t0 = time.perf_counter(); eng.fetch_device(None, None, None, d_out, cap, req=rq, res=rs, pinned_rows=True)
    t1 = time.perf_counter() - t0
    return round(t1 * 1e6, 1)
for pre in ("none", "sync", "none", "sync"):
    out[pre + str(len(out))] = [one(pre) for _ in range(6)]
def plain():
    t0 = time.perf_counter(); eng.fetch_device(None, None, None, d_out, cap, req=rq, res=rs, pinned_rows=True)
    return round((time.perf_counter() - t0) * 1e6, 1)
out["back_to_back"] = [plain() for _ in range(6)]
eng.sync(); out["after_sync"] = [ (eng.sync(), plain())[1] for _ in range(6)]
print(json.dumps(out))
