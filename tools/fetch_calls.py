"""Host-side cost of fetch calls (diagnostic): per call wall time of rmq_fetch into a device buffer
with and without profiling, of rmq_fetch_async + poll, and of the consumer commit, on a config-B
engine after a short append run. Prints one JSON line."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ripplemq_amd.engine import FETCH_RES_DTYPE, Engine, EngineConfig  # noqa: E402
from ripplemq_amd.workload import CONFIGS, make_batch  # noqa: E402


def main():
    spec = CONFIGS["B"]
    P, C = spec.partitions, 4
    eng = Engine(EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 20, index_interval=1024,
                              max_consumers=8, max_batch_records=spec.records, max_batch_bytes=16 << 20,
                              pipeline_depth=4))
    for k in range(16):
        b = make_batch(spec, k)
        eng.append_async(b.pidx, b.lens, b.payload)
    eng.sync()
    pp = np.repeat(np.arange(P, dtype=np.uint32), C)
    cc = np.tile(np.arange(C, dtype=np.uint32), P)
    st = eng.states()
    hw = st["high_watermark"].astype(np.int64)
    g = np.random.default_rng(1)
    cap = P * C * 10 * 128 + 4096
    d_out = eng.device_alloc(cap)
    mx = np.full(P * C, 10, np.uint32)
    out = {}

    def tm(f, k=10):
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
        return [round(x * 1e6, 1) for x in ts]

    off = (np.repeat(hw, C) - (g.random(P * C) * 100).astype(np.int64)).clip(0).astype(np.uint64)
    out["commit_us"] = tm(lambda: eng.commit_consumer_offset(pp, cc, off))
    out["fetch_sync_us"] = tm(lambda: eng.fetch_device(pp, cc, mx, d_out, cap))
    eng.profile(True)
    out["fetch_sync_prof_us"] = tm(lambda: eng.fetch_device(pp, cc, mx, d_out, cap))
    eng.profile(False)
    req = np.zeros((P * C, 4), np.uint32)
    req[:, 0], req[:, 1], req[:, 2] = pp, cc, mx
    res = np.zeros(P * C, FETCH_RES_DTYPE)
    out["fetch_async_poll_us"] = tm(lambda: eng.fetch_poll(eng.fetch_async(None, None, None, d_out=d_out, out_cap=cap,
                                                                            req=req, res=res), wait=True))
    out["fetch_async_issue_us"] = tm(lambda: eng.fetch_poll(eng.fetch_async(None, None, None, d_out=d_out, out_cap=cap,
                                                                             req=req, res=res), wait=True), 3)
    prq, prs = eng.fetch_rows(P * C)
    prq[:] = req
    out["fetch_pinned_async_wait_us"] = tm(lambda: eng.fetch_poll(eng.fetch_async(None, None, None, d_out=d_out, out_cap=cap,
                                                                                   req=prq, res=prs, pinned_rows=True), wait=True))
    out["fetch_pinned_sync_us"] = tm(lambda: eng.fetch_device(None, None, None, d_out, cap, req=prq, res=prs,
                                                              pinned_rows=True))
    rows = [eng.fetch_rows(P * C) for _ in range(8)]
    for rq, _ in rows:
        rq[:] = req

    def burst():
        tks = [eng.fetch_async(None, None, None, d_out=d_out, out_cap=cap, req=rq, res=rs, pinned_rows=True)
               for rq, rs in rows]
        for t in tks:
            eng.fetch_poll(t, wait=True)
    out["fetch_pinned_burst8_us_per_call"] = [round(x / 8, 1) for x in tm(burst, 5)]
    eng.device_free(d_out)
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
