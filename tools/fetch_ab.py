"""Fetch call timing without trusting any one clock: 16384 requests x max 10 on a config-B engine,
median host wall time per call (each call waits for its results) and the engine's event region
(first kernel start to last kernel end). Run it under RMQ_LIB=<library> to compare builds."""
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ripplemq_amd.engine import Engine, EngineConfig  # noqa: E402
from ripplemq_amd.workload import CONFIGS, make_batch  # noqa: E402

spec = CONFIGS["B"]
P = spec.partitions
cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=4 << 20, index_interval=1024,
                   max_batch_records=spec.records, max_batch_bytes=8 << 20, pipeline_depth=4, max_consumers=4)
with Engine(cfg) as eng:
    for q in range(16):
        b = make_batch(spec, q)
        eng.append_async(b.pidx, b.lens, b.payload)
    eng.sync()
    pp = np.repeat(np.arange(P, dtype=np.uint32), 4)
    cc = np.tile(np.arange(4, dtype=np.uint32), P)
    eng.commit_consumer_offset(pp, cc, np.zeros(P * 4, np.uint64))
    for mx in (10, 1024):
        cap = P * 4 * mx * 128 + 4096
        d_out = eng.device_alloc(cap)
        walls, regions = [], []
        for k in range(25):
            prof = k % 2 == 1
            if prof:
                eng.profile(True)
            t0 = time.perf_counter()
            rc, res, used = eng.fetch_device(pp, cc, np.full(P * 4, mx, np.uint32), d_out, cap)
            dt = time.perf_counter() - t0
            if prof:
                regions.append(eng.profile_query(4)[1] * 1e3)
                eng.profile(False)
            elif k:
                walls.append(dt * 1e6)
        print(f"{os.environ.get('RMQ_LIB', 'default')} max={mx}: wall per call median {statistics.median(walls):.0f} us "
              f"(min {min(walls):.0f}), event region median {statistics.median(regions):.0f} us, "
              f"records {int(res['count'].sum())}")
        eng.device_free(d_out)
