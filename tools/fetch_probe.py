"""Probe of rmq_fetch call latency: 16384 requests x max 10 on a config-B engine, wall time per
call with and without the profile events, and the engine's own event region."""
import os
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
    cap = P * 4 * 10 * 128 + 4096
    d_out = eng.device_alloc(cap)
    order = (("states", True), (True, True), (False, True)) if "states_first" in sys.argv else \
        ((False, False), (True, False), (True, True), (False, True), ("states", True), (True, True))
    for prof, commit in order:
        if prof == "states":
            t0 = time.perf_counter()
            st = [eng.state(p) for p in range(P)]
            print(f"{P} state() calls: {(time.perf_counter() - t0) * 1e3:.0f} ms")
            prof = True
        for k in range(6):
            if commit:
                eng.commit_consumer_offset(pp, cc, np.zeros(P * 4, np.uint64))
            if prof:
                eng.profile(True)
            t0 = time.perf_counter()
            rc, res, used = eng.fetch_device(pp, cc, np.full(P * 4, 10, np.uint32), d_out, cap)
            dt = time.perf_counter() - t0
            ms = eng.profile_query(3)[1] if prof else 0.0
            if prof:
                eng.profile(False)
            print(f"profile={prof} commit={commit} round {k}: call {dt * 1e6:.0f} us, event region {ms * 1e3:.0f} us, records {int(res['count'].sum())}")
    eng.device_free(d_out)
