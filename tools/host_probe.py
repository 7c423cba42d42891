"""Probe of the host-batch path (rmq_append from host memory): time in the append call (packing +
DMA issue), time to drain, and the DMA rate of the copy stream alone (pinned staging, one batch)."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ripplemq_amd.engine import Engine, EngineConfig  # noqa: E402
from ripplemq_amd.workload import CONFIGS, make_batch  # noqa: E402

spec = CONFIGS["B"]
cfg = EngineConfig(num_partitions=spec.partitions, replication_factor=3, segment_bytes=4 << 20, index_interval=1024,
                   max_batch_records=spec.records, max_batch_bytes=8 << 20, pipeline_depth=4)
bs = [make_batch(spec, q) for q in range(8)]
with Engine(cfg) as eng:
    for k in range(24):
        b = bs[k % 8]
        eng.append_async(b.pidx, b.lens, b.payload)
    eng.sync()
    calls = []
    t0 = time.perf_counter()
    for k in range(100):
        b = bs[k % 8]
        c0 = time.perf_counter()
        eng.append_async(b.pidx, b.lens, b.payload)
        calls.append(time.perf_counter() - c0)
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    c = np.array(calls) * 1e6
    print(f"100 host batches: {1e3 * (t2 - t0):.1f} ms total, calls {1e3 * (t1 - t0):.1f} ms, drain {1e3 * (t2 - t1):.1f} ms; "
          f"call us median {np.median(c):.0f} p10 {np.percentile(c, 10):.0f} p90 {np.percentile(c, 90):.0f} max {c.max():.0f}")
    bytes_ = bs[0].payload.nbytes + 8 * bs[0].n
    print(f"batch bytes {bytes_ / 1e6:.2f} MB -> {bytes_ * 100 / (t2 - t0) / 1e9:.2f} GB/s overall")
