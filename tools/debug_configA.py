import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from ripplemq_amd.engine import Engine, EngineConfig
from ripplemq_amd.workload import StreamSpec, make_batch
for P, n in [(256, 65536), (256, 32768), (256, 16384), (256, 8192), (128, 65536), (512, 65536)]:
    cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 23, index_interval=1024, max_batch_records=65536)
    with Engine(cfg) as e:
        b = make_batch(StreamSpec(P, n, "rr", size=100, config_index=1), 0)
        out, st = e.append(b.pidx, b.lens, b.payload)
        exp = np.arange(n) // P
        bad = np.flatnonzero(out != exp)
        print(P, n, "bad", bad.size, "first", bad[:6], out[bad[:6]], "ident?", np.array_equal(out[:P], np.arange(P)), flush=True)
        if bad.size:
            print("  out[:20]", out[:20]); print("  out[P:P+20]", out[P:P+20])
            print("  state p0", e.state(0)); print("  state p1", e.state(1))
