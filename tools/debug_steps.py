import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from ripplemq_amd.engine import Engine, EngineConfig
from ripplemq_amd.workload import StreamSpec, make_batch
def log(*a):
    print(f"[{time.time()-T0:7.2f}]", *a, flush=True)
T0 = time.time()
cases = [("small-uniform-100B", dict(num_partitions=8, replication_factor=3, segment_bytes=1 << 16, index_interval=256, max_batch_records=4096), StreamSpec(8, 300, "uniform", size=100)),
         ("small-mixed", dict(num_partitions=8, replication_factor=3, segment_bytes=1 << 16, index_interval=256, max_batch_records=4096), StreamSpec(8, 300, "uniform", size=(0, 700))),
         ("big-records", dict(num_partitions=64, replication_factor=5, segment_bytes=1 << 22, index_interval=1024, max_batch_records=4096, max_batch_bytes=8 << 20), StreamSpec(64, 64, "uniform", size=(64, 16384))),
         ("configB", dict(num_partitions=4096, replication_factor=3, segment_bytes=1 << 23, index_interval=1024, max_batch_records=65536), StreamSpec(4096, 65536, "zipf", size=100, config_index=2))]
which = sys.argv[1:] or [c[0] for c in cases]
for name, kw, spec in cases:
    if name not in which: continue
    log("create", name)
    e = Engine(EngineConfig(**kw))
    log("created")
    for b in range(2):
        bt = make_batch(spec, b)
        t, out = e.append_async(bt.pidx, bt.lens, bt.payload)
        log("submitted", b)
        for i in range(200):
            r = e.poll(t)
            if r: break
            time.sleep(0.05)
        log("poll done" if r else "POLL TIMEOUT", b)
        if not r: sys.exit(3)
        st = e.wait(t)
        log("stats", st, "offs", out[:6])
    log("state0", e.state(0))
    rc, res, buf, used = e.fetch([0, 1], [0, 0], [5, 5])
    log("fetch", rc, res["count"], used)
    e.close()
    log("closed")
