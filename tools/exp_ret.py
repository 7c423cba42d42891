"""Localise a retention difference (GPU vs oracle) seen with large groups of hot-partition batches."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import OracleEngine
from ripplemq_amd.engine import Engine, EngineConfig
from ripplemq_amd.workload import StreamSpec, make_batch


def run(depth, mixed, seg=1 << 18, nb=10):
    cfg = EngineConfig(num_partitions=300, replication_factor=3, segment_bytes=seg, index_interval=256,
                       max_batch_records=20000, pipeline_depth=depth)
    short = StreamSpec(300, 20000, "zipf", size=(0, 112), config_index=31, invalid_frac=0.005)
    mix = StreamSpec(300, 6000, "uniform", size=(0, 3000), config_index=32)
    batches = [make_batch(mix if (mixed and b % 3 == 0) else short, b) for b in range(nb)]
    with Engine(cfg) as dev, OracleEngine(cfg) as ora:
        subs = [dev.append_async(b.pidx, b.lens, b.payload) for b in batches]
        for (t, out), b in zip(subs, batches):
            sd = dev.wait(t)
            oo, so = ora.append(b.pidx, b.lens, b.payload)
            if sd != so or not np.array_equal(out, oo):
                return f"append differs: {sd} vs {so}"
        bad = [p for p in range(300) if dev.state(p) != ora.state(p)]
        if bad:
            p = bad[0]
            d, o = dev.state(p), ora.state(p)
            return f"{len(bad)} partitions differ, e.g. {p}: gpu start {d['log_start_offset']}@{d['log_start_pos']} cpu {o['log_start_offset']}@{o['log_start_pos']} end {o['log_end_pos']}"
    return "ok"


for depth in (1, 2, 4):
    for mixed in (False, True):
        for seg in (1 << 18, 1 << 20):
            print(f"depth {depth} mixed {mixed} seg {seg}: {run(depth, mixed, seg)}", flush=True)
