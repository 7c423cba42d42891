"""One rank of the world-size-N CPU rehearsal of the partition-sharded path (gloo).

Launched by tests/test_distributed.py as a plain subprocess per rank (RANK/WORLD_SIZE/MASTER_*
in the env, MASTER_ADDR=127.0.0.1). Each rank routes every global batch with
ripplemq_amd.sharding.split_batch, appends ITS shard through the oracle handle (CPU stand-in for
the rank's GPU engine), and the results travel to rank 0 by gloo all_gather_object; rank 0
writes them as JSON for the parent test to compare with one engine holding every partition.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle.oracle import OracleEngine, crc32c  # noqa: E402
from ripplemq_amd.engine import EngineConfig  # noqa: E402
from ripplemq_amd.sharding import max_over_ranks, split_batch  # noqa: E402
from ripplemq_amd.workload import StreamSpec, make_batch  # noqa: E402


def main():
    out_path, p_local, batches = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    cfg = EngineConfig(num_partitions=p_local, replication_factor=3, segment_bytes=1 << 16,
                       index_interval=256)
    spec = StreamSpec(world * p_local, 700, "zipf", size=(0, 90), config_index=31)
    offs, t0 = [], time.perf_counter()
    with OracleEngine(cfg) as eng:
        for k in range(batches):
            b = make_batch(spec, k)
            sh = split_batch(b.pidx, b.lens, world, p_local)[rank]
            o, st = eng.append(sh.pidx, sh.lens, b.payload, sh.payload_off)
            assert st["appended"] == len(sh.records)
            offs.append({"records": sh.records.tolist(), "offsets": o.tolist()})
        states = [eng.state(p) for p in range(p_local)]
        rings = [[crc32c(eng.read_segment(r, p).tobytes()) for p in range(p_local)] for r in range(3)]
    t_max = max_over_ranks(time.perf_counter() - t0, dist)
    gathered = [None] * world
    dist.all_gather_object(gathered, {"rank": rank, "offs": offs, "states": states, "rings": rings,
                                      "t_max": t_max})
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(gathered, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
