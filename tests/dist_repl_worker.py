"""One rank of the world-size-N CPU rehearsal of the replica-log rounds (gloo, FORMAT.md §9).

Launched by tests/test_distributed.py as a plain subprocess per rank (RANK/WORLD_SIZE/MASTER_* in
the env, MASTER_ADDR=127.0.0.1). Each rank runs the oracle engine of the partitions it hosts
(CPU stand-in for its GPU engine) and does what the engine's exchange stream does per round, over
gloo instead of RCCL: swap {region bytes} with every peer, send/recv the regions, ingest what it
received, send/recv the acks (FORMAT.md §9 v3: follower log end and status) and apply them. Rank 0 writes every rank's final
partition states and ring digests as JSON for the parent test.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle.oracle import OracleEngine, crc32c  # noqa: E402
from repl_sim import place, rank_batches, rank_cfg  # noqa: E402
from ripplemq_amd.engine import EngineConfig  # noqa: E402
from ripplemq_amd.sharding import rank_view  # noqa: E402
from ripplemq_amd.workload import StreamSpec  # noqa: E402


def exchange(rank, world, send):
    """Grouped point-to-point exchange of byte arrays (sizes first, like the engine)."""
    sizes = torch.tensor([len(send[q]) if q != rank else 0 for q in range(world)], dtype=torch.int64)
    recv_sizes = torch.zeros(world, dtype=torch.int64)
    ops = []
    for q in range(world):
        if q != rank:
            ops.append(dist.P2POp(dist.isend, sizes[q:q + 1].clone(), q))
            ops.append(dist.P2POp(dist.irecv, recv_sizes[q:q + 1], q))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    out, ops = [None] * world, []
    for q in range(world):
        if q == rank:
            continue
        if len(send[q]):
            ops.append(dist.P2POp(dist.isend, torch.from_numpy(np.ascontiguousarray(send[q])), q))
        out[q] = torch.zeros(int(recv_sizes[q]), dtype=torch.uint8)
        if int(recv_sizes[q]):
            ops.append(dist.P2POp(dist.irecv, out[q], q))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return [None if t is None else t.numpy() for t in out]


def main():
    out_path, ppr, rounds, group = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    view = rank_view(rank, world, ppr, 3)
    base = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 16, index_interval=256)
    spec = StreamSpec(ppr, 500, "zipf", size=(0, 120), config_index=71)
    batches = rank_batches(spec, rank, rounds, group)
    with OracleEngine(rank_cfg(base, view, rank)) as eng:
        place(eng, view, world)
        for k in range(rounds):
            for b in batches[k * group:(k + 1) * group]:
                eng.append(b.pidx, b.lens, b.payload)
            rnd = eng.round_no()
            regions = [eng.round_region(q) if q != rank else np.zeros(0, np.uint8) for q in range(world)]
            eng.end_round()
            got = exchange(rank, world, regions)
            acks = [np.zeros(0, np.uint8)] * world
            for q in range(world):
                if q != rank and got[q].size:
                    acks[q] = np.ascontiguousarray(eng.ingest(q, got[q])).reshape(-1).view(np.uint8)
            back = exchange(rank, world, acks)
            for q in range(world):
                if q != rank and back[q].size:
                    eng.apply_acks(q, back[q].view(np.uint64).reshape(-1, 2), rnd)
        n = len(view.gp)
        states = [eng.state(p) for p in range(n)]
        rings = [[crc32c(eng.read_segment(s, p).tobytes()) for s in range(3)] for p in range(n)]
    gathered = [None] * world
    dist.all_gather_object(gathered, {"rank": rank, "states": states, "rings": rings})
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(gathered, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
