"""One rank of the world-size-3 CPU rehearsal of leader election over gloo (tests/test_election.py).

Launched as a plain subprocess per rank (RANK/WORLD_SIZE/MASTER_* in the env, 127.0.0.1). Each rank
runs the oracle engine of the partitions it hosts, does a replication round per step over gloo as
tests/dist_repl_worker.py does (regions, ingest, acks; then the commit notices), with rank 0's
regions and notices to the others lost during tests/election_world.py's ISOLATED rounds (a one-byte
marker stands for a lost region: the receiver ingests it as missed), and then one
ripplemq_amd.election.ElectionDriver tick whose RequestVotes and answers travel over gloo
(GlooChannel). Rank 0 writes every rank's election log and final states as JSON.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dist_repl_worker import exchange  # noqa: E402
from election_world import ISOLATED, PPR, RF, ROUNDS, SPEC, _salt  # noqa: E402
from oracle.oracle import OracleEngine  # noqa: E402
from repl_sim import led_batches, place, rank_cfg  # noqa: E402
from ripplemq_amd.election import ElectionDriver, GlooChannel  # noqa: E402
from ripplemq_amd.engine import EngineConfig  # noqa: E402
from ripplemq_amd.sharding import rank_view  # noqa: E402

BASE = dict(num_partitions=1, replication_factor=RF, segment_bytes=1 << 18, index_interval=256,
            max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=2, max_consumers=4)
EMPTY = np.zeros(0, np.uint8)


def one_round(eng, rank, world, lost):
    rnd = eng.round_no()
    send = [EMPTY] * world
    for d in range(world):
        if d != rank:
            send[d] = np.ones(1, np.uint8) if (rank, d) in lost else np.ascontiguousarray(eng.round_region(d))
    eng.end_round()
    got = exchange(rank, world, send)
    acks = [EMPTY] * world
    for q in range(world):
        if q != rank and got[q].size:
            a = eng.ingest(q, EMPTY if got[q].size == 1 else got[q])
            acks[q] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
    back = exchange(rank, world, acks)
    for q in range(world):
        if q != rank and back[q].size:
            eng.apply_acks(q, back[q].view(np.uint64).reshape(-1, 2), rnd)
    # the drain's commit notices (lost with the regions while cut)
    notes = [EMPTY] * world
    for d in range(world):
        if d != rank and (rank, d) not in lost:
            notes[d] = np.ascontiguousarray(eng.commit_notice(d)).reshape(-1).view(np.uint8)
    got = exchange(rank, world, notes)
    for q in range(world):
        if q != rank and got[q].size:
            eng.apply_notice(q, got[q].view(np.uint64).reshape(-1, 2))


def main():
    out_path, seed = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    view = rank_view(rank, world, PPR, RF)
    with OracleEngine(rank_cfg(EngineConfig(**BASE), view, rank)) as eng:
        place(eng, view, world)
        drv = ElectionDriver(eng, view, GlooChannel(), seed=seed)
        log = []
        for k in range(ROUNDS):
            for b in led_batches(SPEC, drv.view, rank, 2, _salt(k) + 1000 * rank):
                eng.append(b.pidx, b.lens, b.payload)
            one_round(eng, rank, world, [(0, 1), (0, 2)] if k in ISOLATED else [])
            log.append([[e.gid, e.term, e.leader, e.started] for e in drv.tick()])
        n = len(view.gp)
        states = [eng.state(p) for p in range(n)]
        final = {"gp": drv.view.gp.tolist(), "ranks": drv.view.ranks.tolist(), "leader_slot": drv.view.leader_slot.tolist()}
        fetched = {}
        for p in range(n):
            if states[p]["is_leader"]:
                rc, res, buf, used = eng.fetch(np.array([p], np.uint32), np.zeros(1, np.uint32),
                                               np.full(1, 100000, np.uint32))
                fetched[int(view.gp[p])] = buf[:used].tobytes().hex()
    gathered = [None] * world
    dist.all_gather_object(gathered, {"rank": rank, "log": log, "states": states, "final": final, "fetched": fetched})
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(gathered, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
