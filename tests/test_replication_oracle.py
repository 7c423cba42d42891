"""Replica-log rounds on the CPU oracle (FORMAT.md §9): every follower ends with its
leader's log, bytes and offsets; quorum acks commit; refused rounds (CRC, log mismatch) do not."""
import numpy as np
import pytest

from repl_sim import exchange_round, place, rank_batches, rank_cfg
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import rank_view, replica_ranks
from ripplemq_amd.workload import StreamSpec

BASE = EngineConfig(num_partitions=1, replication_factor=3, segment_bytes=1 << 16, index_interval=256,
                    max_batch_records=4096)


def build(oracle_mod, world, ppr, rf=3, base=BASE):
    views = [rank_view(r, world, ppr, rf) for r in range(world)]
    oras = []
    for r in range(world):
        b = EngineConfig(**{**base.__dict__, "replication_factor": rf})
        o = oracle_mod.OracleEngine(rank_cfg(b, views[r], r))
        place(o, views[r], world)
        oras.append(o)
    return views, oras


def local_of(views, rank, gp):
    return int(np.flatnonzero(views[rank].gp == gp)[0])


def check_followers(views, oras, ppr, rf, full_ring=True):
    W = len(oras)
    for g in range(W):
        for gp in range(g * ppr, (g + 1) * ppr):
            lp = local_of(views, g, gp)
            ls = oras[g].state(lp)
            assert ls["commit"] == ls["log_end_offset"], (gp, ls)
            ring = oras[g].read_segment(0, lp)
            for slot, r in enumerate(replica_ranks(g, gp, W, rf)):
                if r == g:
                    continue
                fp = local_of(views, r, gp)
                fs = oras[r].state(fp)
                assert fs["log_end_offset"] == ls["log_end_offset"] and fs["log_end_pos"] == ls["log_end_pos"]
                assert fs["is_leader"] == 0
                assert np.array_equal(oras[r].read_segment(slot, fp), ring), f"gp {gp} slot {slot} ring"


@pytest.mark.parametrize("world,rf", [(2, 3), (3, 3), (4, 3), (8, 3), (8, 5)])
def test_rounds_replicate_every_log(oracle_mod, world, rf):
    ppr, G, R = 8, 2, 3
    views, oras = build(oracle_mod, world, ppr, rf)
    spec = StreamSpec(ppr, 300, "zipf", size=(0, 150), config_index=51)
    try:
        batches = [rank_batches(spec, r, R, G) for r in range(world)]
        for k in range(R):
            for r in range(world):
                for b in batches[r][k * G:(k + 1) * G]:
                    _, st = oras[r].append(b.pidx, b.lens, b.payload)
                    assert st["appended"] == b.n
            exchange_round(oras)
        check_followers(views, oras, ppr, rf)
        assert sum(int(o.counters()[0]) for o in oras) == (rf - 1) * sum(b.n for bs in batches for b in bs)
    finally:
        for o in oras:
            o.close()


def test_retention_on_followers_per_round(oracle_mod):
    # 64 KB rings: the hot partitions wrap inside a round; follower rings still equal the leader's
    world, ppr, G, R = 3, 4, 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 400, "zipf", size=(40, 160), config_index=52)
    try:
        for k in range(R):
            for r in range(world):
                for b in rank_batches(spec, r, R, G)[k * G:(k + 1) * G]:
                    oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras)
        check_followers(views, oras, ppr, 3)
        assert max(o.state(p)["log_start_offset"] for o in oras for p in range(len(views[0].gp))) > 0
    finally:
        for o in oras:
            o.close()


def test_refused_rounds_do_not_commit_on_their_own(oracle_mod):
    world, ppr = 3, 4
    views, oras = build(oracle_mod, world, ppr)
    spec = StreamSpec(ppr, 200, "uniform", size=(1, 100), config_index=53)
    try:
        for r in range(world):
            b = rank_batches(spec, r, 1, 1)[0]
            oras[r].append(b.pidx, b.lens, b.payload)
        # rank 0's region to rank 1 has a flipped payload byte: rank 1 refuses the entry it hits,
        # rank 2 accepts everything, so rank 0's partitions still commit on the quorum {0, 2}
        regions = exchange_round(oras, keep_regions=True, corrupt=(0, 1, -5))
        assert oras[1].counters()[1] == 1
        for gp in range(ppr):
            s = oras[0].state(local_of(views, 0, gp))
            assert s["commit"] == s["log_end_offset"]
        # rank 2 misses rank 0's next round: the round after that no longer continues its log
        for k in (1, 2):
            for r in range(world):
                b = rank_batches(spec, r, 3, 1)[k]
                oras[r].append(b.pidx, b.lens, b.payload)
            exchange_round(oras, skip=(0, 2) if k == 1 else None)
        assert oras[2].counters()[2] > 0
        assert regions[0][1].size > 0
    finally:
        for o in oras:
            o.close()


def test_leader_change_truncates_follower(oracle_mod):
    # Raft's follower truncation (FORMAT.md §9): rank 0's third round is lost, leadership of its
    # partitions moves to slot 1 at term 2; rank 0 drops its uncommitted tail and follows
    from repl_sim import leader_change_script, run_script_oracle
    world, rf, ppr, group = 3, 3, 6, 2
    spec = StreamSpec(ppr, 300, "uniform", size=(0, 120), config_index=71)
    base = EngineConfig(num_partitions=1, replication_factor=rf, segment_bytes=1 << 16, index_interval=256,
                        max_batch_records=4096, pipeline_depth=group)
    views, new, phases = leader_change_script(spec, world, rf, ppr, group)
    cfgs = [rank_cfg(base, views[r], r) for r in range(world)]
    oras = [oracle_mod.OracleEngine(c) for c in cfgs]
    try:
        for r in range(world):
            place(oras[r], views[r], world)
        # before the change: rank 0 holds a tail nobody else has
        run_script_oracle(oras, views, phases[:3], world)
        s0 = [oras[0].state(p) for p in range(ppr)]
        assert all(s["log_end_offset"] > s["commit"] for s in s0)
        f1 = {int(views[1].gp[i]): oras[1].state(i) for i in range(len(views[1].gp))}
        assert all(f1[int(views[0].gp[p])]["log_end_offset"] == s0[p]["commit"] for p in range(ppr)
                   if int(views[0].gp[p]) in f1)
        run_script_oracle(oras, views, phases[3:], world)
        c = oras[0].counters()
        assert c[1] == 0 and c[2] == 0, c  # nothing refused: rank 0 truncated and accepted
        for p in range(ppr):  # rank 0 now follows: same log end and term as the new leader
            g = int(views[0].gp[p])
            r1 = int(views[0].ranks[p][1])
            q = int(np.flatnonzero(views[r1].gp == g)[0])
            lead, fol = oras[r1].state(q), oras[0].state(p)
            assert fol["log_end_offset"] == lead["log_end_offset"] and fol["term"] == 2 == lead["term"]
            assert lead["commit"] == lead["log_end_offset"] > s0[p]["commit"]
            assert fol["log_end_pos"] == lead["log_end_pos"]
            a = oras[0].read_segment(int(np.flatnonzero(views[0].ranks[p] == 0)[0]), p)
            b = oras[r1].read_segment(int(np.flatnonzero(views[r1].ranks[q] == r1)[0]), q)
            lo, hi = fol["log_start_pos"], fol["log_end_pos"]
            S = fol["segment_bytes"]
            idx = (np.arange(lo, hi) % S)
            assert np.array_equal(a[idx], b[idx])
    finally:
        for o in oras:
            o.close()
