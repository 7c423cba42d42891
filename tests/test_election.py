"""Leader election across ranks (ripplemq_amd/election.py).

Reference: jraft's election timer and RequestVote (PartitionRaftServer.java:85,89), the winner's
onLeaderStart (PartitionStateMachine.java:121-126) and the leader-map update
(PartitionManager.java:248-275). The scenario (tests/election_world.py): rank 0 leads its
partitions, its regions and commit notices stop reaching its followers for four rounds; the
followers' election ticks elect one of them per partition, every rank moves the leader slot, and the
new leader serves the committed records and commits new ones while rank 0 truncates its tail.
Checked on per-rank oracles in threads, on three gloo processes (the host channel and the rounds over
gloo, as bench.py's ranks), and on GPU engines against the oracles.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from election_world import PPR, RF, SPEC, WORLD, _salt, check_world, run_gpu_world, run_oracle_world
from repl_sim import led_batches, rank_cfg
from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.sharding import rank_view
from ripplemq_amd.tier import split_records

HERE = os.path.dirname(os.path.abspath(__file__))
BASE = dict(num_partitions=1, replication_factor=RF, segment_bytes=1 << 18, index_interval=256,
            max_batch_records=4096, max_batch_bytes=1 << 20, pipeline_depth=2, max_consumers=4)


def _committed_prefix(gid: int) -> list[bytes]:
    """Rank 0's records of gid from the two rounds before the isolation, in append order (the
    reference's messages.addAll): every replica acknowledged them, so a new leader holds them."""
    view0 = rank_view(0, WORLD, PPR, RF)
    out = []
    for k in range(2):
        for b in led_batches(SPEC, view0, 0, 2, _salt(k)):
            pos = np.concatenate([[0], np.cumsum(b.lens.astype(np.int64))])
            out += [bytes(b.payload[pos[i]:pos[i + 1]]) for i in np.flatnonzero(b.pidx == gid)]
    return out


def _serves(img: bytes, gid: int) -> None:
    msgs = [m for _, _, m in split_records(img)]
    want = _committed_prefix(gid)
    assert len(msgs) > len(want) and msgs[:len(want)] == want, (gid, len(msgs), len(want))


def test_election_threads_oracle(oracle_mod):
    views = [rank_view(r, WORLD, PPR, RF) for r in range(WORLD)]
    oras = [oracle_mod.OracleEngine(rank_cfg(EngineConfig(**BASE), views[r], r)) for r in range(WORLD)]
    try:
        log, final = run_oracle_world(oras, views)
        moved = check_world(log, final, oras)
        for gid, (term, leader) in moved.items():
            p = int(np.flatnonzero(final[leader].gp == gid)[0])
            rc, res, buf, used = oras[leader].fetch(np.array([p], np.uint32), np.zeros(1, np.uint32),
                                                    np.full(1, 100000, np.uint32))
            assert rc == 0 and res["status"][0] == 0
            _serves(bytes(buf[:used]), gid)
    finally:
        for o in oras:
            o.close()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_election_gloo_world3(tmp_path):
    out = tmp_path / "election.json"
    port = _free_port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_election_worker.py"), str(out), "5"],
                                      env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    got = json.loads(out.read_text())
    logs = [[[tuple(x) for x in tick] for tick in g["log"]] for g in got]
    assert all(lg == logs[0] for lg in logs)
    els = [x for tick in logs[0] for x in tick]
    assert len({(g, t) for g, t, _, _ in els}) == len(els)  # one leader per (partition, term)
    moved = {g: (t, c) for g, t, c, s in els if s}
    assert set(moved) == set(range(PPR)) and all(t >= 2 for t, _ in moved.values()), els
    for gid, (term, leader) in moved.items():
        _serves(bytes.fromhex(got[leader]["fetched"][str(gid)]), gid)
        sts = [s for g in got for p, s in enumerate(g["states"]) if g["final"]["gp"][p] == gid]
        assert len(sts) == RF and len({s["log_end_offset"] for s in sts}) == 1, sts
        assert sum(s["is_leader"] for s in sts) == 1
    # the gloo run and the in-process run of the same scenario decide the same elections
    import oracle.oracle as om
    views = [rank_view(r, WORLD, PPR, RF) for r in range(WORLD)]
    oras = [om.OracleEngine(rank_cfg(EngineConfig(**BASE), views[r], r)) for r in range(WORLD)]
    try:
        want, _ = run_oracle_world(oras, views)
        assert [[tuple(x) for x in tick] for tick in want[0]] == logs[0]
    finally:
        for o in oras:
            o.close()


@pytest.mark.gpu
def test_election_gpu(oracle_mod):
    from parity import compare_state
    from ripplemq_amd.engine import Engine, LocalHub

    views = [rank_view(r, WORLD, PPR, RF) for r in range(WORLD)]
    cfgs = [rank_cfg(EngineConfig(**BASE), views[r], r) for r in range(WORLD)]
    hub = LocalHub(WORLD)
    engs = [Engine(c) for c in cfgs]
    oras = []
    try:
        log, final = run_gpu_world(engs, hub, views)
        oras = [oracle_mod.OracleEngine(c) for c in cfgs]
        want, _ = run_oracle_world(oras, views)
        assert log == want, (log, want)
        moved = check_world(log, final, engs)
        for r in range(WORLD):
            def local_slots(p, r=r):
                return [s for s in range(RF) if final[r].ranks[p][s] == r]
            compare_state(engs[r], oras[r], cfgs[r], local_slots=local_slots)
        for gid, (term, leader) in moved.items():
            p = int(np.flatnonzero(final[leader].gp == gid)[0])
            rc, res, buf, used = engs[leader].fetch(np.array([p], np.uint32), np.zeros(1, np.uint32),
                                                    np.full(1, 100000, np.uint32))
            assert rc == 0 and res["status"][0] == 0
            _serves(bytes(buf[:used]), gid)
    finally:
        for o in oras:
            o.close()
        for e in engs:
            e.close()
        hub.close()


@pytest.mark.gpu
def test_vote_with_groups_in_flight_gpu():
    """rmq_vote is not collective: a leader whose launch groups are still forming or in
    flight answers RMQ_PENDING (the Python call: not granted) and changes nothing — no flush, which
    with a transport every rank would have to join; after the next collective sync the same
    RequestVote of a newer term is granted and the leader steps down."""
    import threading

    from repl_sim import place
    from ripplemq_amd.engine import Engine, LocalHub

    views = [rank_view(r, WORLD, PPR, RF) for r in range(WORLD)]
    cfgs = [rank_cfg(EngineConfig(**BASE), views[r], r) for r in range(WORLD)]
    hub = LocalHub(WORLD)
    engs = [Engine(c) for c in cfgs]
    bar = threading.Barrier(WORLD, timeout=120)
    seen = {}
    errs = []

    def body(r):
        try:
            e = engs[r]
            e.attach_local(hub)
            place(e, views[r])
            bs = led_batches(SPEC, views[r], r, 1, _salt(0) + 1000 * r)
            v = views[r]
            led = int(np.flatnonzero(v.ranks[np.arange(len(v.gp)), v.leader_slot] == r)[0])
            bar.wait()
            if r == 0:
                for b in bs:
                    e.append_async(b.pidx, b.lens, b.payload)  # a group forming on rank 0 only
                t0 = e.lib.rmq_vote  # (the raw status, through the Python wrapper's argument types)
                import ctypes as C
                g = C.c_uint32(7)
                seen["rc"] = t0(e.h, led, 5, 1, 99, 1 << 40, C.byref(g))
                seen["granted"] = g.value
            bar.wait()
            if r != 0:
                e.append_async(np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
            e.sync()  # collective: the round carries rank 0's group
            bar.wait()
            if r == 0:
                before = e.state(led)
                seen["before"] = (before["term"], before["is_leader"])
                seen["again"] = e.vote(led, 5, 1, 99, 1 << 40)
                after = e.state(led)
                seen["after"] = (after["term"], after["is_leader"])
            bar.wait()
        except BaseException as ex:  # noqa: BLE001 - reported below
            errs.append((r, ex))
            bar.abort()

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(WORLD)]
    try:
        for t in ts:
            t.start()
        for t in ts:
            t.join(240)
            assert not t.is_alive(), "a rank hung"
        assert not errs, errs
        from ripplemq_amd import _abi as A
        assert seen["rc"] == A.RMQ_PENDING and seen["granted"] == 0, seen
        assert seen["before"] == (1, 1), seen  # nothing changed by the pending vote
        assert seen["again"] is True and seen["after"] == (5, 0), seen
    finally:
        for e in engs:
            e.close()
        hub.close()
