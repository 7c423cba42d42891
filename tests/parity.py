"""Scenario driver: run one op list through the GPU engine and the CPU oracle, compare everything.

Bar (bit-exact, integer/byte path): out offsets, append stats, every partition's state (log end,
start, commit, high watermark, matchIndex row, term start), the live sparse-index entries, the
retained window of every local replica ring (or the whole ring for small configs), consumer
offsets, and fetch results + fetched bytes.
"""
from __future__ import annotations

import numpy as np

from ripplemq_amd.workload import Batch


def ring_window(eng, cfg, replica, p, st):
    """Bytes of the retained log window [log_start_pos, log_end_pos) read out of the ring."""
    S = st["segment_bytes"]
    lo, hi = st["log_start_pos"], st["log_end_pos"]
    if hi - lo > S:
        lo = hi - S
    n = hi - lo
    if n == 0:
        return np.zeros(0, np.uint8)
    a = lo % S
    if a + n <= S:
        return eng.read_segment(replica, p, a, n)
    return np.concatenate([eng.read_segment(replica, p, a, S - a), eng.read_segment(replica, p, 0, n - (S - a))])


def compare_state(dev, ora, cfg, parts=None, full_rings=False, local_slots=None):
    P, I = cfg.num_partitions, cfg.index_interval
    for p in (range(P) if parts is None else parts):
        sd, so = dev.state(p), ora.state(p)
        assert sd == so, f"partition {p} state\n gpu={sd}\n cpu={so}"
        slots = range(cfg.replication_factor) if local_slots is None else local_slots(p)
        for r in slots:
            if full_rings:
                a, b = dev.read_segment(r, p), ora.read_segment(r, p)
            else:
                a, b = ring_window(dev, cfg, r, p, sd), ring_window(ora, cfg, r, p, so)
            if not np.array_equal(a, b):
                bad = np.flatnonzero(a != b)
                raise AssertionError(f"ring p={p} r={r}: {bad.size} bytes differ, first at {bad[0]}")
        m_lo = -(-so["log_start_pos"] // I)
        m_hi = so["log_end_pos"] // I
        if m_hi >= m_lo:
            cnt = m_hi - m_lo + 1
            ia, ib = dev.read_index(p, m_lo, cnt), ora.read_index(p, m_lo, cnt)
            assert np.array_equal(ia, ib), f"index p={p} m=[{m_lo},{m_hi}]"
        assert np.array_equal(dev.consumer_offsets(p), ora.consumer_offsets(p)), f"consumer offsets p={p}"


def run_ops(dev, ora, cfg, ops, check=True, full_rings=False, parts=None, local_slots=None):
    """Apply ops to both engines, comparing outputs of every op and state after each append."""
    log = []
    submitted = appended = 0
    for op in ops:
        kind = op[0]
        if kind == "append":
            b: Batch = op[1]
            poff = op[2] if len(op) > 2 else None
            payload = op[3] if len(op) > 3 else b.payload
            od, sd = dev.append(b.pidx, b.lens, payload, poff)
            oo, so = ora.append(b.pidx, b.lens, payload, poff)
            assert sd == so, f"append stats gpu={sd} cpu={so}"
            if not np.array_equal(od, oo):
                bad = np.flatnonzero(od != oo)
                raise AssertionError(f"out_offsets differ at {bad[:8]}: gpu={od[bad[:8]]} cpu={oo[bad[:8]]}")
            log.append(("append", sd))
            submitted += len(b.pidx)
            appended += sd["appended"]
            if check:
                compare_state(dev, ora, cfg, parts, full_rings, local_slots)
        elif kind == "consumer_commit":
            rd, std = dev.commit_consumer_offset(*op[1:4])
            ro, sto = ora.commit_consumer_offset(*op[1:4])
            assert rd == ro and np.array_equal(std, sto), (rd, ro, std, sto)
        elif kind == "fetch":
            out_cap = op[4] if len(op) > 4 else None
            rd, resd, bd, ud = dev.fetch(op[1], op[2], op[3], out_cap)
            ro, reso, bo, uo = ora.fetch(op[1], op[2], op[3], out_cap)
            assert rd == ro, (rd, ro)
            assert ud == uo, (ud, uo)
            if not np.array_equal(resd, reso):
                bad = np.flatnonzero(resd != reso)
                raise AssertionError(f"fetch res differ at {bad[:4]}:\n gpu={resd[bad[:4]]}\n cpu={reso[bad[:4]]}")
            n = min(ud, len(bd))
            assert np.array_equal(bd[:n], bo[:n]), "fetched bytes differ"
            log.append(("fetch", resd, bd))
        elif kind == "become_leader":
            dev.become_leader(op[1], op[2])
            ora.become_leader(op[1], op[2])
        elif kind == "set_replicas":
            dev.set_replicas(op[1], op[2], op[3])
            ora.set_replicas(op[1], op[2], op[3])
        elif kind == "set_segments":
            dev.set_segments(op[1], op[2])
            ora.set_segments(op[1], op[2])
            if check:
                compare_state(dev, ora, cfg, parts, full_rings, local_slots)
        elif kind == "ack":
            dev.ack(op[1], op[2], op[3])
            ora.ack(op[1], op[2], op[3])
            if check:
                compare_state(dev, ora, cfg, parts, full_rings, local_slots)
        else:
            raise ValueError(kind)
    if check:
        compare_state(dev, ora, cfg, parts, full_rings, local_slots)
    # a scenario whose every batch is rejected (e.g. batches larger than the ring) compares empty
    # logs and proves nothing
    assert not submitted or appended, "no record was appended: the scenario is vacuous"
    return log


def compare_bulk(dev, ora, cfg, local_slots=None, chunk=4096):
    """compare_state for many partitions: states by one bulk read-back per side
    (rmq_get_partition_states), then each partition's retained ring window of every local slot, its
    live index entries and consumer offsets."""
    P, I = cfg.num_partitions, cfg.index_interval
    for a in range(0, P, chunk):
        n = min(chunk, P - a)
        sd, so = dev.states(a, n), ora.states(a, n)
        if not np.array_equal(sd, so):
            bad = [a + i for i in range(n) if sd[i].tobytes() != so[i].tobytes()]
            p = bad[0]
            raise AssertionError(f"{len(bad)} partition states differ, first {p}\n gpu={dev.state(p)}\n cpu={ora.state(p)}")
        for i in range(n):
            p = a + i
            st = {"segment_bytes": int(so[i]["segment_bytes"]), "log_start_pos": int(so[i]["log_start_pos"]),
                  "log_end_pos": int(so[i]["log_end_pos"])}
            slots = range(cfg.replication_factor) if local_slots is None else local_slots(p)
            for r in slots:
                x, y = ring_window(dev, cfg, r, p, st), ring_window(ora, cfg, r, p, st)
                if not np.array_equal(x, y):
                    bad = np.flatnonzero(x != y)
                    raise AssertionError(f"ring p={p} r={r}: {bad.size} bytes differ, first at {bad[0]}")
            m_lo = -(-st["log_start_pos"] // I)
            m_hi = st["log_end_pos"] // I
            if m_hi >= m_lo:
                cnt = m_hi - m_lo + 1
                assert np.array_equal(dev.read_index(p, m_lo, cnt), ora.read_index(p, m_lo, cnt)), f"index p={p}"
            assert np.array_equal(dev.consumer_offsets(p), ora.consumer_offsets(p)), f"consumer offsets p={p}"
