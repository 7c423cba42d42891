#!/usr/bin/env python3
"""Benchmark: committed msgs/s of the Partition-Raft append+CRC+commit path (BASELINE.json).

Workload (BASELINE.json configs[2], the metric's configuration): per GPU, 4096 partitions,
RF = 3 replicas co-located, Zipf(s = 1.1) partition load over a random permutation of ranks,
100-byte records in 65536-record batches. One step = one rmq_append of one batch: partition
ranking, offsets, CRC32C, three replica copies, sparse index, quorum commit, high watermark,
retention. Inputs are resident in HBM before timing (a pool of distinct batches larger than the
256 MiB Infinity Cache, so payload reads come from HBM). The engine applies the batches in launch
groups of --group (cfg.pipeline_depth); every batch keeps its own semantics.

Multi-GPU (config C's layout, configs[3]): one process per GPU (torch.distributed.run, or this
script spawning its ranks); GPU g leads 4096 partitions (global ids [4096 g, 4096 (g + 1))) and holds
the RF - 1 = 2 follower replicas of other GPUs' partitions, spread over all its peers
(ripplemq_amd.sharding.replica_ranks). Each launch group of appends is one replication round over
RCCL (xGMI): grouped send/recv of the round's records to the followers, CRC-checking follower
ingest, acks back into the leaders' matchIndex rows (FORMAT.md §9) -> weak scaling, records counted
once they are committed on a quorum. torch.distributed (gloo) is used only for the host barrier, the
max-over-ranks of the timed region and handing rank 0's RCCL id to the others.

roofline: achieved = algorithmic bytes per launch / mean launch duration = algorithmic bytes of
the batches applied in the timed region / the region's time between HIP events recorded on the
engine's own stream before its first and after its last launch (rmq_profile_*); algorithmic bytes
per record = (8 + L) read + RF * (16 + L) written, plus RF*8 + 16 per partition
per batch.
"""
from __future__ import annotations

import argparse
import collections
import dataclasses
import gc
import glob
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# Load the engine (and with it /opt/rocm's HIP runtime) before anything imports torch.
from ripplemq_amd._abi import RMQ_FETCH_COMMIT  # noqa: E402
from ripplemq_amd.engine import FETCH_RES_DTYPE, Engine, EngineConfig, rccl_unique_id  # noqa: E402
from ripplemq_amd.sharding import max_over_ranks, rank_view  # noqa: E402
from ripplemq_amd.rings import partition_traffic, pool_layout, ring_sizes  # noqa: E402
from ripplemq_amd.workload import CONFIGS, StreamSpec, make_batch, record_bytes  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
INDEX_INTERVAL = 1024
RING_FLOOR = 64 << 10  # smallest ring of the load policy
XGMI_LINK_GBS = 153.0  # one xGMI link, one direction; 7 per GPU in an 8-GPU node


def algorithmic_bytes(n: int, payload: float, rf: int, P: int) -> float:
    """Per batch of n records carrying `payload` bytes: (8 + L) read and RF (16 + L) written per
    record, RF * 8 + 16 per partition."""
    return n * (8 + rf * 16) + (1 + rf) * payload + P * (rf * 8 + 16)


def ring_plan(args, spec: StreamSpec, batches, view) -> dict:
    """Ring bytes of every local partition (ripplemq_amd.rings): --rings load sizes each ring from
    the traffic of the rank's input batches (retain --retain-batches batches of the partition's
    mean traffic, a 64 KiB floor); --rings equal gives every partition --segment-mb. A follower
    replica is sized like its leader (the Zipf ranking is the same on every rank)."""
    P = len(view.gp)
    if args.rings == "equal":
        seg = (args.segment_mb or 4) << 20
        return {"policy": "equal", "segment_bytes": seg, "pool_bytes": 0, "sizes": np.full(P, seg, np.uint64),
                "grown": np.zeros(0, np.uint32), "grown_bytes": np.zeros(0, np.uint64)}
    mean, peak = partition_traffic(batches, spec.partitions)
    by_local = ring_sizes(mean, peak, args.retain_batches, RING_FLOOR, INDEX_INTERVAL,
                          max_bytes=(args.segment_mb << 20) if args.segment_mb else 1 << 40)
    lay = pool_layout(by_local[np.asarray(view.gp, np.int64) % spec.partitions])
    sizes = np.maximum(by_local[np.asarray(view.gp, np.int64) % spec.partitions], np.uint64(lay.segment_bytes))
    return {"policy": "load", "segment_bytes": lay.segment_bytes, "pool_bytes": lay.pool_bytes, "sizes": sizes,
            "grown": lay.grown, "grown_bytes": lay.grown_bytes, "free_bytes": lay.free_bytes}


def ring_report(rings: dict, rf: int, group: int, P: int) -> dict:
    """HBM held by the logs and what the hottest partition retains, next to equal rings."""
    sizes = rings["sizes"]
    pool = rings["pool_bytes"] or int(sizes.sum())
    equal_same = 1 << int(np.floor(np.log2(pool / P)))  # equal power-of-two rings in the same pool
    index_bytes = (pool // INDEX_INTERVAL) * (2 * group + 2) * 16
    return {"policy": rings["policy"], "pool_bytes_per_replica": pool, "ring_bytes_total": rf * pool,
            "index_bytes": index_bytes, "hbm_total_bytes": rf * pool + index_bytes,
            "ring_bytes_min": int(sizes.min()), "ring_bytes_hot": int(sizes.max()),
            "partitions_grown": int((sizes > sizes.min()).sum()),
            "equal_ring_same_pool": equal_same, "hot_retention_vs_equal_same_pool": int(sizes.max()) / equal_same,
            "equal_16mib_total_bytes": rf * P * (16 << 20)}


def pmc_traffic(group: int, config: str):
    """HBM bytes per BATCH of the pipeline kernel from the newest committed PMC summary taken at this
    group size and config (profiles/*_pmc_traffic.json, written by tools/pmc_summary.py from the
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench; `measured_at` names the commit of the
    code it measured), or (None, None)."""
    found = (None, None)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("group") == group and d.get("config") == config and "traffic_bytes_per_batch" in d:
            src = os.path.relpath(path, REPO) + (f" (measured at {d['measured_at']})" if d.get("measured_at") else "")
            found = (d["traffic_bytes_per_batch"], src)
    return found


def cpu_baseline(spec: StreamSpec, rf: int, seg: int, budget_s: float, name: str = "B") -> dict:
    """The C oracle on a bounded sample of the workload: one thread (ro_append), then
    partitions sharded over the host cores this process may use (ro_append_sharded, pinned
    threads); `value` is the sharded rate. The rings the sample touches are first-touched before the
    timed region, as the device rings are allocated before the GPU's."""
    from oracle.oracle import OracleEngine  # cpu_baseline leg only

    cfg = EngineConfig(num_partitions=spec.partitions, replication_factor=rf, segment_bytes=seg,
                       index_interval=1024, max_batch_records=spec.records)
    distinct = [make_batch(spec, 10_000 + i) for i in range(8)]
    host = host_cpus()
    threads = host["usable"]
    recs1, t1, nb1 = 0, 0.0, 0
    with OracleEngine(cfg) as ora:
        while t1 < budget_s / 4 and nb1 < 200:
            b = distinct[nb1 % len(distinct)]
            t0 = time.perf_counter()
            _, st = ora.append(b.pidx, b.lens, b.payload)
            t1 += time.perf_counter() - t0
            assert st["appended"] == b.n, st
            recs1 += b.n
            nb1 += 1
    rate1 = recs1 / t1
    nb = int(min(1200, max(len(distinct), rate1 * budget_s / spec.records)))
    seq = [distinct[k % len(distinct)] for k in range(nb)]
    reps = np.bincount(np.arange(nb) % len(distinct), minlength=len(distinct))
    touched = np.zeros(spec.partitions, np.float64)
    for b, r in zip(distinct, reps):
        rb = 16 + (b.lens.astype(np.int64) + 15) // 16 * 16
        touched += r * np.bincount(b.pidx, weights=rb, minlength=spec.partitions)
    with OracleEngine(cfg) as ora:
        ora.reserve(np.minimum(touched, seg).astype(np.uint64))
        t0 = time.perf_counter()
        res = ora.append_sharded(seq, threads)
        tp = time.perf_counter() - t0
    assert all(st["appended"] == spec.records for _, st in res)
    return {"value": nb * spec.records / tp, "unit": "msgs/s", "cores": threads, "kind": "port",
            "single_thread_value": rate1, "single_thread_cores": 1,
            "label": "C restatement of the reference semantics (oracle/ripple_oracle.c), not the Java broker",
            "host": host,
            "sample": f"{nb} batches x {spec.records} records (config {name} stream, "
                      f"{spec.partitions} partitions, RF={rf}) through oracle/ripple_oracle.c "
                      f"ro_append_sharded: partitions sharded over {threads} pinned threads (every CPU "
                      f"this process may use), {tp:.2f} s; 1 thread (ro_append): {nb1} batches, "
                      f"{rate1 / 1e6:.2f} M msgs/s"}


def host_cpus() -> dict:
    """The GPU box's host CPUs as the baseline sees them: model, nproc, the CPUs this process may run
    on (affinity) and the cgroup CPU quota if one is set; `usable` = the CPUs a thread pool can keep
    busy (the affinity set, capped by the quota)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = max(1, min(aff, int(quota)) if quota else aff)
    return {"model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "usable": usable}


def host_leg(eng, batches, steps: int) -> dict:
    """The workload's batches handed over from HOST memory (rmq_append, RMQ_MEM_HOST): the engine
    packs each into a pinned staging slot and moves it with one DMA on its copy stream, overlapped
    with the pipeline; out offsets return through pinned memory. A PCIe-inclusive rate, reported
    beside `value` (which is HBM-resident input), never instead of it."""
    for k in range(2 * len(batches)):  # untimed: the engine sets up its staging slots
        b = batches[k % len(batches)]
        eng.append_async(b.pidx, b.lens, b.payload)
    eng.sync()
    n = batches[0].n
    h2d = 0
    t0 = time.perf_counter()
    for k in range(steps):
        b = batches[k % len(batches)]
        eng.append_async(b.pidx, b.lens, b.payload)
        h2d += 8 * b.n + b.payload.nbytes
    eng.sync()
    dt = time.perf_counter() - t0
    res = {"value": steps * n / dt, "unit": "msgs/s", "steps": steps, "h2d_gbs": h2d / dt / 1e9,
           "ms_per_step": dt * 1e3 / steps,
           "note": "host numpy batches through rmq_append: memcpy into a pinned staging slot, one "
                   "H2D DMA per batch on the copy stream, pipeline waits on its event; h2d_gbs = "
                   "pidx + len + payload bytes over the wall time"}
    # the same batches in page-locked caller memory (RMQ_MEM_PINNED: one DMA per section, no host
    # copy; out offsets written by a DMA into page-locked arrays)
    pinned = []
    for b in batches:
        arrs = (eng.host_empty(b.n, np.uint32), eng.host_empty(b.n, np.uint32), eng.host_empty(b.payload.size, np.uint8))
        arrs[0][:], arrs[1][:], arrs[2][:] = b.pidx, b.lens, b.payload
        pinned.append(arrs)
    outs = [eng.host_empty(n, np.uint64) for _ in range(16)]
    for k in range(2 * len(batches)):
        pi, le, pa = pinned[k % len(pinned)]
        eng.append_pinned_async(pi, le, pa, outs[k % 16])
    eng.sync()
    h2d = 0
    t0 = time.perf_counter()
    for k in range(steps):
        pi, le, pa = pinned[k % len(pinned)]
        eng.append_pinned_async(pi, le, pa, outs[k % 16])
        h2d += 8 * len(pi) + pa.nbytes
    eng.sync()
    dt = time.perf_counter() - t0
    res["pinned"] = {"value": steps * n / dt, "unit": "msgs/s", "steps": steps, "h2d_gbs": h2d / dt / 1e9,
                     "ms_per_step": dt * 1e3 / steps,
                     "note": "the same batches in page-locked caller memory (rmq_host_alloc, "
                             "RMQ_MEM_PINNED): one H2D DMA per section on the copy stream, no host "
                             "copy, out offsets by DMA into page-locked arrays"}
    for arrs in pinned:
        for a in arrs:
            eng.host_release(a)
    for a in outs:
        eng.host_release(a)
    return res


def mixed_engine_leg(cfg: EngineConfig, rings: dict, pool, args) -> dict:
    """The mixed leg on an engine of its own whose rings retain --mixed-retain batches of each
    partition's traffic (the bench engine's retain 64, about a millisecond of appends: consumers of
    max = 10 on hot partitions fall further behind than that within a few fetches and are reset to
    the log start). The same resident input batches; the rings filled first, untimed."""
    spec = CONFIGS[args.config]
    eng = Engine(dataclasses.replace(cfg, segment_bytes=rings["segment_bytes"], pool_bytes=rings["pool_bytes"]))
    try:
        if rings["grown"].size:
            eng.set_segments(rings["grown"], rings["grown_bytes"])
        d_out = [eng.device_alloc(spec.records * 8) for _ in range(4)]

        def step(k: int) -> int:
            n, dp, dl, dpay, pb, _ = pool[k % len(pool)]
            return eng.append_device(n, dp, dl, dpay, pb, d_out[k % len(d_out)])

        for k in range(int(args.mixed_retain) + 64):  # the rings full (and their pages touched)
            step(k)
        out = mixed_leg(eng, step, spec, args.concurrent_rounds, args.group, fetch_every=args.mixed_fetch_every)
        out["rings"] = ring_report(rings, eng.cfg.replication_factor, args.group, spec.partitions)
        out["retain_batches"] = args.mixed_retain
        for d in d_out:
            eng.device_free(d)
        return out
    finally:
        eng.close()


def mixed_leg(eng, step, spec: StreamSpec, rounds: int, appends: int, consumers: int = 4, mx: int = 10,
              fetch_every: float = 2.0) -> dict:
    """Appends and consumer fetches at once on one engine (configs[4]: concurrent consumer fetch at
    lagging offsets), driven by ONE host thread as a broker's event loop would: per round `appends`
    device-resident batches go to the pipeline, and every (partition, consumer) reads max = 10 and
    commits what it read (ConsumerClientImpl.java:61-117) through rmq_fetch_async with
    RMQ_FETCH_COMMIT: the read-then-commit of each consumer happens on the device, so the next fetch,
    ordered after it on the pipeline stream, reads on from there and four fetches can be in flight
    without a host round trip between them. Fetches are polled without waiting; every fetch runs
    between two pipeline launches (the next launch waits for it). The broker bounds its own
    run-ahead to eight launch groups (rmq_poll_commit), so a fetch returns within about eight
    launches. The consumers are paced: one read-and-commit pass of every consumer per `fetch_every`
    rounds of appends (a pass reads up to max records per consumer), so the mix of the two does not
    depend on how the host's polls happen to fall (unpaced, 106 and 258 passes over 250 rounds on
    two boxes). Reports both rates over the same wall time."""
    P = spec.partitions
    eng.sync()
    st = eng.states()
    hw = st["high_watermark"].astype(np.int64)
    retained = (st["log_end_offset"] - st["log_start_offset"]).astype(np.int64)
    g = np.random.default_rng(0x52495051)
    pp = np.repeat(np.arange(P, dtype=np.uint32), consumers)
    cc = np.tile(np.arange(consumers, dtype=np.uint32), P)
    lag = (g.random(P * consumers) * (np.repeat(retained, consumers) // 2 + 1)).astype(np.int64)
    off = (np.repeat(hw, consumers) - lag).astype(np.uint64)
    eng.commit_consumer_offset(pp, cc, off)
    # passes in flight: each waits behind the appends queued before it on the pipeline stream (up to
    # eight launch groups), so two in flight capped the passes at about one per four rounds
    inflight_f = 4
    rows = [eng.fetch_rows(P * consumers) for _ in range(inflight_f)]  # page-locked request / result rows
    for rq, _ in rows:
        rq[:, 0], rq[:, 1], rq[:, 2], rq[:, 3] = pp, cc, mx, RMQ_FETCH_COMMIT
    hi = spec.size if isinstance(spec.size, int) else spec.size[1]
    cap = P * consumers * mx * (16 + (hi + 15) // 16 * 16) + 4096
    d_out = [eng.device_alloc(cap) for _ in range(inflight_f)]
    fetched = resets = fetches = 0
    t_host = 0.0
    k0 = 10_000
    fq = collections.deque()  # (ticket, slot) of the fetches in flight, oldest first
    nslot = 0

    def take(r):
        nonlocal fetched, resets
        rc, rs, _ = r
        stt = rs["status"]
        if rc or np.any((stt != 0) & (stt != -6)):
            raise SystemExit(f"bench: mixed leg fetch failed rc={rc} statuses={np.unique(stt)}")
        fetched += int(rs["count"].sum())
        resets += int(np.count_nonzero(stt == -6))  # RMQ_EOFFSET: the ring moved past a slow
        # consumer, which resumes at the first retained offset (committed on the device)

    budget = 1.0  # passes the pacing allows so far (one per fetch_every rounds)

    def service() -> bool:
        """Completed fetches in, new ones out (at most inflight_f in flight). False if nothing moved."""
        nonlocal fetches, t_host, nslot, budget
        t1 = time.perf_counter()
        moved = False
        while fq:
            r = eng.fetch_poll(fq[0][0], wait=False)
            if r is None:
                break
            take(r)
            fq.popleft()
            moved = True
        while len(fq) < inflight_f and budget >= 1.0:
            budget -= 1.0
            k = nslot % inflight_f
            nslot += 1
            fq.append((eng.fetch_async(None, None, None, d_out=d_out[k], out_cap=cap, req=rows[k][0], res=rows[k][1],
                                       pinned_rows=True), k))
            fetches += 1
            moved = True
        t_host += time.perf_counter() - t1
        return moved

    t0 = time.perf_counter()
    service()
    window = 8 * appends
    inflight = collections.deque()
    for k in range(rounds):
        for j in range(appends):
            while len(inflight) >= window:
                if eng.poll(inflight[0]) is not None:
                    inflight.popleft()
                elif not service():
                    time.sleep(0)
            inflight.append(step(k0 + k * appends + j))
        budget += 1.0 / fetch_every
        service()
    while fq:
        take(eng.fetch_poll(fq.popleft()[0], wait=True))
    eng.sync()
    dt = time.perf_counter() - t0
    for d in d_out:
        eng.device_free(d)
    for rq, rs in rows:
        eng.host_release(rq)
        eng.host_release(rs)
    recs = rounds * appends * spec.records
    return {"append_msgs_per_s": recs / dt, "fetch_records_per_s": fetched / dt, "rounds": rounds,
            "appends_per_round": appends, "fetches": fetches, "fetch_every_rounds": fetch_every,
            "requests_per_fetch": P * consumers,
            "max_records": mx, "wall_s": dt, "consumer_host_s": t_host,
            "lag_bound": "U[0, retained records / 2] per partition at the start",
            "consumer_resets": resets,
            "note": "one host thread: appends (device-resident batches, at most 8 launch groups not yet "
                    "complete) and, between them, every consumer's read-and-commit at max = 10 through "
                    "rmq_fetch_async with RMQ_FETCH_COMMIT (four fetches in flight, polled without "
                    f"waiting; one pass of every consumer per {fetch_every:g} rounds of appends); both "
                    "rates over the same wall time; consumers start lagging the high "
                    "watermark by U[0, lag_bound] (configs[4] names U[0, 10^6]: that lag is not "
                    "HBM-resident at 4,096 partitions, so it is bounded by what the rings retain)"}


def tier_leg(eng, step, spec: StreamSpec, rounds: int, appends: int, parts: int = 4096, consumers: int = 4) -> dict:
    """The durable tier (ripplemq_amd/tier.py) on the bench engine: the first
    `parts` partitions' committed records spill to segment files (one rmq_fetch per spill, the
    native record scan, one file append per partition) while the workload appends: per round one
    launch group of batches, then a spill. Then consumers lagging BELOW the rings (configs[4]'s
    U[0, 10^6] lag: offsets the rings no longer hold) are served from the files at max = 1024
    (DurableLog.read_images: the record images, as rmq_fetch returns them; PartitionBroker's
    process_batch_read falls back to DurableLog.read on RMQ_EOFFSET). Both timed on the host; the
    record bytes counted are the FORMAT.md §1 images written / read."""
    import shutil
    import tempfile

    from ripplemq_amd.tier import DurableLog

    stride = max(1, spec.partitions // parts)  # every stride-th partition: an even sample of the Zipf ranks
    pidx = np.arange(0, spec.partitions, stride, dtype=np.uint32)
    P = len(pidx)
    cursor = eng.cfg.max_consumers - 1  # keys the replica reads' position cache
    eng.sync()
    st = eng.states()[pidx]
    root = tempfile.mkdtemp(prefix="rmq_tier_", dir=os.environ.get("RMQ_TIER_DIR"))
    try:
        # attached to a running engine: each partition's files start at its current log start
        tier = DurableLog(eng, root, pidx, cursor, segment_file_bytes=256 << 20, start=st["log_start_offset"])
        first = tier.spill()  # untimed: the retained windows at the start
        size0 = sum(int(f.pos[-1]) for f in tier.parts.values())
        tier.phase_s.clear()
        spilled, t_spill, k0 = 0, 0.0, 500_000
        for k in range(rounds):
            for j in range(appends):
                step(k0 + k * appends + j)
            t0 = time.perf_counter()
            spilled += tier.spill()
            t_spill += time.perf_counter() - t0
        sbytes = sum(int(f.pos[-1]) for f in tier.parts.values()) - size0
        eng.sync()
        st = eng.states()
        g = np.random.default_rng(0x5249504C)
        reqs = []
        for p in pidx.tolist():
            f = tier.parts[p]
            lo, hi = f.base, min(int(st["log_start_offset"][p]), f.end)
            if hi > lo:
                reqs += [(p, int(o)) for o in g.integers(lo, hi, consumers)]
        if len(reqs) > 4096:  # a sample of them
            reqs = [reqs[i] for i in g.choice(len(reqs), 4096, replace=False)]
        recs = rbytes = 0
        t0 = time.perf_counter()
        for p, off in reqs:
            n, img = tier.read_images(p, off, 1024)
            recs += n
            rbytes += len(img)
        t_read = time.perf_counter() - t0
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return {"partitions": P, "partition_stride": stride, "rounds": rounds, "appends_per_round": appends,
            "spill": {"records": spilled, "records_per_s": spilled / t_spill if t_spill else None,
                      "gb_per_s": sbytes / t_spill / 1e9 if t_spill else None, "initial_records": first,
                      "ms_per_spill": t_spill * 1e3 / max(rounds, 1),
                      "ms_per_spill_phases": {k: v * 1e3 / max(rounds, 1) for k, v in tier.phase_s.items()}},
            "read_below_rings": {"requests": len(reqs), "records": recs,
                                 "records_per_s": recs / t_read if t_read else None,
                                 "gb_per_s": rbytes / t_read / 1e9 if t_read else None, "max_records": 1024},
            "note": "host-side tier over the engine (spill = one rmq_fetch of the partitions' new records, "
                    "segment-file appends, the consumer table and terms in bulk, one ends file); reads "
                    "are consumers below the rings' retained windows served from the files"}


REPLAY = 4  # fetch kernel runs per timed fetch (rmq_profile_enable(k))


def fetch_leg(eng, spec: StreamSpec, rounds: int, consumers: int = 4) -> dict:
    """Consumer fetch over the bench engine's committed logs (SURVEY §8(d) B_fetch): per round every
    (partition, consumer) commits an offset lagging the high watermark by U[0, retained records]
    (config D's lagging consumers, bounded by what retention keeps), then one rmq_fetch of all
    P x consumers requests into a device buffer, at max = 10 (ConsumerClientImpl.java:21) and
    max = 1024. Timed with HIP events around the fetch kernels on the pipeline stream they run on.
    B_fetch = 2 (16 + L) per returned record (read log, write output) + 8 ceil(log2(index entries))
    per request."""
    P = spec.partitions
    st = eng.states()  # one bulk read-back of every partition's state
    hw = st["high_watermark"].astype(np.int64)
    lo = st["log_start_offset"].astype(np.int64)
    span = (st["log_end_pos"] - st["log_start_pos"]).astype(np.int64)
    idx_entries = np.maximum(1, span // 1024 + 1)
    search_bytes = int((8 * np.ceil(np.log2(idx_entries + 1))).sum()) * consumers
    g = np.random.default_rng(0x52495050)
    pp = np.repeat(np.arange(P, dtype=np.uint32), consumers)
    cc = np.tile(np.arange(consumers, dtype=np.uint32), P)
    out = {"lag_bound": "U[0, retained records] per (partition, consumer): configs[4]'s U[0, 10^6] is not "
                        "HBM-resident at 4,096 partitions"}
    for mx in (10, 1024):
        hi = spec.size if isinstance(spec.size, int) else spec.size[1]
        retained = int(span.sum())
        cap = min(P * consumers * mx * (16 + (hi + 15) // 16 * 16), consumers * retained) + 4096
        d_out = eng.device_alloc(cap)
        recs = nbytes = 0
        t_kern = t_wall = t_reg = 0.0
        t_calls = []
        # untimed calls first: a process's first launch of a kernel loads its code object
        # (~20 ms, measured between the first resolve and gather in profiles/r03q_prof), and each
        # of the engine's four fetch slots allocates its scratch on first use
        for _ in range(4):
            eng.fetch_device(pp, cc, np.full(P * consumers, mx, np.uint32), d_out, cap)
        # and every consumer-commit staging slot once (each allocates its pinned and device buffers
        # on first use; one of them, on some boxes, stalled the next fetch by ~8 ms)
        for _ in range(16):
            eng.commit_consumer_offset(pp, cc, np.zeros(P * consumers, np.uint64))
        eng.sync()
        # the request and result rows in page-locked arrays, reused from call to call
        # (RMQ_FETCH_PINNED_ROWS: DMA both ways, no host copy)
        rows = [eng.fetch_rows(P * consumers) for _ in range(8)]
        for rq, _ in rows:
            rq[:, 0], rq[:, 1], rq[:, 2] = pp, cc, mx
        # the kernel measurement's rows in device memory (RMQ_FETCH_DEVICE_ROWS: no PCIe inside the
        # timed kernels, as the append bench's inputs are resident); the calls below use host rows
        n_rq = P * consumers
        d_req, d_res = eng.device_alloc(16 * n_rq), eng.device_alloc(32 * n_rq)
        eng.h2d(d_req, rows[0][0])
        res = np.empty(n_rq, FETCH_RES_DTYPE)
        for k in range(rounds):
            lag = (g.random(P * consumers) * (np.repeat(hw - lo, consumers) + 1)).astype(np.int64)
            eng.commit_consumer_offset(pp, cc, (np.repeat(hw, consumers) - lag).astype(np.uint64))
            # one synchronous rmq_fetch as an application makes it (page-locked rows, results in place),
            # timed once the round's offset commit is applied (a fetch commits nothing here, so the
            # calls below see the same offsets)
            eng.sync()
            gc.disable()  # (as timeit does: a collector pass is not the call's cost)
            t0 = time.perf_counter()
            rc_c, _, _ = eng.fetch_device(None, None, None, d_out, cap, req=rows[0][0], res=rows[0][1], pinned_rows=True)
            t_calls.append(time.perf_counter() - t0)
            t_wall += t_calls[-1]
            gc.enable()
            if os.environ.get("RMQ_BENCH_CALLS"):  # diagnostic: each timed call's wall time
                print(f"bench: fetch max {mx} call {(time.perf_counter() - t0) * 1e6:.1f} us", file=sys.stderr)
            eng.profile(True)
            rc, _, used = eng.fetch_device(None, None, None, d_out, cap, d_rows=(n_rq, d_req, d_res))
            _, ms_f = eng.profile_query(3)  # the kernels' own dispatch-recorded spans, summed
            eng.profile(False)
            eng.d2h(res, d_res)
            # kernel time: the same fetch's kernels run REPLAY times back to back between two events
            # (idempotent; rows on the device), so no transfer, host gap or early-dispatch span enters
            # it, and a rocprofv3 trace shows the same kernels back to back
            eng.profile(REPLAY)
            eng.fetch_device(None, None, None, d_out, cap, d_rows=(n_rq, d_req, d_res))
            runs, ms_all = eng.profile_query(4)
            ms_r = ms_all / max(runs, 1)
            eng.profile(False)
            if rc or rc_c or np.any(res["status"] != 0) or not np.array_equal(rows[0][1]["count"], res["count"]):
                raise SystemExit(f"bench: fetch leg failed rc={rc} statuses={np.unique(res['status'])}")
            t_kern += ms_f / 1e3
            t_reg += ms_r / 1e3
            recs += int(res["count"].sum())
            nbytes += int(res["bytes"].sum())
        # the same requests as 8 asynchronous calls back to back (rmq_fetch_async: 4 in flight, the
        # host never waits on the GPU between issues; pinned rows), first issue to last result
        # (three bursts: the median, as for the single calls below, so that one host stall of a
        # few ms — seen once per run at random points on some boxes — does not stand for the rate)
        bursts = []
        for _ in range(3):
            eng.sync()
            gc.disable()
            t0 = time.perf_counter()
            tks = [eng.fetch_async(None, None, None, d_out=d_out, out_cap=cap, req=rq, res=rs, pinned_rows=True)
                   for rq, rs in rows]
            t_iss = time.perf_counter() - t0
            n_async = sum(int(eng.fetch_poll(t, wait=True)[1]["count"].sum()) for t in tks)
            bursts.append(n_async / (time.perf_counter() - t0))
            gc.enable()
            if os.environ.get("RMQ_BENCH_CALLS"):
                print(f"bench: fetch max {mx} burst issue {t_iss * 1e6:.1f} us total {n_async / bursts[-1] * 1e6:.1f} us "
                      f"records {n_async}", file=sys.stderr)
        eng.device_free(d_out)
        eng.device_free(d_req)
        eng.device_free(d_res)
        for rq, rs in rows:
            eng.host_release(rq)
            eng.host_release(rs)
        # B_fetch = 2 (H + L) per returned record (fixed-size configs: exact; mixed
        # sizes: the records' bytes in the log layout, which adds their padding to 16 bytes)
        rec_bytes = recs * (16 + spec.size) if isinstance(spec.size, int) else nbytes
        alg = 2 * rec_bytes + search_bytes * rounds
        # the dispatch-recorded span of a launch starts when the command processor takes its packet,
        # which can precede the end of the work before it on the stream (the request copy), so
        # spans overstate kernel time; the roofline uses the replayed kernels' region instead
        # per call: the median call's time (the mean over all calls beside it)
        out[f"max{mx}"] = {"records_per_s_kernels": recs / t_reg,
                           "records_per_s_call": recs / rounds / float(np.median(t_calls)),
                           "records_per_s_call_mean": recs / t_wall,
                           "call_us": [round(x * 1e6, 1) for x in t_calls],
                           "records_per_s_async_calls": float(np.median(bursts)),
                           "records_per_s_async_bursts": bursts,
                           "records_per_request": recs / (rounds * P * consumers),
                           "requests": P * consumers, "rounds": rounds,
                           "roofline": {"bound": "hbm", "achieved": alg / t_reg / 1e9, "peak": HBM_PEAK_GBS,
                                        "unit": "GB/s", "frac": alg / t_reg / 1e9 / HBM_PEAK_GBS,
                                        "kernels": "rmq::fetch_resolve (two requests per wave) + fetch_gather (placement fused)",
                                        "mean_us_per_fetch": t_reg / rounds * 1e6,
                                        "timing": f"per fetch: its kernels run {REPLAY}x back to back between two "
                                                  "HIP events on the pipeline stream, divided by the runs",
                                        "kernel_spans_us_summed": t_kern / rounds * 1e6}}
    out["loop10"] = consumer_loop(eng, spec, pp, cc, hw, lo, g, rounds * 4)
    return out


def consumer_loop(eng, spec: StreamSpec, pp, cc, hw, lo, g, loops: int, mx: int = 10) -> dict:
    """The consumer loop (ConsumerClientImpl.java:61-117): every (partition, consumer) reads max = 10
    and commits what it read, round after round, through RMQ_FETCH_COMMIT (the commit happens on
    the device), from a lag of U[0, retained records]. Each fetch reads on from the end of the one
    before, whose ring position the engine's position cache holds (fetch.hip): the resolve walks
    from there instead of searching the index. A committing fetch runs once (no replay) and needs
    host rows (the call checks them): the rows are page-locked and the kernels read and write them
    across PCIe, so this rate includes that transfer; timed by HIP events around the one run."""
    n = len(pp)
    lag = (g.random(n) * (np.repeat(hw - lo, n // len(hw)) + 1)).astype(np.int64)
    eng.commit_consumer_offset(pp, cc, (np.repeat(hw, n // len(hw)) - lag).astype(np.uint64))
    hi = spec.size if isinstance(spec.size, int) else spec.size[1]
    cap = n * mx * (16 + (hi + 15) // 16 * 16) + 4096
    d_out = eng.device_alloc(cap)
    rq, rs = eng.fetch_rows(n)
    rq[:, 0], rq[:, 1], rq[:, 2], rq[:, 3] = pp, cc, mx, RMQ_FETCH_COMMIT
    eng.sync()
    eng.fetch_device(None, None, None, d_out, cap, req=rq, res=rs, pinned_rows=True)  # the cache's first entries
    recs = nbytes = 0
    t_reg = 0.0
    t_calls = []
    for _ in range(loops):
        eng.profile(True)
        gc.disable()
        t0 = time.perf_counter()
        rc, _, _ = eng.fetch_device(None, None, None, d_out, cap, req=rq, res=rs, pinned_rows=True)
        t_calls.append(time.perf_counter() - t0)
        gc.enable()
        runs, ms = eng.profile_query(4)
        eng.profile(False)
        if rc or np.any(rs["status"] != 0):
            raise SystemExit(f"bench: consumer loop fetch failed rc={rc} statuses={np.unique(rs['status'])}")
        t_reg += ms / 1e3
        recs += int(rs["count"].sum())
        nbytes += int(rs["bytes"].sum())
    eng.device_free(d_out)
    eng.host_release(rq)
    eng.host_release(rs)
    rec_bytes = recs * (16 + spec.size) if isinstance(spec.size, int) else nbytes
    alg = 2 * rec_bytes
    return {"requests": n, "loops": loops, "max_records": mx, "records_per_request": recs / (loops * n),
            "records_per_s_kernels": recs / t_reg, "records_per_s_call": recs / loops / float(np.median(t_calls)),
            "call_us_median": float(np.median(t_calls)) * 1e6,
            "roofline": {"bound": "hbm", "achieved": alg / t_reg / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / t_reg / 1e9 / HBM_PEAK_GBS, "mean_us_per_fetch": t_reg / loops * 1e6,
                         "timing": "per fetch: HIP events around its kernels (one run; page-locked host rows, "
                                   "read and written across PCIe by the kernels)",
                         "bytes": "B_fetch = 2 (16 + L) per returned record (no index search on a cache hit)"}}


class SoloGroup:
    """One rank: the identity group."""
    world = 1
    rank = 0

    def barrier(self):
        pass

    def max(self, x: float) -> float:
        return float(x)

    def bcast(self, obj):
        return obj


class DistGroup:
    """One process per GPU: host barrier / max / broadcast over torch.distributed (gloo)."""

    def __init__(self, dist):
        self.dist = dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()

    def barrier(self):
        self.dist.barrier()

    def max(self, x: float) -> float:
        return max_over_ranks(x, self.dist)

    def bcast(self, obj):
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]


class ThreadGroup:
    """Ranks as threads of one process (--transport local: engines on one GPU, in-process hub)."""

    def __init__(self, world: int):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world

    def view(self, rank: int):
        g = self

        class _Rank:
            world = g.world

            def __init__(self):
                self.rank = rank

            def barrier(self):
                g.bar.wait()

            def max(self, x: float) -> float:
                g.slots[rank] = float(x)
                g.bar.wait()
                m = max(g.slots)
                g.bar.wait()
                return m

            def bcast(self, obj):
                if rank == 0:
                    g.slots[0] = obj
                g.bar.wait()
                v = g.slots[0]
                g.bar.wait()
                return v

        return _Rank()


def run_rank(args, grp, device: int, attach) -> dict | None:
    """One rank's engine, resident input pool, timed region and (rank 0) the JSON line."""
    rank, world = grp.rank, grp.world
    spec = CONFIGS[args.config]
    rf = 5 if args.config == "D" else 3  # configs[4]: RF = 5
    if args.config == "D" and world > 1:  # configs[4]: 4,096 partitions over the node, not per GPU
        spec = dataclasses.replace(spec, partitions=max(1, spec.partitions // world))
    L = spec.size if isinstance(spec.size, int) else None
    view = rank_view(rank, world, spec.partitions, rf)  # world 1: every replica on this GPU
    # the rank's distinct input batches (rank-salted stream keys), made before the engine so that
    # the rings can be sized from their traffic
    batches = [make_batch(spec, 1_000_000 * rank + q) for q in range(args.pool)]
    max_payload = max(int(b.payload.nbytes) for b in batches)
    rings = ring_plan(args, spec, batches, view)
    # the mixed leg's engine: rings that retain --mixed-retain batches (consumers of max = 10 lag the
    # appends on hot partitions; the ring is how far they may fall behind before a reset)
    rings_mixed = (ring_plan(argparse.Namespace(**{**vars(args), "retain_batches": args.mixed_retain}), spec, batches,
                             view)
                   if args.concurrent_rounds > 0 and world == 1 else None)
    cfg = EngineConfig(num_partitions=len(view.gp), replication_factor=rf,
                       segment_bytes=rings["segment_bytes"], pool_bytes=rings["pool_bytes"],
                       index_interval=INDEX_INTERVAL, max_batch_records=spec.records,
                       max_batch_bytes=max(8 << 20, (max_payload + (1 << 20) - 1) >> 20 << 20),
                       pipeline_depth=args.group, device=device, rank=rank)
    eng = Engine(cfg)
    if world > 1:
        attach(eng, grp)
        eng.set_placement(np.arange(len(view.gp), dtype=np.uint32), view.gp, view.ranks, view.leader_slot)
    if rings["grown"].size:  # collective with a transport: every rank grows its rings here
        eng.set_segments(rings["grown"], rings["grown_bytes"])
    dev_name, cus = eng.device_info()

    # resident input pool
    pool = []
    # one device region for the whole pool (a broker's receive ring), or an allocation per array
    sizes = [(b.n * 4, b.n * 4, max(b.payload.nbytes, 4)) for b in batches]
    rnd = lambda x: (x + 4095) // 4096 * 4096  # noqa: E731
    region = eng.device_alloc(sum(rnd(x) for z in sizes for x in z)) if args.inputs == "region" else None
    at = 0

    def carve(nbytes: int) -> int:
        nonlocal at
        if region is None:
            return eng.device_alloc(nbytes)
        at += rnd(nbytes)
        return region + at - rnd(nbytes)

    for b in batches:
        d_pidx = carve(b.n * 4)
        d_len = carve(b.n * 4)
        d_pay = carve(max(b.payload.nbytes, 4))
        eng.h2d(d_pidx, b.pidx)
        eng.h2d(d_len, b.lens)
        eng.h2d(d_pay, b.payload)
        pool.append((b.n, d_pidx, d_len, d_pay, int(b.payload.nbytes), record_bytes(b.lens)))
    mean_payload = float(np.mean([b.payload.nbytes for b in batches]))
    host_batches = batches[:8]
    del batches
    d_out = [eng.device_alloc(spec.records * 8) for _ in range(4)]

    def step(k: int) -> int:
        n, dp, dl, dpay, pb, _ = pool[k % len(pool)]
        return eng.append_device(n, dp, dl, dpay, pb, d_out[k % len(d_out)])

    def barrier():
        eng.sync()  # collective with a transport: every rank flushes the same rounds
        grp.barrier()

    for k in range(args.warmup):
        step(k)
    barrier()
    eng.profile(True)  # HIP events bracket the timed region's launches on the engine's stream
    x0 = eng.replication_stats()
    t0 = time.perf_counter()
    last = 0
    for k in range(args.steps):
        last = step(args.warmup + k)
    t_issue = time.perf_counter() - t0  # host time to submit the steps (diagnostic)
    barrier()
    elapsed = time.perf_counter() - t0
    x1 = eng.replication_stats()
    n_launch, region_ms = eng.profile_query(0)
    n_applied, _ = eng.profile_query(1)
    st = eng.wait(last) if last else {}
    # RMQ_DEBUG timing experiments skip work on purpose: their lines are marked and never checked
    timing_only = os.environ.get("RMQ_DEBUG", "0") not in ("", "0")
    if st and st.get("appended") != spec.records and not timing_only:
        raise SystemExit(f"bench: last batch not fully appended ({st}); the measurement would be void")
    eng.profile(False)
    committed = int(eng.commit_snapshot()[:view.led].sum(dtype=np.uint64))
    if committed != spec.records * (args.warmup + args.steps) and not timing_only:
        raise SystemExit(f"bench: {committed} records committed of {spec.records * (args.warmup + args.steps)} "
                         "appended; the measurement would be void")

    t_max = grp.max(elapsed)
    sent_max = grp.max(float(x1["bytes_sent"] - x0["bytes_sent"]))
    waits_max = grp.max(float(x1["host_waits"] - x0["host_waits"]))
    wait_ms_max = grp.max(float(x1["host_wait_ns"] - x0["host_wait_ns"]) / 1e6)
    if grp.max(float(x1["refused_crc"] + x1["refused_log"])):
        raise SystemExit("bench: a follower refused replication rounds; the measurement would be void")

    n = spec.records
    total_records = n * args.steps * world
    msgs_per_s = total_records / t_max
    out = None
    if rank == 0:
        alg = algorithmic_bytes(n, mean_payload, rf, spec.partitions)
        # algorithmic bytes per launch / mean launch duration = bytes of the applied batches / region
        achieved = alg * n_applied / (region_ms / 1e3) / 1e9 if n_launch and region_ms > 0 else 0.0
        traffic_b, traffic_src = pmc_traffic(args.group, args.config)
        bpl = n_applied / max(n_launch, 1)
        # per launch of THIS run (its launches average bpl batches), from the per-batch PMC figure
        traffic = traffic_b * bpl if traffic_b else None
        out = {
            "metric": "committed msgs/sec (node) + HBM GB/s, 100B msgs, 4096 partitions RF=3",
            "value": msgs_per_s,
            "unit": "msgs/s",
            "n_gpus": world if args.transport != "local" else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max * 1e3 / args.steps,
            "host_issue_us_per_step": t_issue * 1e6 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic" if not timing_only else f"INVALID timing experiment RMQ_DEBUG={os.environ['RMQ_DEBUG']}",
            "config": {"workload": f"config {args.config}: {spec.partitions} partitions/GPU, RF={rf}, "
                                   f"{spec.mode}{'(s=%.1f)' % spec.zipf_s if spec.mode == 'zipf' else ''}, "
                                   f"{L if L else '%d-%d' % spec.size} B records, {n} records/batch",
                       "partitions_per_gpu": spec.partitions, "replication_factor": rf,
                       "records_per_batch": n, "record_payload_bytes": L,
                       "parallelism": (f"partition-sharded x{world}, RF={rf} replicas over "
                                       + ("xGMI (RCCL)" if args.transport == "rccl" else
                                          "the in-process transport on ONE GPU (functional rehearsal)")
                                       if world > 1 else f"1 GPU, RF={rf} replicas co-located"),
                       "batches_per_launch_group": args.group,
                       "rings": ring_report(rings, rf, args.group, len(view.gp))},
            "hbm_gbs_pipeline": alg * args.steps * world / t_max / 1e9,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_per_batch": traffic_b,
                         "traffic_source": traffic_src,
                         "kernel": "rmq::pipeline_kernel",
                         "algorithmic_bytes_per_launch": alg * n_applied / max(n_launch, 1),
                         "mean_kernel_us": region_ms * 1e3 / max(n_launch, 1), "timed_launches": n_launch,
                         "batches_per_launch": n_applied / max(n_launch, 1)},
            "xgmi": None if world == 1 else {
                "bytes_sent_per_gpu_max": sent_max, "achieved": sent_max / t_max / 1e9,
                "host_waits_for_round_sizes": int(waits_max), "host_wait_ms": wait_ms_max,
                # the in-process transport copies inside one GPU: no link is measured
                "peak": None if args.transport == "local" else XGMI_LINK_GBS * (world - 1), "unit": "GB/s",
                "frac": None if args.transport == "local" else sent_max / t_max / 1e9 / (XGMI_LINK_GBS * (world - 1)),
                "note": ("round regions sent per rank (records + record table + directories) over the timed region; "
                         "in-process transport: device copies on one GPU, not an xGMI rate")
                        if args.transport == "local" else
                        "round regions sent per GPU (records + record table + directories) over the timed "
                        "region / the links to the job's other GPUs (one direction)",
                "rounds": x1["rounds"] - x0["rounds"],
                "general_plans": x1["general_plans"] - x0["general_plans"],
                "catchup_entries": x1["catchup_entries"] - x0["catchup_entries"]},
            "append_stats_last": st,
            "device": dev_name,
            "cu_count": cus,
        }
        if args.host_steps > 0 and world == 1:
            out["host_path"] = host_leg(eng, host_batches, args.host_steps)
        # the side legs measure one GPU's engine (at N > 1 rank 0 leads only its share of the
        # partitions, and a rank-0-only rmq_sync could not be collective)
        if args.fetch_rounds > 0 and world == 1:
            out["fetch"] = fetch_leg(eng, spec, args.fetch_rounds)
        if args.concurrent_rounds > 0 and world == 1:
            out["mixed"] = mixed_engine_leg(cfg, rings_mixed, pool, args)
        if args.tier_rounds > 0 and world == 1:
            out["tier"] = tier_leg(eng, step, spec, args.tier_rounds, args.group)
    if region is not None:
        eng.device_free(region)
    else:
        for _, dp, dl, dpay, _, _ in pool:
            eng.device_free(dp)
            eng.device_free(dl)
            eng.device_free(dpay)
    for d in d_out:
        eng.device_free(d)
    eng.close()
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(spec, rf, 4 << 20, args.cpu_budget, args.config)
        else:
            out["cpu_baseline"] = None
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS))
    ap.add_argument("--pool", type=int, default=48, help="distinct resident input batches")
    ap.add_argument("--inputs", default="arrays", choices=["arrays", "region"],
                    help="input pool: a device allocation per array, or one region carved into batches")
    ap.add_argument("--rings", default="load", choices=["load", "equal"],
                    help="load: ring per partition from its traffic in one shared pool (rmq_set_segments); "
                         "equal: every ring --segment-mb (default 4)")
    ap.add_argument("--mixed-retain", type=float, default=1024.0,
                    help="mixed leg: batches of a partition's mean traffic its rings retain (own engine)")
    ap.add_argument("--retain-batches", type=float, default=64.0,
                    help="load policy: batches of a partition's mean traffic its ring retains")
    ap.add_argument("--segment-mb", type=int, default=None,
                    help="equal policy: ring bytes per (replica, partition) [MiB], default 4 (16 MiB rings span "
                         "192 GiB and the first launches of a process run up to 1.5x slower until the "
                         "translation caches warm); load policy: the largest ring [MiB]")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fetch-rounds", type=int, default=10, help="rounds of the fetch leg (0: skip)")
    ap.add_argument("--concurrent-rounds", type=int, default=250,
                    help="rounds of the append+fetch mixed leg (1 GPU; 0: skip)")
    ap.add_argument("--mixed-fetch-every", type=float, default=2.0,
                    help="mixed leg: rounds of appends per read-and-commit pass of every consumer")
    ap.add_argument("--tier-rounds", type=int, default=20,
                    help="rounds of the durable-tier leg (spills + reads below the rings, 1 GPU; 0: skip)")
    ap.add_argument("--host-steps", type=int, default=100,
                    help="batches of the host-memory leg (PCIe-inclusive rate, 1 GPU; 0: skip)")
    ap.add_argument("--watchdog", type=float, default=900.0, help="multi-GPU: exit a rank stuck this long [s]")
    ap.add_argument("--group", type=int, default=4,
                    help="batches per pipeline launch group (cfg.pipeline_depth, 1..8)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "local"],
                    help="local: --gpus ranks as threads on ONE GPU over the in-process transport "
                         "(functional rehearsal of the multi-GPU path; never a scaling number)")
    args = ap.parse_args()

    if args.transport == "local":
        from ripplemq_amd.engine import LocalHub

        world = args.gpus
        hub = LocalHub(world)
        tg = ThreadGroup(world)
        outs, errs = [None] * world, [None] * world

        def body(r):
            try:
                outs[r] = run_rank(args, tg.view(r), 0, lambda eng, grp: eng.attach_local(hub))
            except BaseException as ex:  # noqa: BLE001 - reported below
                errs[r] = ex

        ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for ex in errs:
            if ex is not None:
                raise ex
        print(json.dumps(outs[0]), flush=True)
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start one rank process per GPU ourselves, before this process touches HIP
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        procs = []
        for r in range(args.gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                       LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
        rcs = [p.wait() for p in procs]
        sys.exit(next((rc for rc in rcs if rc), 0))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: the line would misreport n_gpus")
    grp = SoloGroup()
    dist = None
    if world > 1:
        # a rank that waits on a peer forever (a collective out of step) must not hold the node
        wd = threading.Timer(args.watchdog, lambda: (print(f"bench: rank {os.environ.get('RANK')} watchdog "
                                                           f"after {args.watchdog} s", file=sys.stderr, flush=True),
                                                     os._exit(3)))
        wd.daemon = True
        wd.start()
        import torch.distributed as dist  # host-side barrier / max / id broadcast only (gloo)

        dist.init_process_group("gloo")
        grp = DistGroup(dist)

    def attach_rccl(eng, g):
        eng.attach_rccl(g.bcast(rccl_unique_id() if g.rank == 0 else None), g.world)

    device = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RMQ_BENCH_DEVICES"):  # rehearsal only: ranks share the box's few GPUs
        device %= int(os.environ["RMQ_BENCH_DEVICES"])
    out = run_rank(args, grp, device, attach_rccl)
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
