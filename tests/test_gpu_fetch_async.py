"""rmq_fetch_async / rmq_fetch_poll (ABI 6), page-locked rows (ABI 7) and the fetch kernels.

An asynchronous fetch is ordered exactly like rmq_fetch (after every launch issued before it,
before the ones issued after it), so its result must equal a synchronous fetch issued right after
it (whose parity with the oracle test_gpu_pinned.py checks; PartitionStateMachine.java:85-110;
MessageBatchReadRequestProcessor.java:36-42 answers each read from its own closure: the ticket is
that completion). The fetch kernels (a resolve of two requests per wave,
a gather with placement) must give the oracle's results on the same requests, ENOSPC cuts and
bad requests included.
"""
from __future__ import annotations

import numpy as np
import pytest

from parity import run_ops
from ripplemq_amd import _abi as A
from ripplemq_amd.engine import FETCH_RES_DTYPE, Engine, EngineConfig, EngineError
from ripplemq_amd.workload import StreamSpec, make_batch

pytestmark = pytest.mark.gpu


def test_async_fetch_matches_sync_while_appending():
    P = 64
    cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=1 << 18, index_interval=256,
                       max_consumers=2, max_batch_records=4096, pipeline_depth=2)
    spec = StreamSpec(P, 3000, "zipf", size=(1, 300), config_index=44)
    batches = [make_batch(spec, b) for b in range(14)]
    pp = np.arange(P, dtype=np.uint32)
    g = np.random.default_rng(3)
    with Engine(cfg) as dev:
        pending = []
        for k, b in enumerate(batches):
            dev.append_async(b.pidx, b.lens, b.payload)
            if k % 3 == 2:  # consumer 1 moves; its commit is ordered before the next fetches
                dev.commit_consumer_offset(pp, np.ones(P, np.uint32), g.integers(0, 40 * k, P).astype(np.uint64))
            cc = np.full(P, k & 1, np.uint32)
            mx = np.full(P, 1 << 20, np.uint32)
            if k % 2:  # host output (copied back at poll time) / device output
                out = np.zeros(2 << 20, np.uint8)
                tk = dev.fetch_async(pp, cc, mx, out=out, out_cap=out.size)
            else:
                d_out = dev.device_alloc(2 << 20)
                tk = dev.fetch_async(pp, cc, mx, d_out=d_out, out_cap=2 << 20)
            _, res, buf, _ = dev.fetch(pp, cc, mx)  # the same requests, ordered right after it
            pending.append((k, tk, res.copy(), buf.copy(), None if k % 2 else d_out))
        # more than four in flight: the oldest were completed into their arrays when slots ran out
        first = dev.fetch_poll(pending[-1][1], wait=False)  # may be pending or done
        got_first = first is not None
        for k, tk, want, wbuf, d_out in pending[::-1]:
            if got_first and tk is pending[-1][1]:
                r = first
            else:
                r = dev.fetch_poll(tk, wait=True)
            assert r is not None
            _, res, used = r
            for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                assert np.array_equal(res[f], want[f]), (k, f)
            assert used == int(want["bytes"].sum())
            if d_out is None:
                assert np.array_equal(tk.out[:used], wbuf[:used]), k
            else:
                got = np.empty(used, np.uint8)
                dev.d2h(got, d_out)
                assert np.array_equal(got, wbuf[:used]), k
                dev.device_free(d_out)
        with pytest.raises(EngineError) as ei:  # answered once
            dev.fetch_poll(pending[0][1], wait=True)
        assert ei.value.status == A.RMQ_EINVAL
        dev.sync()


def test_coalesced_async_fetches(oracle_mod):
    """Asynchronous fetches that commit nothing are held back and launched together, up to four
    tickets in one resolve + gather pair (engine.cpp fetch_flush); a committing fetch, any other call,
    a fifth ticket or a poll launches the held ones first. Every ticket's results, bytes and the
    consumer table equal the oracle's, which runs the same calls one after the other."""
    P, C = 64, 4
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 18, index_interval=256,
                       max_consumers=C, max_batch_records=4096, pipeline_depth=2)
    spec = StreamSpec(P, 3000, "zipf", size=(1, 300), config_index=58)
    g = np.random.default_rng(58)
    pp = np.arange(P, dtype=np.uint32)
    # (kind, args): "f" async fetch (consumer, max, commit, device output), "a" append, "s" sync fetch
    ops = [("a", 0), ("a", 1), ("f", (0, 10, False, True)), ("f", (1, 50, False, False)), ("f", (2, 1000, False, True)),
           ("f", (3, 7, False, False)),                      # the fourth: the four go as one pair
           ("f", (1, 20, False, True)), ("f", (2, 5, False, False)),
           ("f", (1, 30, True, False)),                      # commits: the two held go first, then it
           ("f", (1, 40, False, True)), ("f", (0, 9, False, False)), ("f", (3, 64, False, True)),
           ("a", 2),                                          # an append launches the three held
           ("f", (2, 11, True, True)), ("f", (0, 12, False, False)), ("f", (1, 13, False, False)),
           ("s", (3, 100))]                                   # a synchronous fetch: held ones first
    offs = g.integers(0, 200, P * C).astype(np.uint64)
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        for e in (dev, ora):
            e.commit_consumer_offset(np.repeat(pp, C), np.tile(np.arange(C, dtype=np.uint32), P), offs)
        want, got, held = [], [], []
        for kind, x in ops:
            if kind == "a":  # (applied before it returns, as the oracle's)
                b = make_batch(spec, x)
                dev.append(b.pidx, b.lens, b.payload)
                ora.append(b.pidx, b.lens, b.payload)
                continue
            c, mx = x[0], x[1]
            commit = kind == "f" and x[2]
            rc, res, buf, used = ora.fetch(pp, np.full(P, c, np.uint32), np.full(P, mx, np.uint32),
                                           out_cap=4 << 20, commit=commit)
            want.append((res.copy(), bytes(buf[:used])))
            if kind == "s":
                rc, res, buf, used = dev.fetch(pp, np.full(P, c, np.uint32), np.full(P, mx, np.uint32), out_cap=4 << 20)
                got.append((res.copy(), bytes(buf[:used])))
                continue
            req = np.zeros((P, 4), np.uint32)
            req[:, 3] = A.RMQ_FETCH_COMMIT if commit else 0
            if x[3]:
                d_out = dev.device_alloc(4 << 20)
                tk = dev.fetch_async(pp, np.full(P, c, np.uint32), np.full(P, mx, np.uint32), d_out=d_out,
                                     out_cap=4 << 20, req=req)
            else:
                d_out = None
                tk = dev.fetch_async(pp, np.full(P, c, np.uint32), np.full(P, mx, np.uint32),
                                     out=np.zeros(4 << 20, np.uint8), out_cap=4 << 20, req=req)
            held.append((len(got), tk, d_out))
            got.append(None)
        for k, tk, d_out in held:
            rc, res, used = dev.fetch_poll(tk, wait=True)
            if d_out is None:
                data = bytes(tk.out[:used])
            else:
                h = np.empty(used, np.uint8)
                dev.d2h(h, d_out)
                data = bytes(h)
                dev.device_free(d_out)
            got[k] = (res.copy(), data)
        for k, ((gr, gb), (wr, wb)) in enumerate(zip(got, want)):
            for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                assert np.array_equal(gr[f], wr[f]), (k, f)
            assert gb == wb, k
        assert np.array_equal(dev.consumer_table(), ora.consumer_table())


def test_async_fetch_empty_and_unknown():
    cfg = EngineConfig(num_partitions=8, replication_factor=1, segment_bytes=1 << 16, index_interval=256,
                       max_consumers=1, max_batch_records=1024)
    with Engine(cfg) as dev:
        tk = dev.fetch_async(np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32))
        assert dev.fetch_poll(tk, wait=False)[0] == A.RMQ_OK
        tk.ticket = 1 << 40
        with pytest.raises(EngineError):
            dev.fetch_poll(tk)


@pytest.mark.parametrize("replay", [1, 3])
def test_fetch_agrees_with_oracle(oracle_mod, replay):
    """20k requests (two per resolve wave, odd counts too), unknown partitions, bad consumers,
    zero-record slices, an output that ends mid-way and records of 1..4000 bytes; with the
    profiling replay (rmq_profile_enable(3): every fetch's kernels run three times) the results
    are the same."""
    P, C = 512, 4
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 21, index_interval=512,
                       max_consumers=C, max_batch_records=65536)
    spec = StreamSpec(P, 30000, "zipf", size=(1, 4000), config_index=8)
    g = np.random.default_rng(9)
    n = 20000
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        dev.profile(replay if replay > 1 else 0)
        ops = [("append", make_batch(spec, b)) for b in range(2)]
        p = g.integers(0, P + 8, n)
        c = g.integers(0, C + 1, n)
        pc = np.repeat(np.arange(P), C)
        cc = np.tile(np.arange(C), P)
        ops.append(("consumer_commit", pc, cc, g.integers(0, 150, P * C)))
        mx = g.integers(0, 60, n)
        ops.append(("fetch", p, c, mx))
        ops.append(("fetch", p, c, mx, 3 << 20))
        ops.append(("fetch", p[:7], c[:7], mx[:7]))
        ops.append(("fetch", p[:1], c[:1], mx[:1]))
        ops.append(("fetch", p, c, np.full(n, 1024)))
        run_ops(dev, ora, cfg, ops, check=False)


def _commit_loop(eng, P, C, rounds, batches, mx, cap):
    """Appends interleaved with read-and-commit fetches of every (partition, consumer)."""
    pp = np.repeat(np.arange(P, dtype=np.uint32), C)
    cc = np.tile(np.arange(C, dtype=np.uint32), P)
    out = []
    for k in range(rounds):
        for b in batches[k]:
            eng.append(b.pidx, b.lens, b.payload)
        rc, res, buf, used = eng.fetch(pp, cc, np.full(P * C, mx, np.uint32), out_cap=cap, commit=True)
        out.append((rc, res.copy(), bytes(buf[:used])))
    return out


def test_fetch_commit_matches_oracle(oracle_mod):
    """RMQ_FETCH_COMMIT: the consumers advance by what they were served (ConsumerClientImpl's
    read-then-commit in one call); an output cut mid-way commits nothing for the requests that did
    not fit; rings small enough that slow consumers fall below retention (RMQ_EOFFSET: they resume
    at the first retained offset)."""
    P, C = 64, 2
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 14, index_interval=256,
                       max_consumers=C, max_batch_records=4096)
    spec = StreamSpec(P, 1500, "zipf", size=(1, 300), config_index=46)
    batches = [[make_batch(spec, 2 * k), make_batch(spec, 2 * k + 1)] for k in range(6)]
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        for cap in (1 << 20, 20000):
            got = _commit_loop(dev, P, C, 6, batches if cap > 20000 else batches[::-1], 7, cap)
            want = _commit_loop(ora, P, C, 6, batches if cap > 20000 else batches[::-1], 7, cap)
            for k, (g, w) in enumerate(zip(got, want)):
                assert g[0] == w[0], (cap, k)
                for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                    assert np.array_equal(g[1][f], w[1][f]), (cap, k, f)
                assert g[2] == w[2], (cap, k)
            assert np.array_equal(dev.consumer_table(), ora.consumer_table())
        st = np.concatenate([g[1]["status"] for g in got])
        assert (st == A.RMQ_EOFFSET).any() and (st == A.RMQ_ENOSPC).any()
        # two committing requests for one consumer in a call: refused as a whole
        with pytest.raises(EngineError) as ei:
            dev.fetch(np.zeros(2, np.uint32), np.zeros(2, np.uint32), np.full(2, 5, np.uint32), out_cap=1 << 16,
                      commit=True)
        assert ei.value.status == A.RMQ_EINVAL
        # an unknown flag bit in any row (first, middle, the last of a count that is not a multiple of
        # four): the call is refused whole, nothing committed
        table = dev.consumer_table().copy()
        d_out = dev.device_alloc(1 << 16)
        for n, at, bit in ((7, 6, 4), (9, 0, 1 << 31), (16, 9, 8), (1, 0, 16)):  # (2: RMQ_FETCH_REPLICA, ABI 10)
            req = np.zeros((n, 4), np.uint32)
            req[:, 0], req[:, 2], req[:, 3] = np.arange(n) % P, 5, A.RMQ_FETCH_COMMIT
            req[at, 3] |= bit
            with pytest.raises(EngineError) as ei:
                dev.fetch_device(None, None, None, d_out, 1 << 16, req=req)
            assert ei.value.status == A.RMQ_EINVAL, (n, at, bit)
        assert np.array_equal(dev.consumer_table(), table)
        dev.device_free(d_out)


def _cache_script(eng, P, C, spec, moves):
    """Read-and-commit rounds (position-cache hits), rounds whose consumers the application moved
    (misses), a plain read (the next fetch re-reads: a miss), slices longer than the walk (search)."""
    pp = np.repeat(np.arange(P, dtype=np.uint32), C)
    cc = np.tile(np.arange(C, dtype=np.uint32), P)
    out = []
    for k in range(10):
        b = make_batch(spec, k)
        eng.append(b.pidx, b.lens, b.payload)
        if k in moves:
            eng.commit_consumer_offset(pp[::2], cc[::2], moves[k])
        mx = np.full(P * C, (3, 10, 40)[k % 3], np.uint32)
        rc, res, buf, used = eng.fetch(pp, cc, mx, out_cap=1 << 22, commit=k != 5)
        out.append((rc, res.copy(), bytes(buf[:used])))
    return out


def test_position_cache_hits_and_misses(oracle_mod):
    """The fetch position cache (fetch.hip: the ring position of the record after each consumer's
    last served slice): consumers reading on from their last slice walk from the cached position,
    the others search the index; rings small enough that retention passes cached positions. Every
    result equals the oracle's, which has no cache."""
    P, C = 32, 3
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 15, index_interval=256,
                       max_consumers=C, max_batch_records=4096)
    spec = StreamSpec(P, 2000, "zipf", size=(1, 200), config_index=48)
    g = np.random.default_rng(48)
    moves = {3: g.integers(0, 400, P * C // 2 + (P * C) % 2).astype(np.uint64),
             7: g.integers(0, 900, P * C // 2 + (P * C) % 2).astype(np.uint64)}
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        got = _cache_script(dev, P, C, spec, moves)
        want = _cache_script(ora, P, C, spec, moves)
        for k, (gw, ww) in enumerate(zip(got, want)):
            assert gw[0] == ww[0], k
            for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                assert np.array_equal(gw[1][f], ww[1][f]), (k, f)
            assert gw[2] == ww[2], k
        assert np.array_equal(dev.consumer_table(), ora.consumer_table())
        st = np.concatenate([x[1]["status"] for x in got])
        assert (st == A.RMQ_EOFFSET).any() and (st == A.RMQ_OK).any()


def _dup_rows_script(eng, P, C, spec, seed):
    """Fetch calls where every (partition, consumer) appears eight times with different max values
    (allowed: none commits); then each consumer moves to the end of one of its slices and reads on."""
    g = np.random.default_rng(seed)
    for b in range(3):
        bt = make_batch(spec, b)
        eng.append(bt.pidx, bt.lens, bt.payload)
    pc = np.repeat(np.arange(P, dtype=np.uint32), C), np.tile(np.arange(C, dtype=np.uint32), P)
    eng.commit_consumer_offset(pc[0], pc[1], g.integers(0, 50, P * C).astype(np.uint64))
    out = []
    for k in range(12):
        pidx, cons = np.tile(pc[0], 8), np.tile(pc[1], 8)
        mx = g.integers(1, 40, pidx.size).astype(np.uint32)
        rc, res, buf, used = eng.fetch(pidx, cons, mx, out_cap=1 << 23)
        out.append((rc, res.copy(), bytes(buf[:used])))
        pick = g.integers(0, 8, P * C) * (P * C) + np.arange(P * C)
        nxt = res["start_offset"][pick] + res["count"][pick]
        eng.commit_consumer_offset(pc[0], pc[1], nxt.astype(np.uint64))
    return out


def test_position_cache_duplicate_rows(oracle_mod):
    """requests of one (partition, consumer) in one call each leave a position-cache
    entry; the entry is one 16-byte store, so the next call, reading on from one of the slices,
    walks from a true {offset, position} pair. Every result equals the oracle's (no cache)."""
    P, C = 16, 2
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 20, index_interval=256,
                       max_consumers=C, max_batch_records=4096)
    spec = StreamSpec(P, 3000, "uniform", size=(1, 300), config_index=57)
    with Engine(cfg) as dev, oracle_mod.OracleEngine(cfg) as ora:
        got, want = _dup_rows_script(dev, P, C, spec, 57), _dup_rows_script(ora, P, C, spec, 57)
        for k, (gw, ww) in enumerate(zip(got, want)):
            assert gw[0] == ww[0], k
            for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                assert np.array_equal(gw[1][f], ww[1][f]), (k, f)
            assert gw[2] == ww[2], k
        assert all((x[1]["count"] > 0).any() for x in got)


def test_device_rows_match_host_rows():
    """RMQ_FETCH_DEVICE_ROWS (ABI 9): request and result rows in device memory give the results of
    the same requests from host rows; their flags word is ignored (a read-and-commit flag commits
    nothing: the host never checked those requests); host outputs are refused with device rows."""
    P, C = 128, 2
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 18, index_interval=256,
                       max_consumers=C, max_batch_records=8192)
    spec = StreamSpec(P, 6000, "zipf", size=(1, 400), config_index=49)
    g = np.random.default_rng(49)
    with Engine(cfg) as dev:
        for b in range(4):
            bt = make_batch(spec, b)
            dev.append(bt.pidx, bt.lens, bt.payload)
        n = 3001
        req = np.zeros((n, 4), np.uint32)
        req[:, 0] = g.integers(0, P + 2, n)
        req[:, 1] = g.integers(0, C + 1, n)
        req[:, 2] = g.integers(0, 30, n)
        dev.commit_consumer_offset(np.repeat(np.arange(P, dtype=np.uint32), C), np.tile(np.arange(C, dtype=np.uint32), P),
                                   g.integers(0, 60, P * C).astype(np.uint64))
        cap = 64 << 20  # (every request fits: at most 3001 x 30 records of 416 bytes)
        d_out, d_out2 = dev.device_alloc(cap), dev.device_alloc(cap)
        rc_w, want, used_w = dev.fetch_device(None, None, None, d_out, cap, req=req.copy())
        table = dev.consumer_table().copy()
        req[:, 3] = A.RMQ_FETCH_COMMIT  # ignored with device rows
        d_req, d_res = dev.device_alloc(16 * n), dev.device_alloc(32 * n)
        dev.h2d(d_req, req)
        rc, none, used = dev.fetch_device(None, None, None, d_out2, cap, d_rows=(n, d_req, d_res))
        assert none is None and rc == rc_w == A.RMQ_OK and used == used_w
        got = np.empty(n, want.dtype)
        dev.d2h(got, d_res)
        for f in ("status", "start_offset", "count", "bytes", "out_pos"):
            assert np.array_equal(got[f], want[f]), f
        a, b = np.empty(used, np.uint8), np.empty(used, np.uint8)
        dev.d2h(a, d_out)
        dev.d2h(b, d_out2)
        assert np.array_equal(a, b)
        assert np.array_equal(dev.consumer_table(), table)
        assert (want["count"] > 0).any()
        out = np.zeros(64, np.uint8)
        rc = dev.lib.rmq_fetch(dev.h, A.C.c_void_p(d_req), n, A.RMQ_MEM_HOST | A.RMQ_FETCH_DEVICE_ROWS,
                               out.ctypes.data_as(A.C.c_void_p), 64, A.C.c_void_p(d_res), None)
        assert rc == A.RMQ_EINVAL
        for d in (d_out, d_out2, d_req, d_res):
            dev.device_free(d)


def test_pinned_rows_from_registered_and_plain_memory():
    """RMQ_FETCH_PINNED_ROWS with rows the caller page-locked itself (rmq_host_register: mapped, so
    the kernels read and write them in place) and with ordinary pageable rows (not mapped: staged
    like unflagged rows): both give the results of an ordinary fetch of the same requests."""
    P, C = 200, 2
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 18, index_interval=256,
                       max_consumers=C, max_batch_records=8192)
    spec = StreamSpec(P, 5000, "zipf", size=(1, 300), config_index=53)
    g = np.random.default_rng(53)
    with Engine(cfg) as dev:
        for b in range(3):
            bt = make_batch(spec, b)
            dev.append(bt.pidx, bt.lens, bt.payload)
        cap = 8 << 20
        for register in (True, False):
            n = 2 * P + 13
            # (rows page-aligned: hipHostRegister locks whole pages)
            raw_q, raw_s = np.zeros(16 * n + 8192, np.uint8), np.zeros(32 * n + 8192, np.uint8)
            oq, os_ = (-raw_q.ctypes.data) % 4096, (-raw_s.ctypes.data) % 4096
            req = raw_q[oq:oq + 16 * n].view(np.uint32).reshape(n, 4)
            res = raw_s[os_:os_ + 32 * n].view(FETCH_RES_DTYPE)
            req[:, 0] = g.integers(0, P + 2, n)
            req[:, 1] = g.integers(0, C, n)
            req[:, 2] = g.integers(0, 500, n)
            if register:
                dev.host_register(req)
                dev.host_register(res)
            try:
                out = np.zeros(cap, np.uint8)
                tk = dev.fetch_async(None, None, None, out=out, out_cap=cap, req=req, res=res, pinned_rows=True)
                rc, got, used = dev.fetch_poll(tk, wait=True)
                rc_w, want, wbuf, used_w = dev.fetch(req[:, 0].copy(), req[:, 1].copy(), req[:, 2].copy(), out_cap=cap)
                assert rc == rc_w == A.RMQ_OK and used == used_w, register
                assert got is res
                for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                    assert np.array_equal(res[f], want[f]), (register, f)
                assert (res["count"] > 0).any()
                for r in np.flatnonzero((res["status"] == 0) & (res["bytes"] > 0)):
                    a, b = int(res["out_pos"][r]), int(res["out_pos"][r] + res["bytes"][r])
                    assert np.array_equal(out[a:b], wbuf[a:b]), (register, r)
            finally:
                if register:
                    dev.host_unregister(req)
                    dev.host_unregister(res)


def test_pinned_rows_match_sync():
    """RMQ_FETCH_PINNED_ROWS (ABI 7): requests and result rows in page-locked arrays go by DMA alone;
    six fetches in flight (more than the four slots), host and device outputs, one output cut
    mid-way (ENOSPC): every result equals a synchronous fetch of the same requests issued right
    after it, and sizes change from call to call through the same slots (the chunk sums a gather
    zeroes for its slot's next fetch)."""
    P, C = 256, 2
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 18, index_interval=256,
                       max_consumers=C, max_batch_records=8192)
    spec = StreamSpec(P, 6000, "zipf", size=(1, 400), config_index=47)
    g = np.random.default_rng(11)
    with Engine(cfg) as dev:
        for b in range(6):
            bt = make_batch(spec, b)
            dev.append_async(bt.pidx, bt.lens, bt.payload)
        pending, cap_of = [], []
        for k in range(6):
            n = [P * C, 5, P * C, 77, 1, P * C][k]
            req, res = dev.fetch_rows(n)
            req[:, 0] = g.integers(0, P + 3, n)
            req[:, 1] = g.integers(0, C, n)
            req[:, 2] = g.integers(0, 2000, n)
            cap = 1 << 16 if k == 2 else 8 << 20
            cap_of.append(cap)
            if k % 2:
                out = np.zeros(cap, np.uint8)
                tk = dev.fetch_async(None, None, None, out=out, out_cap=cap, req=req, res=res, pinned_rows=True)
                d_out = None
            else:
                d_out = dev.device_alloc(cap)
                tk = dev.fetch_async(None, None, None, d_out=d_out, out_cap=cap, req=req, res=res, pinned_rows=True)
            rc_w, want, wbuf, used_w = dev.fetch(req[:, 0].copy(), req[:, 1].copy(), req[:, 2].copy(), out_cap=cap)
            pending.append((tk, rc_w, want.copy(), wbuf.copy(), used_w, d_out))
        for k, (tk, rc_w, want, wbuf, used_w, d_out) in enumerate(pending):
            rc, res, used = dev.fetch_poll(tk, wait=True)
            assert rc == rc_w, k
            for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                assert np.array_equal(res[f], want[f]), (k, f)
            assert used == used_w, k
            served = (res["status"] == 0) & (res["bytes"] > 0)
            if d_out is None:
                got = tk.out
            else:
                n_cp = min(used, cap_of[k])  # (bytes needed can exceed the output after a cut)
                got = np.empty(max(n_cp, 1), np.uint8)
                if n_cp:
                    dev.d2h(got[:n_cp], d_out)
                dev.device_free(d_out)
            for r in np.flatnonzero(served):
                a, b = int(res["out_pos"][r]), int(res["out_pos"][r] + res["bytes"][r])
                assert np.array_equal(got[a:b], wbuf[a:b]), (k, r)
        assert pending[2][1] == A.RMQ_ENOSPC
        # the synchronous call with page-locked rows (read and written in place by its kernels)
        for k, cap in ((0, 8 << 20), (1, 1 << 16)):
            n = P * C
            req, res = dev.fetch_rows(n)
            req[:, 0] = g.integers(0, P + 3, n)
            req[:, 1] = g.integers(0, C, n)
            req[:, 2] = g.integers(0, 2000, n)
            d_out = dev.device_alloc(cap)
            rc, got, used = dev.fetch_device(None, None, None, d_out, cap, req=req, res=res, pinned_rows=True)
            rc_w, want, wbuf, used_w = dev.fetch(req[:, 0].copy(), req[:, 1].copy(), req[:, 2].copy(), out_cap=cap)
            assert rc == rc_w and used == used_w, k
            assert got is res
            for f in ("status", "start_offset", "count", "bytes", "out_pos"):
                assert np.array_equal(res[f], want[f]), (k, f)
            n_cp = min(used, cap)
            buf = np.empty(max(n_cp, 1), np.uint8)
            if n_cp:
                dev.d2h(buf[:n_cp], d_out)
            for r in np.flatnonzero((res["status"] == 0) & (res["bytes"] > 0)):
                a, b = int(res["out_pos"][r]), int(res["out_pos"][r] + res["bytes"][r])
                assert np.array_equal(buf[a:b], wbuf[a:b]), (k, r)
            dev.device_free(d_out)
        dev.sync()


@pytest.mark.parametrize("dma_in", ["1", "0"])
def test_rows_by_dma_match_rows_in_place(monkeypatch, dma_in):
    """RMQ_FETCH_DMA=2 (a measured knob, off by default): request rows copied to the device and result
    rows copied back around the kernels (RMQ_FETCH_DMA_IN=0: result rows only) give the results of
    the default path, where the kernels read and write the rows in place; host and device outputs,
    synchronous and asynchronous calls, page-locked and staged rows."""
    P, C = 96, 2
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=1 << 18, index_interval=256,
                       max_consumers=C, max_batch_records=8192)
    spec = StreamSpec(P, 4000, "zipf", size=(1, 300), config_index=57)
    g = np.random.default_rng(57)
    n = 2 * P + 7
    p, c, mx = g.integers(0, P + 2, n), g.integers(0, C, n), g.integers(0, 400, n)
    cap = 4 << 20

    def run():
        out = []
        with Engine(cfg) as dev:
            for b in range(3):
                bt = make_batch(spec, b)
                dev.append(bt.pidx, bt.lens, bt.payload)
            rc, res, buf, used = dev.fetch(p, c, mx, out_cap=cap)  # staged rows, host output
            out.append((rc, res.copy(), bytes(buf[:used])))
            req, rs = dev.fetch_rows(n)
            req[:, 0], req[:, 1], req[:, 2] = p, c, mx
            d_out = dev.device_alloc(cap)
            tk = dev.fetch_async(None, None, None, d_out=d_out, out_cap=cap, req=req, res=rs, pinned_rows=True)
            rc, res, used = dev.fetch_poll(tk, wait=True)
            got = np.empty(max(used, 1), np.uint8)
            if used:
                dev.d2h(got[:used], d_out)
            out.append((rc, res.copy(), bytes(got[:used])))
            dev.device_free(d_out)
        return out

    want = run()
    monkeypatch.setenv("RMQ_FETCH_DMA", "2")
    monkeypatch.setenv("RMQ_FETCH_DMA_IN", dma_in)
    got = run()
    for k, (a, b) in enumerate(zip(got, want)):
        assert a[0] == b[0] == A.RMQ_OK, k
        for f in ("status", "start_offset", "count", "bytes", "out_pos"):
            assert np.array_equal(a[1][f], b[1][f]), (k, f)
        assert a[2] == b[2], k
    assert (want[0][1]["count"] > 0).any()
