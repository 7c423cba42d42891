"""RMQ_FETCH_COMMIT on the oracle (CPU): a committing fetch is the consumer client's read-then-commit
(ConsumerClientImpl.java:61-117: read max 10, then commit offset + count) in one call, restated in
oracle/ripple_oracle.c ro_fetch; the GPU engine is compared with it in
tests/test_gpu_fetch_async.py::test_fetch_commit_matches_oracle."""
from __future__ import annotations

import numpy as np

from refmodel import Broker
from ripplemq_amd import _abi as A
from ripplemq_amd.engine import EngineConfig


def test_fetch_commit_is_read_then_commit(oracle_mod):
    P, C = 4, 2
    cfg = EngineConfig(num_partitions=P, replication_factor=1, segment_bytes=1 << 16, index_interval=256,
                       max_consumers=C, max_batch_records=1024)
    g = np.random.default_rng(2)
    ref = Broker("t", P)
    with oracle_mod.OracleEngine(cfg) as ora:
        for _ in range(3):
            pidx = g.integers(0, P, 200).astype(np.uint32)
            lens = g.integers(0, 40, 200).astype(np.uint32)
            payload = g.integers(0, 256, int(lens.sum()), dtype=np.uint8)
            ora.append(pidx, lens, payload)
            pos = 0
            for p, ln in zip(pidx, lens):
                ref.produce(int(p), payload[pos:pos + ln].tobytes())
                pos += ln
        pp = np.repeat(np.arange(P, dtype=np.uint32), C)
        cc = np.tile(np.arange(C, dtype=np.uint32), P)
        for _ in range(8):  # each consumer reads 10, commits, and reads on from there
            rc, res, buf, _ = ora.fetch(pp, cc, np.full(P * C, 10, np.uint32), commit=True)
            assert rc == A.RMQ_OK and np.all(res["status"] == 0)
            for k in range(P * C):
                msgs, off = ref.consume(int(pp[k]), f"c{cc[k]}", 10)  # read max 10, commit off + n
                assert int(res["count"][k]) == len(msgs) and int(res["start_offset"][k]) == off
        table = ora.consumer_table()
        for p in range(P):
            for c in range(C):
                assert int(table[p][c]) == ref.sms[p].get_consumer_offset(f"c{c}")
        # a cut output commits nothing for the requests that did not fit
        before = ora.consumer_table().copy()
        rc, res, _, _ = ora.fetch(pp, cc, np.full(P * C, 1000, np.uint32), out_cap=64, commit=True)
        cut = res["status"] == A.RMQ_ENOSPC
        assert rc == A.RMQ_ENOSPC and cut.any()
        after = ora.consumer_table()
        for k in np.flatnonzero(cut):
            assert after[pp[k]][cc[k]] == before[pp[k]][cc[k]]
        # two committing requests for one consumer in a call are refused
        rc, _, _, _ = ora.fetch(np.zeros(2, np.uint32), np.zeros(2, np.uint32), np.full(2, 1, np.uint32),
                                out_cap=1 << 12, commit=True)
        assert rc == A.RMQ_EINVAL
