"""Oracle semantics of per-partition ring sizes (rmq_set_segments, FORMAT.md §2 / §4): growing keeps
every retained record, shrinking applies retention at the new size first, fetched bytes of the
records that stay are unchanged. Checked against tests/refmodel.py's view of the same stream."""
import numpy as np

from ripplemq_amd.engine import EngineConfig
from ripplemq_amd.workload import StreamSpec, make_batch


def _fetch_all(ora, p, n):
    ora.commit_consumer_offset(np.array([p], np.uint32), np.zeros(1, np.uint32), np.zeros(1, np.uint64))
    return ora.fetch(np.array([p], np.uint32), np.zeros(1, np.uint32), np.array([n], np.uint32))


def test_grow_then_shrink_keeps_offsets_and_bytes(oracle_mod):
    P, S, I = 4, 1 << 14, 1024
    cfg = EngineConfig(num_partitions=P, replication_factor=2, segment_bytes=S, index_interval=I,
                       max_batch_records=2000)
    spec = StreamSpec(P, 400, "zipf", size=(1, 200), config_index=58)
    with oracle_mod.OracleEngine(cfg) as ora:
        for b in range(3):
            x = make_batch(spec, b)
            ora.append(x.pidx, x.lens, x.payload)
        hot = int(np.argmax([ora.state(p)["log_end_offset"] for p in range(P)]))
        st0 = ora.state(hot)
        rc, res, before, _ = _fetch_all(ora, hot, 1 << 20)
        ora.set_segments([hot], [4 * S])  # grow: nothing evicted, same bytes from the same offsets
        st1 = ora.state(hot)
        assert st1["segment_bytes"] == 4 * S
        assert {k: v for k, v in st1.items() if k != "segment_bytes"} == {k: v for k, v in st0.items() if k != "segment_bytes"}
        rc1, res1, after, _ = _fetch_all(ora, hot, 1 << 20)
        assert np.array_equal(before, after) and np.array_equal(res, res1)
        for b in range(3, 9):  # the bigger ring now retains more than S bytes
            x = make_batch(spec, b)
            ora.append(x.pidx, x.lens, x.payload)
        st2 = ora.state(hot)
        assert st2["log_end_pos"] - st2["log_start_pos"] > S
        ora.set_segments([hot], [4 * I])  # shrink: retention at 4 KiB first (FORMAT.md §4 rule)
        st3 = ora.state(hot)
        m = -(-(st2["log_end_pos"] - 4 * I) // I)
        e = ora.read_index(hot, m, 1)[0]
        assert (st3["log_start_offset"], st3["log_start_pos"]) == (int(e[0]), int(e[1]))
        assert st3["log_end_pos"] - st3["log_start_pos"] <= 4 * I
        # the records that stay read back the same as before the shrink
        ora.commit_consumer_offset(np.array([hot], np.uint32), np.zeros(1, np.uint32),
                                   np.array([st3["log_start_offset"]], np.uint64))
        rc4, res4, kept, _ = ora.fetch(np.array([hot], np.uint32), np.zeros(1, np.uint32), np.array([1 << 20], np.uint32))
        assert rc4 == 0 and res4["count"][0] == st3["log_end_offset"] - st3["log_start_offset"]
        pos = ora.record_pos(hot, st3["log_start_offset"])
        assert pos == st3["log_start_pos"]
