"""Debug: the set_segments parity scenario op by op, dumping the first ring difference."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from parity import compare_state
from oracle.oracle import OracleEngine
from ripplemq_amd.engine import Engine, EngineConfig
from ripplemq_amd.workload import StreamSpec, make_batch

P, S = 32, 1 << 16
cfg = EngineConfig(num_partitions=P, replication_factor=3, segment_bytes=S, index_interval=1024,
                   max_batch_records=4096, pool_bytes=3 * P * S)
spec = StreamSpec(P, 3000, "zipf", size=(1, 300), config_index=56)
first = [make_batch(spec, b) for b in range(5)]
load = np.bincount(np.concatenate([b.pidx for b in first]), minlength=P)
order = np.argsort(-load, kind="stable")
hot, cold = order[:4], order[-6:]
print("hot", hot, "shrunk", np.concatenate([cold, order[4:6]]))
ops = [("append", b) for b in first] + [("seg", hot, np.full(4, 4 * S, np.uint64)),
       ("seg", np.concatenate([cold, order[4:6]]), np.full(8, 4096, np.uint64))]
ops += [("append", make_batch(spec, b)) for b in range(5, 12)]
pp = np.arange(P, dtype=np.uint32)
if "nocc" not in sys.argv:
    ops += [("cc", pp, np.zeros(P, np.uint32), pp * 7)]
if "nofetch" not in sys.argv:
    ops += [("fetch", pp, np.zeros(P, np.uint32), np.full(P, 64, np.uint32))]
seg2 = hot[:1] if "only17" in sys.argv else hot[:2]
ops += [("seg", seg2, np.full(seg2.size, 2 * S if "seg128" in sys.argv else S, np.uint64))]
ops += [("append", make_batch(spec, b)) for b in range(12, 14)]
with Engine(cfg) as dev, OracleEngine(cfg) as ora:
    for k, op in enumerate(ops):
        if op[0] == "append":
            b = op[1]
            if "drop17" in sys.argv and k > 14:
                keep = b.pidx != 17
                offs = np.concatenate([[0], np.cumsum(b.lens, dtype=np.int64)])
                pay = np.concatenate([b.payload[offs[i]:offs[i + 1]] for i in np.flatnonzero(keep)])
                b = type(b)(b.pidx[keep], b.lens[keep], pay)
            print("before", k, {q: (ora.state(q)["log_start_pos"], ora.state(q)["log_end_pos"], ora.state(q)["log_end_offset"]) for q in (17, 8)})
            od, sd = dev.append(b.pidx, b.lens, b.payload)
            oo, so = ora.append(b.pidx, b.lens, b.payload)
            assert sd == so and np.array_equal(od, oo), (k, sd, so)
        elif op[0] == "cc":
            dev.commit_consumer_offset(*op[1:4]); ora.commit_consumer_offset(*op[1:4])
        elif op[0] == "fetch":
            a1 = dev.fetch(*op[1:4]); a2 = ora.fetch(*op[1:4])
            assert a1[0] == a2[0] and np.array_equal(a1[1], a2[1]), "fetch"
        else:
            dev.set_segments(op[1], op[2]); ora.set_segments(op[1], op[2])
            print("seg", k, [(int(p), dev.state(int(p))["segment_bytes"]) for p in op[1]])
        nbad = 0
        for p in range(P):
            sd_, so_ = dev.state(p), ora.state(p)
            assert sd_ == so_, (k, p, sd_, so_)
            for r in range(3):
                a, bb = dev.read_segment(r, p), ora.read_segment(r, p)
                if not np.array_equal(a, bb):
                    bad = np.flatnonzero(a != bb)
                    print(f"op {k} {op[0]}: p={p} r={r} {bad.size} bytes differ [{bad[0]}..{bad[-1]}] state {so_}")
                    lo = bad[0] // 16 * 16
                    S_ = so_["segment_bytes"]; s0 = so_["log_start_pos"] % S_
                    pieces = sorted(set((bad // 16).tolist()))
                    print("  pieces", [(q * 16, so_["log_start_pos"] + ((q * 16 - s0) % S_)) for q in pieces][:12])
                    print("  gpu zero pieces", sum(1 for q in pieces if not a[16*q:16*q+16].any()), "of", len(pieces))
                    rp = [ora.record_pos(p, o) for o in range(so_["log_start_offset"], so_["log_end_offset"] + 1)]
                    for q in pieces:
                        lp = so_["log_start_pos"] + ((q * 16 - s0) % S_)
                        k2 = max(i for i, x in enumerate(rp) if x <= lp)
                        hdr = ora.read_segment(r, p, rp[k2] % S_, 16)
                        L = int(np.frombuffer(hdr[8:12].tobytes(), np.uint32)[0])
                        g16 = a[16 * q:16 * q + 16]
                        where = []
                        if g16.any():
                            for p2 in range(P):
                                for r2 in range(3):
                                    ring2 = ora.read_segment(r2, p2)
                                    v = np.lib.stride_tricks.sliding_window_view(ring2, 16)[::16]
                                    hit = np.flatnonzero((v == g16).all(axis=1))
                                    if hit.size:
                                        where.append((p2, r2, (hit * 16).tolist()[:3]))
                        exp = ora.read_segment(r, p, q * 16, 16)
                        print("     expected", exp.tolist())
                        print(f"   piece at pos {lp}: record {so_['log_start_offset'] + k2} at {rp[k2]} L={L} piece {(lp - rp[k2]) // 16} gpu={g16.tolist()} found_in={where}")
                    nbad += 1
        if nbad:
            sys.exit(1)
    print("all equal")
