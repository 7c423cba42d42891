# L2 (TCC) hits and misses of the pipeline kernel with and without the XCD task order (RMQ_S3_XCD),
# one rocprofv3 --pmc pass each (two TCC counters). bash tools/exp_tcc.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
Q="--steps 300 --warmup 50 --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
for x in 1 0; do
  echo "[exp] $(date +%T) RMQ_S3_XCD=$x"
  (cd /tmp && export TMPDIR=/tmp && RMQ_S3_XCD=$x timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d "$R/gpurun_out/${T}_tcc$x" -o t -- python3 "$R/bench.py" $Q) > "$R/gpurun_out/${T}_tcc$x.log" 2>&1 || { echo FAILED; tail -20 "$R/gpurun_out/${T}_tcc$x.log"; exit 1; }
done
python3 - "$R/gpurun_out/${T}" <<'PY'
import csv, glob, statistics, sys, collections
for x in ("1", "0"):
    f = glob.glob(sys.argv[1] + f"_tcc{x}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(dict)
    grids = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "pipeline_kernel" not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        per[r["Dispatch_Id"]]["grid"] = int(r["Grid_Size"])
    g = collections.Counter(v["grid"] for v in per.values()).most_common(1)[0][0]
    rows = [v for v in per.values() if v["grid"] == g and "TCC_HIT_sum" in v and "TCC_MISS_sum" in v]
    h = statistics.mean(v["TCC_HIT_sum"] for v in rows); m = statistics.mean(v["TCC_MISS_sum"] for v in rows)
    print(f"RMQ_S3_XCD={x}: {len(rows)} launches, TCC hits {h:,.0f} misses {m:,.0f} per launch, hit rate {h / (h + m):.3f}")
PY
