# HBM traffic of the fetch kernels (FETCH_SIZE and WRITE_SIZE, separate rocprofv3 --pmc passes) over
# the bench's fetch leg. bash tools/pmc_fetch.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
Q="--steps 20 --warmup 5 --fetch-rounds 10 --concurrent-rounds 0 --tier-rounds 0 --no-cpu-baseline --host-steps 0"
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c -f csv -d "$R/gpurun_out/${T}_$c" -o p -- python3 "$R/bench.py" $Q) > "$R/gpurun_out/${T}_$c.log" 2>&1 || { echo "FAILED $c"; tail -20 "$R/gpurun_out/${T}_$c.log"; exit 1; }
done
python3 - "$R/gpurun_out/$T" <<'PY'
import csv, glob, statistics, sys
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(sys.argv[1] + f"_{c}/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "fetch_" in r["Kernel_Name"]]
    for k in ("fetch_resolve", "fetch_gather"):
        v = [float(r["Counter_Value"]) for r in rows if k in r["Kernel_Name"]]
        # the max = 10 section comes first: its first 40 dispatches (10 rounds x 4 replays)
        print(c, k, "dispatches", len(v), "max10 mean KiB", round(statistics.mean(v[:40]), 1))
PY
