# Fetch experiment: fetch parity tests, then the fetch and mixed legs with the current library and
# variants/<V>, then a kernel trace of the current fetch leg. bash tools/exp_fetch.sh <tag> <V>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; V=$2
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; tail -30 "gpurun_out/$out"; exit 1; }; }
run 600 "${T}_pytest.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "fetch or consumer or golden or failover or pinned or tier or state_machine"
tail -2 gpurun_out/${T}_pytest.log
FQ="--steps 400 --warmup 10 --no-cpu-baseline --host-steps 0 --tier-rounds 0"
for k in 1 2; do
  for m in cur $([ "$V" = "-" ] || echo $V); do
    if [ $m = cur ]; then L=$R/ripplemq_amd/libripplemq_engine.so; else L=$R/variants/$V/libripplemq_engine.so; fi
    RMQ_LIB=$L run 300 "${T}_legs_${m}_$k.json" python bench.py $FQ --concurrent-rounds 120
  done
done
python3 - gpurun_out/${T}_legs_*.json <<'PY'
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); F=d["fetch"]
    for k in ("max10","max1024"):
        x=F[k]; r=x["roofline"]; print(f.split("/")[-1], k, "us/fetch %.1f" % r["mean_us_per_fetch"], "frac %.3f" % r["frac"], "kern %.2fG call %.2fG async %.2fG" % (x["records_per_s_kernels"]/1e9, x["records_per_s_call"]/1e9, x["records_per_s_async_calls"]/1e9))
    if "loop10" not in F: pass
    else: x=F["loop10"]; r=x["roofline"]; print("   loop10 us/fetch %.1f frac %.3f kern %.2fG call %.2fG recs/req %.2f" % (r["mean_us_per_fetch"], r["frac"], x["records_per_s_kernels"]/1e9, x["records_per_s_call"]/1e9, x["records_per_request"]))
    m=d["mixed"]; print("   mixed", round(m["append_msgs_per_s"]/1e9,3), "G app", round(m["fetch_records_per_s"]/1e6,1), "M fetched resets", m["consumer_resets"], "of", m["fetches"]*m["requests_per_fetch"])
PY
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_fetchkt" -o kt -- python3 "$R/bench.py" --steps 20 --warmup 5 --fetch-rounds 10 --concurrent-rounds 0 --tier-rounds 0 --no-cpu-baseline --host-steps 0) > "$R/gpurun_out/${T}_fetchkt.log" 2>&1 || exit 1
grep -h "fetch" gpurun_out/${T}_fetchkt/*kernel_stats.csv | cut -c1-200
echo "[exp] $(date +%T) done"
