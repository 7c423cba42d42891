# Fetch rows by DMA vs in place (RMQ_FETCH_DMA 0 / 1 / 2): the fetch parity tests with DMA for every
# fetch, then the fetch and mixed legs under each setting. bash tools/exp_dma.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; tail -30 "gpurun_out/$out"; exit 1; }; }
RMQ_FETCH_DMA=2 RMQ_FETCH_DMA_IN=${IN:-1} run 600 "${T}_pytest_dma2.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "fetch or consumer or pinned or golden"
tail -2 gpurun_out/${T}_pytest_dma2.log
FQ="--steps 400 --warmup 10 --no-cpu-baseline --host-steps 0 --tier-rounds 0 --concurrent-rounds 120"
for k in 1 2; do
  for m in 0 1 2; do
    RMQ_BENCH_CALLS=1 RMQ_FETCH_DMA=$m RMQ_FETCH_DMA_IN=${IN:-1} run 300 "${T}_legs_dma${m}_$k.json" python bench.py $FQ
  done
done
python3 - gpurun_out/${T}_legs_*.json <<'PY'
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); F=d["fetch"]
    for k in ("max10","max1024"):
        x=F[k]; r=x["roofline"]; print(f.split("/")[-1], k, "us/fetch %.1f" % r["mean_us_per_fetch"], "frac %.3f" % r["frac"], "kern %.2fG call %.2fG async %.2fG (%.2fx)" % (x["records_per_s_kernels"]/1e9, x["records_per_s_call"]/1e9, x["records_per_s_async_calls"]/1e9, x["records_per_s_async_calls"]/x["records_per_s_call"]))
    x=F["loop10"]; r=x["roofline"]; print("   loop10 us/fetch %.1f kern %.2fG call %.2fG call_us %.1f" % (r["mean_us_per_fetch"], x["records_per_s_kernels"]/1e9, x["records_per_s_call"]/1e9, x["call_us_median"]))
    m=d["mixed"]; print("   mixed", round(m["append_msgs_per_s"]/1e9,3), "G app", round(m["fetch_records_per_s"]/1e6,1), "M fetched resets", m["consumer_resets"], "of", m["fetches"]*m["requests_per_fetch"])
PY
echo "[exp] $(date +%T) done"
