# Side legs: the GPU test suite, the tier leg, config D, the 2-rank rehearsal. bash tools/exp_side.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; tail -30 "gpurun_out/$out"; exit 1; }; }
run 900 "${T}_pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
tail -2 gpurun_out/${T}_pytest_gpu.log
run 300 "${T}_tier.json" python bench.py --steps 200 --warmup 20 --no-cpu-baseline --host-steps 0 --fetch-rounds 0 --concurrent-rounds 0 --tier-rounds 20
python3 -c "import json,sys; d=json.loads(open('gpurun_out/${T}_tier.json').read().strip().splitlines()[-1]); print(json.dumps(d['tier']))"
run 300 "${T}_D.json" python bench.py --config D --steps 200 --warmup 20 --no-cpu-baseline --host-steps 0 --fetch-rounds 0 --concurrent-rounds 0 --tier-rounds 0
python3 tools/show_lines.py gpurun_out/${T}_D.json
run 300 "${T}_local2.json" python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0
python3 -c "import json; d=json.loads(open('gpurun_out/${T}_local2.json').read().strip().splitlines()[-1]); x=d['xgmi']; print('local2', d['value']/1e9, x['host_waits_for_round_sizes'], x['host_wait_ms'])"
echo "[exp] $(date +%T) done"
