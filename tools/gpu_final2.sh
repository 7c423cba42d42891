# Round measurement: smoke, default bench line (N=1, CPU baseline, fetch and host legs), two
# driver-shaped 20-step lines, config D, rocprofv3 kernel stats of the default line, PMC
# FETCH_SIZE / WRITE_SIZE passes (separate runs). usage: bash tools/gpu_final2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench20_$rep.json 2> gpurun_out/${T}_bench20_$rep.err || exit 1
done
timeout -k 10 300 python bench.py --config D --pool 16 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_benchD.json 2> gpurun_out/${T}_benchD.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_prof -o kt -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${T}_bench_prof.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/${T}_pmc_fetch -o pf -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > $R/gpurun_out/${T}_pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/${T}_pmc_write -o pw -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > $R/gpurun_out/${T}_pmc_write.log 2>&1
