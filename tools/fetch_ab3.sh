# Fetch legs of the current library, variants/<V> (same tree) and a whole older tree
# variants/<OLD>/tree (its own bench.py and library), two rounds (run through gpurun):
#   bash tools/fetch_ab3.sh <tag> <V> <OLD>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
T=$1; V=$2; O=$3
FQ="--steps 100 --warmup 10 --no-cpu-baseline --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 200 python bench.py $FQ > gpurun_out/${T}_cur_$k.json 2> gpurun_out/${T}_cur_$k.err || exit 1
  RMQ_LIB=$R/variants/$V/libripplemq_engine.so timeout -k 10 200 python bench.py $FQ > gpurun_out/${T}_${V}_$k.json 2> gpurun_out/${T}_${V}_$k.err || exit 1
  (cd variants/$O/tree && timeout -k 10 200 python bench.py $FQ) > gpurun_out/${T}_${O}_$k.json 2> gpurun_out/${T}_${O}_$k.err || exit 1
done
echo "[fetch_ab3] done"
