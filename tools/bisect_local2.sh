set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in 3732dfa 52bc272 18747fd 778dc9c df20f68; do
  (cd variants/$c/tree && timeout -k 10 200 python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 > "$GRAFT_REPO_ROOT/gpurun_out/bis_$c.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bis_$c.err") || echo "FAILED $c"
done
echo done
