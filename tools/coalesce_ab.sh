FQ="--steps 100 --warmup 10 --no-cpu-baseline --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py $FQ > gpurun_out/r06c_on_$k.json 2>/dev/null || exit 1
  RMQ_FETCH_COALESCE=1 timeout -k 10 200 python bench.py $FQ > gpurun_out/r06c_off_$k.json 2>/dev/null || exit 1
done
