# The canonical GPU measurement procedure (run through gpurun from the repo root):
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Steps, each under its own time limit; the script stops at the first failing step and writes
# everything under gpurun_out/<tag>_*:
#   tests      pytest -m gpu (all GPU parity tests), log in <tag>_pytest_gpu.log
#   tests:K    the same restricted to `-k K`
#   smoke      __graft_entry__.smoke()
#   bench      default bench line (2000 steps, CPU baseline, fetch, concurrent and host legs)
#   bench20    two driver-shaped lines (--steps 20 --warmup 5)
#   steady     one 600-step line without the side legs
#   kt20       kernel trace of a 20-step line (fill / drain launches)
#   benchD     config D (RF 5, 64 B..16 KB) line
#   ab[:NAME]  A/B of the current library against variants/NAME/ (default head; 400- and 20-step lines, 2 pairs)
#   local2     2-rank rehearsal on one GPU over the in-process transport (+ kernel trace)
#   local4     4-rank rehearsal (config C shape);  local8  the same with 8 ranks
#   ab2[:NAME] A/B of the 2-rank rehearsal against variants/NAME/ (default head)
#   prof       rocprofv3 --kernel-trace --stats of the default line (kernel stats CSV)
#   pmc        rocprofv3 FETCH_SIZE and WRITE_SIZE passes (separate runs) of a 300-step line
#   stamps     per-wave phase stamps of launch 100 (RMQ_STAMPS) + timing-only RMQ_DEBUG lines
#   legs       fetch / mixed / tier legs of a short line
#   calls      host-side cost per fetch call (tools/fetch_calls.py)
#   fetchkt    rocprofv3 kernel trace of the fetch leg (replayed kernels)
#   envab:VAR=v[,CFG]  GPU tests with an environment knob, then three off/on pairs of lines
#   group      launch-group size sweep;  Dprof  config D line, stamps and apply-launch trace
#   roles      phase stamps of the role-split stage 3 and of the default launch
#   sq / memc  SQ / memory-pipeline counters of the apply launches (tools/pmc_apply.sh)
#   knob:VAR=v1,v2  steady and 20-step lines per value;  dbg:B1,B2  timing-only RMQ_DEBUG lines
#   coalesce   fetch legs with asynchronous fetch coalescing on / off;  caps:S1:S2,...  ranking caps
#   fetchab3:V:OLD  fetch legs of the current library, variants/V and the older tree variants/OLD/tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
T=$1
shift
mkdir -p gpurun_out
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
run() {  # run <seconds> <out file> <command...>: stdout to the file, stderr to <file>.err
  local lim=$1 out=$2
  shift 2
  echo "[gpu.sh] $(date +%T) $out: $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[gpu.sh] FAILED rc=$? $out"; tail -20 "gpurun_out/$out.err"; exit 1; }
}
prof() {  # prof <seconds> <name> <rocprofv3 args...> -- <python args...>
  local lim=$1 name=$2
  shift 2
  echo "[gpu.sh] $(date +%T) rocprofv3 $name"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL "$lim" rocprofv3 "$@") > "$R/gpurun_out/${T}_$name.log" 2>&1 || { echo "[gpu.sh] FAILED rocprofv3 $name"; tail -20 "$R/gpurun_out/${T}_$name.log"; exit 1; }
}
for step in "$@"; do
  case $step in
    tests) run 1000 "${T}_pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ;;
    tests:*) run 600 "${T}_pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "${step#tests:}" ;;
    smoke) run 300 "${T}_smoke.txt" python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 500 "${T}_bench.json" python bench.py ;;
    bench20) for k in 1 2; do run 200 "${T}_bench20_$k.json" python bench.py --gpus 1 --steps 20 --warmup 5; done ;;
    steady) run 300 "${T}_steady.json" python bench.py --steps 600 --warmup 60 $Q ;;
    kt20)  # kernel trace of a driver-shaped line (20 steps): the fill and drain launches
      prof 200 kt20 --kernel-trace -f csv -d "$R/gpurun_out/${T}_kt20" -o kt -- python3 "$R/bench.py" --steps 20 --warmup 5 $Q ;;
    benchD) run 300 "${T}_benchD.json" python bench.py --config D --pool 16 --steps 200 --warmup 20 --no-cpu-baseline --host-steps 0 ;;
    ab|ab:*)  # ab:NAME compares against variants/NAME/ (default head)
      V=head; [ "$step" != ab ] && V=${step#ab:}
      for k in 1 2; do
        for v in cur $V; do
          if [ $v = cur ]; then L=$R/ripplemq_amd/libripplemq_engine.so; else L=$R/variants/$V/libripplemq_engine.so; fi
          RMQ_LIB=$L run 200 "${T}_${v}_400_$k.json" python bench.py --steps 400 --warmup 40 $Q
          RMQ_LIB=$L run 200 "${T}_${v}_20_$k.json" python bench.py --steps 20 --warmup 5 $Q
        done
      done ;;
    local2)
      run 300 "${T}_local2.json" python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 $Q
      prof 300 local2_prof --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_local2_kt" -o kt -- python3 "$R/bench.py" --gpus 2 --transport local --steps 100 --warmup 10 --segment-mb 2 --pool 8 $Q ;;
    ab2|ab2:*)  # A/B of the 2-rank rehearsal: current library vs variants/NAME/ (default head; NAME+NAME2: several), two rounds
      V=head; [ "$step" != ab2 ] && V=${step#ab2:}
      for k in 1 2; do
        for v in cur ${V//+/ }; do
          if [ $v = cur ]; then L=$R/ripplemq_amd/libripplemq_engine.so; else L=$R/variants/$v/libripplemq_engine.so; fi
          RMQ_LIB=$L run 300 "${T}_local2_${v}_$k.json" python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 $Q
        done
      done ;;
    local2kt:*)  # rehearsal kernel trace with variants/NAME/
      V=${step#local2kt:}
      RMQ_LIB=$R/variants/$V/libripplemq_engine.so prof 300 local2_prof_$V --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_local2_kt_$V" -o kt -- python3 "$R/bench.py" --gpus 2 --transport local --steps 100 --warmup 10 --segment-mb 2 --pool 8 $Q ;;
    local4) run 300 "${T}_local4.json" python bench.py --gpus 4 --transport local --steps 100 --warmup 10 --segment-mb 1 --pool 4 --config C $Q ;;
    local8)  # the N = 8 bench path (8 ranks, configs[3]'s shape) as threads on one GPU
      run 400 "${T}_local8.json" python bench.py --gpus 8 --transport local --steps 60 --warmup 6 --segment-mb 1 --pool 4 --config C $Q ;;
    prof) prof 500 prof --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_prof" -o kt -- python3 "$R/bench.py" --no-cpu-baseline --host-steps 0 ;;
    pmc)
      prof 150 pmc_fetch --pmc FETCH_SIZE -f csv -d "$R/gpurun_out/${T}_pmc_fetch" -o pf -- python3 "$R/bench.py" --steps 300 --warmup 50 $Q
      prof 150 pmc_write --pmc WRITE_SIZE -f csv -d "$R/gpurun_out/${T}_pmc_write" -o pw -- python3 "$R/bench.py" --steps 300 --warmup 50 $Q ;;
    stamps)
      RMQ_STAMPS=gpurun_out/${T}_st.csv RMQ_STAMPS_AT=100 run 200 "${T}_stamped.json" python bench.py --steps 600 --warmup 60 $Q
      python tools/pipe_stamps.py "gpurun_out/${T}_st.csv" > "gpurun_out/${T}_stamps.txt" 2>&1
      for d in 1 16; do RMQ_DEBUG=$d run 200 "${T}_dbg$d.json" python bench.py --steps 400 --warmup 40 $Q; done ;;
    dbg:*)  # dbg:B1,B2,...: timing-only RMQ_DEBUG lines (results invalid) beside a plain one
      run 200 "${T}_dbg0.json" python bench.py --steps 400 --warmup 40 $Q
      for d in $(echo "${step#dbg:}" | tr , ' '); do RMQ_DEBUG=$d run 200 "${T}_dbg$d.json" python bench.py --steps 400 --warmup 40 $Q; done ;;
    knob:*)  # knob:VAR=v1,v2,...: steady and 20-step lines per value of one environment knob
      kv=${step#knob:}; var=${kv%%=*}
      for val in $(echo "${kv#*=}" | tr , ' '); do
        env "$var=$val" timeout -k 10 200 python bench.py --steps 600 --warmup 60 $Q > "gpurun_out/${T}_${var}_${val}_600.json" 2>&1 || exit 1
        env "$var=$val" timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > "gpurun_out/${T}_${var}_${val}_20.json" 2>&1 || exit 1
      done ;;
    legs)  # the side legs (fetch, mixed, tier) on a short line
      run 300 "${T}_legs.json" python bench.py --steps 200 --warmup 20 --no-cpu-baseline --host-steps 0 ;;
    calls) run 200 "${T}_calls.json" python tools/fetch_calls.py ;;
    fetchkt)  # kernel trace of the fetch leg alone (its kernels replayed back to back, bench.py REPLAY)
      prof 200 fetchkt --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_fetchkt" -o kt -- python3 "$R/bench.py" --steps 20 --warmup 5 --fetch-rounds 10 --concurrent-rounds 0 --tier-rounds 0 --no-cpu-baseline --host-steps 0 ;;
    fetchprof|fetchprof:*)  # kernel trace of the fetch legs (short append run), current library and variants/NAME
      V=${step#fetchprof}; V=${V#:}
      FQ="--steps 100 --warmup 10 --no-cpu-baseline --concurrent-rounds 0 --host-steps 0"
      prof 300 fetchprof_cur --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_fetchprof_cur" -o kt -- python3 "$R/bench.py" $FQ
      if [ -n "$V" ]; then
        RMQ_LIB=$R/variants/$V/libripplemq_engine.so prof 300 fetchprof_$V --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_fetchprof_$V" -o kt -- python3 "$R/bench.py" $FQ
      fi ;;
    xstamps)  # phase stamps of one launch of the 2-rank rehearsal (transport kernel, 8 waves/workgroup)
      RMQ_STAMPS=gpurun_out/${T}_xst.csv RMQ_STAMPS_AT=60 run 300 "${T}_xstamped.json" python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 $Q
      python tools/pipe_stamps.py "gpurun_out/${T}_xst.csv" > "gpurun_out/${T}_xstamps.txt" 2>&1 ;;
    envab:*)  # envab:VAR=v[,CFG]: GPU tests with the knob set, then three pairs of 400- and 20-step lines off / on
      kv=${step#envab:}; CF=B; case $kv in *,*) CF=${kv#*,}; kv=${kv%%,*};; esac
      run 900 "${T}_envab_pytest.log" env "$kv" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "parity or golden or pipelined or config or large or world8 or replication"
      for k in 1 2 3; do
        run 200 "${T}_envab_off_$k.json" python bench.py --config $CF --steps 400 --warmup 40 $Q
        run 200 "${T}_envab_on_$k.json" env "$kv" python bench.py --config $CF --steps 400 --warmup 40 $Q
        run 200 "${T}_envab_off20_$k.json" python bench.py --config $CF --steps 20 --warmup 5 $Q
        run 200 "${T}_envab_on20_$k.json" env "$kv" python bench.py --config $CF --steps 20 --warmup 5 $Q
      done
      python3 tools/show_lines.py gpurun_out/${T}_envab_*.json ;;
    group)  # launch-group size sweep (20- and 600-step lines, two rounds)
      for k in 1 2; do
        for g in 4 5 6 8; do
          run 200 "${T}_g${g}_20_$k.json" python bench.py --steps 20 --warmup 8 --group $g $Q
          run 200 "${T}_g${g}_600_$k.json" python bench.py --steps 600 --warmup 60 --group $g $Q
        done
      done ;;
    Dprof)  # config D: a line, phase stamps of one launch, the apply launches' kernel trace
      DQ="--config D --pool 16 --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
      run 200 "${T}_D.json" python bench.py --steps 400 --warmup 40 $DQ
      RMQ_STAMPS=gpurun_out/${T}_Dst.csv RMQ_STAMPS_AT=60 run 200 "${T}_Dstamped.json" python bench.py --steps 200 --warmup 40 $DQ
      python tools/pipe_stamps.py "gpurun_out/${T}_Dst.csv" > "gpurun_out/${T}_Dstamps.txt" 2>&1 || true
      RMQ_SPLIT=2 prof 200 Dkt --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_Dkt" -o kt -- python3 "$R/bench.py" --steps 200 --warmup 20 $DQ ;;
    roles)  # phase stamps of the role-split stage 3 (RMQ_S3_ROLES=4) and of the default launch
      RMQ_S3_ROLES=4 RMQ_STAMPS=gpurun_out/${T}_rst.csv RMQ_STAMPS_AT=50 run 200 "${T}_rstamped.json" python bench.py --steps 300 --warmup 30 $Q
      RMQ_STAMPS=gpurun_out/${T}_st0.csv RMQ_STAMPS_AT=50 run 200 "${T}_stamped0.json" python bench.py --steps 300 --warmup 30 $Q
      python tools/roles_stamps.py "gpurun_out/${T}_rst.csv" > "gpurun_out/${T}_roles_stamps.txt" 2>&1
      python tools/pipe_stamps.py "gpurun_out/${T}_st0.csv" >> "gpurun_out/${T}_roles_stamps.txt" 2>&1 ;;
    coalesce)  # fetch legs with asynchronous fetch coalescing on (default) and off, three pairs
      FQ="--steps 100 --warmup 10 --no-cpu-baseline --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
      for k in 1 2 3; do
        run 200 "${T}_on_$k.json" python bench.py $FQ
        RMQ_FETCH_COALESCE=1 run 200 "${T}_off_$k.json" python bench.py $FQ
      done ;;
    caps:*)  # caps:S1:S2,S1:S2,...  ranking workgroup caps (RMQ_S1_WGS / RMQ_S2_WGS, 0 = none), 400- and 20-step lines, two rounds
      for k in 1 2; do
        for c in $(echo "${step#caps:}" | tr , ' '); do
          s1=${c%%:*}; s2=${c##*:}
          RMQ_S1_WGS=$s1 RMQ_S2_WGS=$s2 run 200 "${T}_${s1}_${s2}_400_$k.json" python bench.py --steps 400 --warmup 40 $Q
          RMQ_S1_WGS=$s1 RMQ_S2_WGS=$s2 run 200 "${T}_${s1}_${s2}_20_$k.json" python bench.py --steps 20 --warmup 5 $Q
        done
      done ;;
    fetchab3:*)  # fetchab3:V:OLD  fetch legs of the current library, variants/V and a whole older tree variants/OLD/tree
      V=${step#fetchab3:}; O=${V#*:}; V=${V%%:*}
      FQ="--steps 100 --warmup 10 --no-cpu-baseline --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
      for k in 1 2; do
        run 200 "${T}_cur_$k.json" python bench.py $FQ
        RMQ_LIB=$R/variants/$V/libripplemq_engine.so run 200 "${T}_${V}_$k.json" python bench.py $FQ
        (cd variants/$O/tree && timeout -k 10 200 python bench.py $FQ) > "gpurun_out/${T}_${O}_$k.json" 2> "gpurun_out/${T}_${O}_$k.json.err" || { echo "[gpu.sh] FAILED $O $k"; exit 1; }
      done ;;
    sq|memc)  # SQ / memory-pipeline counters of the apply launches (tools/pmc_apply.sh)
      bash tools/pmc_apply.sh "${T}_$step" $([ $step = sq ] && echo sq || echo mem) ;;
    *) echo "[gpu.sh] unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] $(date +%T) done"
