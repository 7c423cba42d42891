# Run one gpurun command, waiting while the pool has no free box (exit 3 / transient: nothing ran,
# nothing charged). Any other outcome ends it. usage: tools/gpurun_when_free.sh <timeout> <out> <cmd>
T=$1; O=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$O" 2>&1
  rc=$?
  if grep -q "status=transient" "$O"; then sleep 90; continue; fi
  exit $rc
done
exit 3
