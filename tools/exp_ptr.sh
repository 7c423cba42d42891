# Host cost per fetch call with and without the Python address cache (RMQ_PY_PTR_CACHE), two each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for k in 1 2; do for c in 1 0; do
  RMQ_PY_PTR_CACHE=$c timeout -k 10 200 python tools/fetch_calls.py > gpurun_out/r05P_calls_${c}_$k.json 2> gpurun_out/r05P_calls_${c}_$k.err || exit 1
  python3 -c "
import json,statistics; d=json.loads(open('gpurun_out/r05P_calls_${c}_$k.json').read().strip().splitlines()[-1]); print('cache $c', 'pinned sync', statistics.median(d['fetch_pinned_sync_us']), 'burst8/call', statistics.median(d['fetch_pinned_burst8_us_per_call']))"
done; done
