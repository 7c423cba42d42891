# Mixed leg pacing sweep (consumer passes per rounds of appends). bash tools/exp_mixed.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for k in 1 2; do for fe in 2 2.5; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --host-steps 0 --fetch-rounds 0 --tier-rounds 0 --mixed-fetch-every $fe > gpurun_out/r05mx_${fe}_$k.json 2> gpurun_out/r05mx_${fe}_$k.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r05mx_${fe}_$k.json').read().strip().splitlines()[-1]); m=d['mixed']; print('every $fe', round(m['append_msgs_per_s']/1e9,3), 'G app', round(m['fetch_records_per_s']/1e9,3), 'G fetched', m['fetches'], 'fetches', m['consumer_resets'], 'resets of', m['fetches']*m['requests_per_fetch'])"
done; done
