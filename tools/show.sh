tail -2 gpurun_out/pytest_gpu.log
for f in b_serial b_overlap; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step']*1000,2), 'us/step', {k: round(v,2) for k,v in d['kernels_us'].items()})"; done
