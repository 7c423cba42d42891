cd /root/repo
for f in gpurun_out/b_*.log; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['mean_kernel_us'],2), 'us frac', round(d['roofline']['frac'],3))"; done
for f in gpurun_out/st_*.txt; do echo "== $f"; cat $f; done
