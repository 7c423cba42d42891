# usage: bash tools/show_envs.sh <tag>: env, 20-step and 1000-step bench lines, stage-3 stamps
for f in gpurun_out/$1_*_env.txt; do
  b=${f%_env.txt}
  echo "== $(cat $f)"
  for s in b20 b1000; do
    python3 -c "
import json
d=json.loads(open('${b}_$s.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$s', round(d['value']/1e9,3),'G msgs/s  frac',round(r['frac'],3),' launch',round(r['mean_kernel_us'],1),'us')" 2>/dev/null || tail -2 ${b}_$s.json
  done
  grep -A4 "stage 3" ${b}_stamps.txt | head -5
done
