#!/bin/bash
# round 6, v6: Greedy population with / without the policy fused into the observation
# (A/B), the greedy kernel profile, and the k_observe cost split
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out; mkdir -p $O; cd $R
for i in 1 2 3; do
  for v in A B; do
    env_b=""; [ $v = B ] && env_b="AIGAR_NO_GREEDY_FUSE=1"
    env $env_b timeout -k 10 120 python bench.py --policy greedy --steps 200 --warmup 20 --no-cpu-baseline --no-pixels \
      --batched-arenas 0 > $O/r06_v6_gab_${v}$i.json 2>/dev/null || { echo "greedy ab $v failed"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/r06_v6_gab_${v}$i.json').read().strip().splitlines()[-1]);b=d['breakdown_ms_per_step'];print('greedy $v', round(d['value']/1e6,2), 'M/s ms/step %.4f obs %.4f' % (d['ms_per_step'], b['observe']))"
  done
done
bash tools/gpu.sh r06_v6 prof_greedy || exit 1
bash tools/obs_split.sh r06_v6 tools/var/lib_obsstop2.so tools/var/lib_obsstop3.so tools/var/lib_obsstop4.so tools/var/lib_obsnostore.so
