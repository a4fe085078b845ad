#!/bin/bash
# round 6, v4: the whole GPU suite at exact float tolerance (no -x: every failure listed),
# then glibc trig vs correctly rounded trig (A/B, random population), then the Greedy
# population with and without the policy fused into the observation
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/r06_v4_pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/r06_v4_pytest_gpu.log | tail -25
[ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "suite rc=$rc"; exit 1; }
bash tools/gpu.sh r06_v4 ab:tools/var/lib_crtrig.so:3 || exit 1
for i in 1 2 3; do
  for v in A B; do
    env_b=""; [ $v = B ] && env_b="AIGAR_NO_GREEDY_FUSE=1"
    env $env_b timeout -k 10 120 python bench.py --policy greedy --steps 200 --warmup 20 --no-cpu-baseline --no-pixels \
      --batched-arenas 0 > $O/r06_v4_gab_${v}$i.json 2>/dev/null || { echo "greedy ab $v failed"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/r06_v4_gab_${v}$i.json').read().strip().splitlines()[-1]);print('greedy $v', round(d['value']/1e6,2), 'M/s ms/step %.4f' % d['ms_per_step'])"
  done
done
