#!/bin/bash
# greedy C3: food reservation rounds sweep + one kernel-trace profile
set -o pipefail
R=$GRAFT_REPO_ROOT
for r in 1 2 4 8; do
  AIGAR_FOOD_ROUNDS=$r timeout -k 10 300 python $R/bench.py --policy greedy --steps 150 --warmup 100 --no-cpu-baseline > $R/gpurun_out/greedy_r$r.json 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp
AIGAR_FOOD_ROUNDS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_greedy -o run -- python3 $R/bench.py --policy greedy --steps 100 --warmup 100 --no-cpu-baseline > $R/gpurun_out/prof_greedy.log 2>&1 || exit 1
echo ok
