#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
for p in random greedy; do
for r in 1 2 3 4; do
  AIGAR_FOOD_ROUNDS=$r timeout -k 10 300 python $R/bench.py --policy $p --steps 200 --warmup 100 --no-cpu-baseline > $R/gpurun_out/rb_${p}_$r.json 2>/dev/null || exit 1
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_greedy2 -o run -- python3 $R/bench.py --policy greedy --steps 100 --warmup 100 --no-cpu-baseline > $R/gpurun_out/prof_greedy2.log 2>&1 || exit 1
echo ok
