#!/bin/bash
# late-game C3: long warm-up, then the usual timed steps; reports serial work per tick
set -o pipefail
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  AIGAR_FOOD_ROUNDS=$r timeout -k 10 400 python $R/bench.py --steps 200 --warmup ${WARM:-3000} --no-cpu-baseline > $R/gpurun_out/late_r$r.json 2>/dev/null || exit 1
done
echo ok
