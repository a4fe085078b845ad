#!/bin/bash
# parity check + bench at food reservation rounds 1..3
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python $R/tools/gpu_check.py > $R/gpurun_out/check_exp.log 2>&1 || { echo check failed; exit 1; }
for r in 1 2 3; do
  AIGAR_FOOD_ROUNDS=$r timeout -k 10 200 python $R/bench.py --steps 300 --warmup 30 --no-cpu-baseline > $R/gpurun_out/bench_rounds$r.json 2>/dev/null || exit 1
done
echo ok
