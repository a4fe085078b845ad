#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python $R/tools/gpu_check.py > $R/gpurun_out/check_p2.log 2>&1 || { echo check failed; exit 1; }
timeout -k 10 600 python -m pytest $R/tests/test_gpu_greedy.py $R/tests/test_gpu_parity.py -x -q > $R/gpurun_out/pytest_p2.log 2>&1 || { echo pytest failed; exit 1; }
for p in random greedy; do
  timeout -k 10 300 python $R/bench.py --policy $p --steps 200 --warmup 100 --no-cpu-baseline > $R/gpurun_out/bench_p2_$p.json 2> $R/gpurun_out/bench_p2_$p.err || exit 1
done
echo ok
