#!/bin/bash
# C3 bench with both synthetic populations (+ facade/greedy GPU tests)
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest $R/tests/test_gpu_facade.py -x -q > $R/gpurun_out/pytest_facade.log 2>&1 || { echo facade tests failed; exit 1; }
for p in random greedy; do
  timeout -k 10 300 python $R/bench.py --policy $p --steps 200 --warmup 50 > $R/gpurun_out/bench_$p.json 2> $R/gpurun_out/bench_$p.err || exit 1
done
echo ok
