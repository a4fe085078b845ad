#!/bin/bash
# usage (GPU box): bash tools/gpu_iter7.sh TAG SO_B -- greedy phase timing (in-tree diagnostics build),
# greedy A/B of the in-tree build against SO_B, then the greedy / pp parity tests on SO_B
set -o pipefail
TAG=$1; B=$2
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 200 python tools/phase_timing.py run 50 greedy > gpurun_out/${TAG}_pt_greedy.txt 2>&1 || { echo "pt rc=$?"; exit 1; }
grep -E "k_spawn_plan" gpurun_out/${TAG}_pt_greedy.txt | head -9
echo "== greedy B = $B"; AB_ARGS="--policy greedy" bash tools/ab.sh ${TAG}_g $B 3 || exit 1
AIGAR_SO=$R/$B timeout -k 10 400 python -u -m pytest tests/test_gpu_greedy.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_b.log 2>&1 || { echo "pytest B rc=$?"; tail -30 gpurun_out/${TAG}_pytest_b.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest_b.log
timeout -k 10 200 python tools/pp_diag.py > gpurun_out/${TAG}_ppdiag.txt 2>&1 || { echo "ppdiag rc=$?"; exit 1; }
cat gpurun_out/${TAG}_ppdiag.txt | grep nw
echo done
