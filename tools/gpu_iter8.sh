#!/bin/bash
# usage (GPU box): bash tools/gpu_iter8.sh TAG SO_B -- GPU suite (in-tree), greedy and random A/B of the
# in-tree build against SO_B, pp-pass diagnostics and greedy phase timing
set -o pipefail
TAG=$1; B=$2
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest_gpu.log
echo "== greedy B = $B"; AB_ARGS="--policy greedy" bash tools/ab.sh ${TAG}_g $B 3 || exit 1
echo "== random B = $B"; bash tools/ab.sh ${TAG}_r $B 2 || exit 1
timeout -k 10 200 python tools/pp_diag.py > gpurun_out/${TAG}_ppdiag.txt 2>&1 || { echo "ppdiag rc=$?"; exit 1; }
grep nw gpurun_out/${TAG}_ppdiag.txt
timeout -k 10 200 python tools/phase_timing.py run 50 greedy > gpurun_out/${TAG}_pt_greedy.txt 2>&1 || { echo "pt rc=$?"; exit 1; }
grep -E "k_spawn_plan" gpurun_out/${TAG}_pt_greedy.txt | head -9
echo done
