#!/bin/bash
# usage (GPU box): bash tools/gpu_iter6.sh TAG SO_B SO_C -- GPU suite, A/B against SO_B and SO_C, phase timing
set -o pipefail
TAG=$1; B=$2; C=$3
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest_gpu.log
echo "== B = $B"; bash tools/ab.sh ${TAG}_b $B 3 || exit 1
echo "== B = $C"; bash tools/ab.sh ${TAG}_c $C 3 || exit 1
timeout -k 10 200 python tools/phase_timing.py run 50 random > gpurun_out/${TAG}_pt_random.txt 2>&1 || { echo "pt rc=$?"; exit 1; }
grep -E "k_food_prep" gpurun_out/${TAG}_pt_random.txt | head -8
echo done
