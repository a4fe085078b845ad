#!/bin/bash
# usage (GPU box): bash tools/gpu_iter5.sh TAG SO_B -- GPU suite, A/B against SO_B, kernel traces of both
set -o pipefail
TAG=$1; B=$2
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_run.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_run.log 2>&1 || { echo "pytest run rc=$?"; tail -30 gpurun_out/${TAG}_pytest_run.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest_gpu.log
bash tools/ab.sh ${TAG} $B 3 || exit 1
bash tools/prof_ab.sh ${TAG} $B > gpurun_out/${TAG}_prof_ab.txt 2>&1 || { echo "prof rc=$?"; exit 1; }
grep -E "^==|total kernel" gpurun_out/${TAG}_prof_ab.txt
echo done
