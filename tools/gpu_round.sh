#!/bin/bash
# Round GPU pass: tests (optionally a subset), then tools/gpu_iter.sh TAG.
# usage (GPU box): bash tools/gpu_round.sh TAG [pytest targets...]
set -o pipefail
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
T=${@:-tests}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
bash tools/gpu_iter.sh $TAG
