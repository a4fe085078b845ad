#!/bin/bash
# usage (GPU box): bash tools/gpu_ab2.sh TAG SO_B [SO_C ...] -- GPU suite on the in-tree build, then A/B
# of the in-tree build against each variant (tools/ab.sh, 3 alternating rounds each)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest_gpu.log
i=0
for so in "$@"; do
  i=$((i + 1))
  echo "== B = $so"
  bash tools/ab.sh ${TAG}_$i $so 3 || exit 1
done
