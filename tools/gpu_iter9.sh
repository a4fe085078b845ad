#!/bin/bash
# usage (GPU box): bash tools/gpu_iter9.sh TAG SO_B -- GPU suite (in-tree), random A/B (4 rounds) of the
# in-tree build against SO_B, kernel trace of the in-tree build
set -o pipefail
TAG=$1; B=$2
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_pytest_gpu.log
echo "== random B = $B"; bash tools/ab.sh ${TAG}_r $B 4 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  if [ $v = A ]; then so=""; else so=$R/$B; fi
  AIGAR_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof_$v -o run -- python3 $R/bench.py --profile-run --steps 200 --warmup 20 > $R/gpurun_out/${TAG}_prof_$v.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  python3 $R/tools/prof_summary.py $R/gpurun_out/${TAG}_prof_$v/run_kernel_stats.csv > $R/gpurun_out/${TAG}_${v}_kernel_summary.txt || exit 1
  echo $v; head -3 $R/gpurun_out/${TAG}_${v}_kernel_summary.txt; grep total $R/gpurun_out/${TAG}_${v}_kernel_summary.txt
done
echo done
