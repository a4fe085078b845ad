#!/bin/bash
# Round-3 GPU iteration: selected tests, default bench, rocprofv3 kernel trace of
# the timed graph region, PMC bytes of every step kernel (two passes).
# usage (GPU box): bash tools/gpu_r3.sh TAG [pytest targets...]
set -o pipefail
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|^E " gpurun_out/pytest_gpu_$TAG.log | head -20; exit 1; }
  tail -1 gpurun_out/pytest_gpu_$TAG.log
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench rc=$?"; tail gpurun_out/bench_$TAG.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --profile-run --steps 200 --warmup 20 > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $R && bash tools/pmc.sh $TAG || exit 1
echo done
