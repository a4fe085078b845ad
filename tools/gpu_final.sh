#!/bin/bash
# Session-closing GPU pass (gpurun box): full GPU suite, default bench (all side
# lines), rocprofv3 kernel trace of the timed graph region, PMC bytes of k_observe.
# usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench rc=$?"; tail gpurun_out/bench_$TAG.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --profile-run --steps 200 --warmup 20 > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $R && bash tools/pmc.sh $TAG || exit 1
echo done
