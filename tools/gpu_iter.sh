#!/bin/bash
# One GPU iteration on the gpurun box: parity check, short bench, kernel-trace profile.
# usage: bash tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 500 python $R/tools/gpu_check.py > $R/gpurun_out/check_$TAG.log 2>&1 || { echo "check failed rc=$?"; exit 1; }
timeout -k 10 300 python $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err || { echo "bench failed rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --batched-arenas 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed rc=$?"; exit 1; }
echo done
