#!/bin/bash
# GPU box: tiled tests, then the rocprofv3 kernel-trace summary of the timed graph region only
# (bench.py --profile-run: warm-up + timed graph replays, one call per step), C3 from the matured start.
set -o pipefail
TAG=${1:-x}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py -m gpu -v --timeout 500 --timeout-method thread > gpurun_out/pytest_tiled_$TAG.log 2>&1; echo "tiled rc=$?"; grep -E "FAILED|^E  " gpurun_out/pytest_tiled_$TAG.log | head
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --profile-run --steps 200 --warmup 20 > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed rc=$?"; tail $R/gpurun_out/prof_$TAG.log; exit 1; }
echo done
