#!/bin/bash
# Full GPU test suite on the gpurun box: bash tools/gpu_suite.sh TAG [pytest targets...]
set -o pipefail
TAG=${1:-x}; shift
mkdir -p gpurun_out
T=${@:-tests}
timeout -k 10 1000 python -u -m pytest $T -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_$TAG.log | head -20
tail -2 gpurun_out/pytest_gpu_$TAG.log
exit $rc
