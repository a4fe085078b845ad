#!/bin/bash
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_facade_nn.py tests/test_gpu_facade.py tests/test_gpu_run.py -m gpu -v --timeout 500 --timeout-method thread > gpurun_out/pytest_f2_$TAG.log 2>&1; rc=$?
grep -E "PASSED|FAILED|^E  " gpurun_out/pytest_f2_$TAG.log | head -40
exit $rc
