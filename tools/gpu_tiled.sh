mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_tiled.py -v --timeout 600 --timeout-method thread > gpurun_out/pytest_tiled_$1.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_tiled_$1.log
exit $rc
