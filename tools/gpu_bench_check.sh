#!/bin/bash
# GPU box: selected tests, then the default bench and a 2-rank gloo rehearsal of the N > 1 path
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_tiled.py -m gpu -v --timeout 500 --timeout-method thread -k "matured or c3_tiled or small_halo" > gpurun_out/pytest_sel_$TAG.log 2>&1; echo "pytest rc=$?"; grep -E "PASSED|FAILED|^E  " gpurun_out/pytest_sel_$TAG.log | head -20
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
AIGAR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { echo "bench2 failed rc=$?"; tail -20 gpurun_out/bench2_$TAG.err; exit 1; }
echo done
