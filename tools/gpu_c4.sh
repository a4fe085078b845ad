#!/bin/bash
# C4 rehearsal on one GPU box: bench.py --gpus N with N ranks sharing the card
# (gloo backend, messages staged through host memory: RCCL cannot put two ranks
# on one device), plus the default N = 1 line.  bash tools/gpu_c4.sh TAG [N...]
set -o pipefail
TAG=${1:-x}; shift
NS=${@:-2 8}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench_n1_$TAG.json 2> gpurun_out/bench_n1_$TAG.err || exit 1
for N in $NS; do
  AIGAR_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 50 --warmup 10 \
    --no-cpu-baseline --no-pixels --batched-arenas 0 > gpurun_out/bench_n${N}_gloo_$TAG.json 2> gpurun_out/bench_n${N}_gloo_$TAG.err || exit 1
done
tail -c 600 gpurun_out/bench_n1_$TAG.json
