#!/bin/bash
# SQ instruction / wait counters for the observation kernel (one pass, 8 SQ slots).
# usage (GPU box): bash tools/pmc_sq.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_observe" --output-format csv \
  -d $R/gpurun_out/pmcsq_${TAG} -o run -- python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --batched-arenas 0 \
  > $R/gpurun_out/pmcsq_${TAG}.log 2>&1 || { echo "pmc failed rc=$?"; exit 1; }
echo done
