#!/bin/bash
# Cache-level counters of every kernel of the bench's timed step (one pass per
# counter group, within gfx950's per-block limits: <= 4 TCP, <= 2 TA, <= 4 TCC, <= 8 SQ).
# usage (GPU box): bash tools/pmc_l1.sh TAG
set -o pipefail
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || echo "list rc=$?"
i=0
for C in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
         "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv \
    -d $R/gpurun_out/pmcl1_${TAG}_$i -o run -- python3 $R/bench.py --profile-run --steps 30 --warmup 10 "$@" \
    > $R/gpurun_out/pmcl1_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 $R/gpurun_out/pmcl1_${TAG}_$i.log; exit 1; }
done
echo done
