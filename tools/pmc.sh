#!/bin/bash
# HBM-side byte counters for EVERY kernel of the bench's timed step (FETCH_SIZE
# and WRITE_SIZE do not fit one TCC pass on gfx950: one pass each).
# usage (GPU box): bash tools/pmc.sh TAG [extra bench.py args]
set -o pipefail
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv \
    -d $R/gpurun_out/pmc_${TAG}_$C -o run -- python3 $R/bench.py --profile-run --steps 30 --warmup 10 "$@" \
    > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "pmc $C failed rc=$?"; exit 1; }
done
echo done
