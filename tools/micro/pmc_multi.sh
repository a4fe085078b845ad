#!/bin/bash
# k_observe FETCH_SIZE / WRITE_SIZE for several library builds on one box.
# usage (GPU box): bash tools/micro/pmc_multi.sh SO...
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for SO in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    AIGAR_SO=$R/$SO timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex "k_observe" --output-format csv \
      -d $R/gpurun_out/pmcm_${i}_$C -o run -- python3 $R/bench.py --steps 30 --warmup 10 --no-cpu-baseline --batched-arenas 0 \
      > $R/gpurun_out/pmcm_${i}_$C.log 2>&1 || { echo "pmc $SO $C failed"; exit 1; }
  done
  echo "$i $SO" >> $R/gpurun_out/pmcm_index.txt
  i=$((i+1))
done
echo done
