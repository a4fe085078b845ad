#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of k_observe for the in-tree library and one variant, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for V in base:$R/aigar_amd/libaigar_hip.so alt:$R/$1; do
  T=${V%%:*}; SO=${V#*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    AIGAR_SO=$SO timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex "k_observe" --output-format csv \
      -d $R/gpurun_out/pmcab_${T}_$C -o run -- python3 $R/bench.py --steps 30 --warmup 10 --no-cpu-baseline --batched-arenas 0 \
      > $R/gpurun_out/pmcab_${T}_$C.log 2>&1 || { echo "pmc $T $C failed"; exit 1; }
  done
done
echo done
