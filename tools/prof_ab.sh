#!/bin/bash
# Kernel-trace profiles of the in-tree build (A) and variant builds (B...):
# bash tools/prof_ab.sh TAG SO_B [SO_C ...]   (GPU box)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for so in "" "$@"; do
  [ -n "$so" ] && so=$R/$so
  v=$(printf "\\x$(printf %x $((65 + i)))"); i=$((i + 1))
  AIGAR_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_$v -o run -- python3 $R/bench.py --profile-run --steps 200 --warmup 20 > $R/gpurun_out/prof_${TAG}_$v.log 2>&1 || { echo "prof $v rc=$?"; exit 1; }
  echo "== $v ${so:-in-tree}"
  python3 $R/tools/prof_summary.py $R/gpurun_out/prof_${TAG}_$v/run_kernel_stats.csv || exit 1
done
