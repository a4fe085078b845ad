#!/bin/bash
# k_observe cost split (GPU box): kernel-trace durations and SQ counters of the
# in-tree build and of the stop / no-store variants in tools/var (results invalid,
# timing only).  usage: bash tools/obs_split.sh TAG VARIANT.so ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out
bash $R/tools/prof_ab.sh ${TAG}_obs "$@" > $R/gpurun_out/${TAG}_obs_prof.txt 2>&1 || { echo "prof rc=$?"; tail -5 $R/gpurun_out/${TAG}_obs_prof.txt; exit 1; }
grep -E "^==|k_observe" $R/gpurun_out/${TAG}_obs_prof.txt
i=0
for so in "" "$@"; do
  v=$(printf "\\x$(printf %x $((65 + i)))"); i=$((i + 1))
  AIGAR_SO=${so:+$R/$so} bash $R/tools/pmc_sq.sh ${TAG}_$v > /dev/null || { echo "pmc $v failed"; exit 1; }
  echo "== $v ${so:-in-tree}"; cat $R/gpurun_out/pmcsq_${TAG}_$v.txt
done
