#!/bin/bash
# usage (GPU box): bash tools/gpu_probe2.sh  -- translation micro, then k_observe store-policy A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 120 ./tools/var/tlb > gpurun_out/tlb.txt 2>&1 || { echo "tlb rc=$?"; cat gpurun_out/tlb.txt; exit 1; }
cat gpurun_out/tlb.txt
bash tools/ab.sh obswt tools/var/lib_obs_wt.so 3 || exit 1
bash tools/ab.sh obswt2 tools/var/lib_obs_wt2.so 3 || exit 1
