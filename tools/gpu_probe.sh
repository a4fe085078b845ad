#!/bin/bash
# Round-3 probe pass (GPU box): the kernel-floor micro, the tick-kernel floor A/B
# (empty-bodied variants, timing only), then the full round measurement.
# usage: bash tools/gpu_probe.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 120 ./tools/var/kfloor > gpurun_out/kfloor.txt 2>&1 || { echo "kfloor rc=$?"; exit 1; }
cat gpurun_out/kfloor.txt
bash tools/prof_ab.sh floor tools/var/lib_floor_opq.so tools/var/lib_floor_cmp.so > gpurun_out/floor_ab.txt 2>&1 || { echo "floor rc=$?"; tail gpurun_out/floor_ab.txt; exit 1; }
bash tools/gpu_final.sh $TAG
