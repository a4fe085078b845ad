#!/bin/bash
# k_observe cost per phase (GPU box): the in-tree build and builds that stop
# after the prologue / walk / rank (-DAIGAR_OBS_STOP=1..3, results invalid):
# kernel trace durations and SQ instruction counters of each.
# usage: bash tools/obs_phase_cost.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out
bash $R/tools/prof_ab.sh ${TAG}_obs tools/var/lib_obsstop1.so tools/var/lib_obsstop2.so tools/var/lib_obsstop3.so > $R/gpurun_out/${TAG}_obs_prof.txt 2>&1 || { echo "prof rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 3; do
  so=""; [ $v -gt 0 ] && so=$R/tools/var/lib_obsstop$v.so
  AIGAR_SO=$so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES --output-format csv \
    -d $R/gpurun_out/${TAG}_obspmc_$v -o run -- python3 $R/bench.py --profile-run --steps 20 --warmup 5 \
    > $R/gpurun_out/${TAG}_obspmc_$v.log 2>&1 || { echo "pmc $v rc=$?"; tail -3 $R/gpurun_out/${TAG}_obspmc_$v.log; exit 1; }
done
echo done
