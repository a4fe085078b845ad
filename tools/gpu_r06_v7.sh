#!/bin/bash
# round 6, v7: GPU suite (exact tolerance), the observation's ordered per-square
# pellet sums (A, in-tree) vs the previous commit (B), SQ counters of k_observe
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu.sh r06_v7 suite ab:tools/var/base_v6.so:3 || exit 1
bash tools/pmc_sq.sh r06_v7_A > /dev/null && cat $O/pmcsq_r06_v7_A.txt
