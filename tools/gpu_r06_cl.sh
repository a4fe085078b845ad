#!/bin/bash
# round-6 clustered-Greedy pass: GPU suite, clustered Greedy ticks (tools/clustered.py)
# and bench alternations against SO_B, a kernel profile of the clustered ticks
#   bash tools/gpu_r06_cl.sh TAG SO_B
set -o pipefail
T=$1; SO=$2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in 1 2; do
  echo -n "A "; timeout -k 10 100 python3 tools/clustered.py 200 || exit 1
  echo -n "B "; AIGAR_SO=$(pwd)/$SO timeout -k 10 100 python3 tools/clustered.py 200 || exit 1
done
AB_ARGS="--policy greedy" bash tools/abn.sh ${T}g 2 $SO || exit 1
bash tools/abn.sh $T 2 $SO || exit 1
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_pcl -o run -- python3 $R/tools/clustered.py 100 > $R/gpurun_out/${T}_pcl.log 2>&1 || { echo "prof failed"; exit 1; }
python3 $R/tools/prof_summary.py $R/gpurun_out/${T}_pcl/run_kernel_stats.csv > $R/gpurun_out/${T}_pcl_summary.txt; head -14 $R/gpurun_out/${T}_pcl_summary.txt
if [ -f $R/ab/pt.so ]; then  # the phase-timing build on the clustered world (greedy)
  cd $R && AIGAR_PT_SO=$R/ab/pt.so AIGAR_PT_START=$R/data/c3_greedy_late.npz timeout -k 10 200 python3 tools/phase_timing.py run 30 greedy > gpurun_out/${T}_ptcl.log 2>&1 || { echo "pt failed"; exit 1; }
  grep -E "k_spawn_plan|k_players|pp serial|pp group" gpurun_out/${T}_ptcl.log
fi
