#!/bin/bash
# round-6 pass: GPU suite, clustered Greedy A/B against SO_B, random bench A/B, and
# k_merge_pv's split on the clustered world from the cost-diagnostic builds
# (ab/nopv.so: no playerVirusOverlap serial pass; ab/nomerge.so: no mergePlayerCells)
#   bash tools/gpu_r06_diag.sh TAG SO_B
set -o pipefail
T=$1; SO=$2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in 1 2; do
  echo -n "A "; timeout -k 10 100 python3 tools/clustered.py 200 || exit 1
  echo -n "B "; AIGAR_SO=$(pwd)/$SO timeout -k 10 100 python3 tools/clustered.py 200 || exit 1
done
bash tools/abn.sh $T 2 $SO || exit 1
R=$(pwd); cd /tmp && export TMPDIR=/tmp
for v in "" nopv nomerge; do
  so=${v:+$R/ab/$v.so}
  AIGAR_SO=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_d${v} -o run -- python3 $R/tools/clustered.py 60 > $R/gpurun_out/${T}_d${v}.log 2>&1 || { echo "prof $v failed"; exit 1; }
  echo "== ${v:-in-tree}"; python3 $R/tools/prof_summary.py $R/gpurun_out/${T}_d${v}/run_kernel_stats.csv > $R/gpurun_out/${T}_d${v}_summary.txt
  grep -E "k_merge_pv|k_spawn_plan|total" $R/gpurun_out/${T}_d${v}_summary.txt
done
