#!/bin/bash
# round-6 pass for a variant library (the tree keeps the validated build): the GPU
# suite on SO_V, clustered Greedy and random bench alternations (A = in-tree, B = SO_V)
#   bash tools/gpu_r06_var.sh TAG SO_V
set -o pipefail
T=$1; SO=$2
mkdir -p gpurun_out
AIGAR_SO=$(pwd)/$SO timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in 1 2; do
  echo -n "A "; timeout -k 10 100 python3 tools/clustered.py 200 || exit 1
  echo -n "B "; AIGAR_SO=$(pwd)/$SO timeout -k 10 100 python3 tools/clustered.py 200 || exit 1
done
bash tools/abn.sh $T 2 $SO || exit 1
