#!/bin/bash
# round-6 A/B pass: GPU suite, then the in-tree build against variant builds
#   bash tools/gpu_r06_ab.sh TAG ROUNDS SO_B [SO_C ...]
set -o pipefail
T=$1; N=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
bash tools/abn.sh $T $N "$@" || exit 1
bash tools/prof_ab.sh $T "$@" > gpurun_out/${T}_prof.txt 2>&1 || exit 1
grep -E "^==|total kernel" gpurun_out/${T}_prof.txt
