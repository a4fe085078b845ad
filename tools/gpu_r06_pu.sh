#!/bin/bash
# round-6 pellet-update pass: GPU suite, A/B against the previous build, phase timing
set -o pipefail
T=${1:-r06_pu}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
bash tools/abn.sh $T 3 ab/base.so || exit 1
export AIGAR_PT_SO=$PWD/ab/pt.so
timeout -k 10 150 python tools/phase_timing.py run 40 random > gpurun_out/${T}_pt_random.txt 2>&1 || exit 1
timeout -k 10 150 python tools/phase_timing.py run 40 greedy > gpurun_out/${T}_pt_greedy.txt 2>&1 || exit 1
grep -E "k_pel_update|k_food_commit" gpurun_out/${T}_pt_random.txt gpurun_out/${T}_pt_greedy.txt | grep -v -E "skew|per CU"
