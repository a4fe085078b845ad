#!/bin/bash
# round-6 Greedy A/B pass: GPU suite, Greedy and random alternations against SO_B, Greedy kernel profiles
#   bash tools/gpu_r06_abg.sh TAG SO_B
set -o pipefail
T=$1; SO=$2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
AB_ARGS="--policy greedy" bash tools/abn.sh ${T}g 3 $SO || exit 1
bash tools/abn.sh $T 2 $SO || exit 1
R=$(pwd); cd /tmp && export TMPDIR=/tmp
i=0
for so in "" "$SO"; do
  v=$(printf "\\x$(printf %x $((65 + i)))"); i=$((i + 1))
  AIGAR_SO=${so:+$R/$so} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_pg_$v -o run -- python3 $R/bench.py --profile-run --steps 100 --warmup 20 --policy greedy > $R/gpurun_out/${T}_pg_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
  echo "== $v ${so:-in-tree}"; python3 $R/tools/prof_summary.py $R/gpurun_out/${T}_pg_$v/run_kernel_stats.csv | grep -E "k_spawn_plan|total"
done
