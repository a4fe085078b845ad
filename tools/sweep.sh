#!/bin/bash
# Batched-arena scale sweep (SURVEY.md §8d "scale sweeps"): env-steps/s and the
# observation kernel's effective GB/s as the number of independent arenas per
# GPU grows.  usage (GPU box): bash tools/sweep.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
OUT=gpurun_out/sweep_$TAG.jsonl; : > $OUT
run() {  # workload arenas steps
  timeout -k 10 240 python bench.py --workload $1 --arenas $2 --steps $3 --warmup 5 --no-cpu-baseline >> $OUT 2> gpurun_out/sweep_${TAG}_$1_$2.err \
    || { echo "sweep $1 x$2 failed rc=$?"; tail -5 gpurun_out/sweep_${TAG}_$1_$2.err; exit 1; }
  tail -1 $OUT | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%s x%d: %.3g env-steps/s, %.3f ms/step, k_observe %.1f us %.0f GB/s' % (sys.argv[1], int(sys.argv[2]), d['value'], d['ms_per_step'], r['avg_launch_ms']*1e3, r['achieved']))" $1 $2
}
run c3 1 100 && run c3 4 50 && run c3 16 20 && run c3 64 10 && \
run c5 8 50 && run c5 64 20 && run c5 256 10 && run c5 1024 5
echo done
