set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 120 $R/tools/micro/launch_floor > $R/gpurun_out/launch_floor.log 2>&1 || exit 1
for r in 1 2 3 4; do
  AIGAR_FOOD_ROUNDS=$r timeout -k 10 200 python $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $R/gpurun_out/bench_r$r.json 2>/dev/null || exit 1
done
echo ok
