set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out
for cfg in "20 5" "20 50" "100 5" "200 20" "20 5"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-pixels --batched-arenas 0 --no-c4 > $O/stepsweep_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/stepsweep_$1_$2.json').read().strip().splitlines()[-1]);print('steps $1 warmup $2: %.2f M  %.1f us/step' % (d['value']/1e6, d['ms_per_step']*1e3))"
done
