#!/bin/bash
# Greedy-population bench, in-tree library vs the given builds, alternating, same box.
# usage (GPU box): bash tools/micro/ab_greedy.sh SO...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/ab_greedy.txt
for rep in 1 2; do
  for SO in aigar_amd/libaigar_hip.so "$@"; do
    AIGAR_SO=$GRAFT_REPO_ROOT/$SO timeout -k 10 120 python bench.py --policy greedy --steps 100 --warmup 10 --no-cpu-baseline --batched-arenas 0 > /tmp/b.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('/tmp/b.json')); print(sys.argv[1], round(d['value']), d['ms_per_step'], d['breakdown_ms_per_step'], d['world']['serial_work_per_tick'])" $SO >> gpurun_out/ab_greedy.txt
  done
done
