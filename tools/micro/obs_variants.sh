#!/bin/bash
# A/B of k_observe builds (tools/micro/libaigar_hip_*.so vs the in-tree library): C3 x1 and x16, C5-size x64.
# usage (GPU box): bash tools/micro/obs_variants.sh SO...
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
OUT=gpurun_out/obs_variants.txt; : > $OUT
for SO in aigar_amd/libaigar_hip.so "$@"; do
  for CFG in "c3 1 100" "c3 16 20" "c5 64 20"; do
    set -- $CFG
    AIGAR_SO=$R/$SO timeout -k 10 120 python bench.py --workload $1 --arenas $2 --steps $3 --warmup 5 --no-cpu-baseline --batched-arenas 0 > /tmp/b.json 2>/tmp/b.err || { echo "fail $SO $CFG"; tail -3 /tmp/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('/tmp/b.json')); r=d['roofline']; print('%-40s %s x%-3s %.4g env-steps/s %.3f ms obs %.1f us %.0f GB/s' % (sys.argv[1], sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['avg_launch_ms']*1e3, r['achieved']))" $SO $1 $2 | tee -a $OUT
  done
done
