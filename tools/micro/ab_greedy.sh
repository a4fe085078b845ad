set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/ab_greedy.txt
for SO in aigar_amd/libaigar_hip.so tools/micro/libaigar_hip_prev.so aigar_amd/libaigar_hip.so tools/micro/libaigar_hip_prev.so; do
  AIGAR_SO=$GRAFT_REPO_ROOT/$SO timeout -k 10 120 python bench.py --policy greedy --steps 100 --warmup 10 --no-cpu-baseline --batched-arenas 0 > /tmp/b.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('/tmp/b.json')); print(sys.argv[1], d['value'], d['breakdown_ms_per_step'])" $SO >> gpurun_out/ab_greedy.txt
done
