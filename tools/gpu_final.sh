#!/bin/bash
# A whole measurement pass on one box (TAG): the GPU suite, smoke(), the default
# bench line, the driver's own command twice, kernel traces (random and greedy
# populations), the PMC bytes of every step kernel and the observation's SQ counters
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu.sh $TAG suite || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/${TAG}_smoke.log; exit 1; }
tail -1 $O/${TAG}_smoke.log
bash tools/gpu.sh $TAG bench || exit 1
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_bench_driver_cmd$k.json 2> $O/${TAG}_bench_driver_cmd$k.err || { echo "driver cmd failed"; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/${TAG}_bench_driver_cmd$k.json').read().strip().splitlines()[-1]);print('driver cmd %.2f M/s ms/step %.4f' % (d['value']/1e6, d['ms_per_step']))"
done
bash tools/gpu.sh $TAG prof prof_greedy pmc || exit 1
bash tools/pmc_sq.sh ${TAG} > /dev/null && cat $O/pmcsq_${TAG}.txt
