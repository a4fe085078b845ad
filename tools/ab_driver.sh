#!/bin/bash
# A/B of the in-tree build against another .so on the driver's own command line
# (--steps 20 --warmup 5: the window right after the start world's load).
#   bash tools/ab_driver.sh TAG SO_B [rounds]
set -o pipefail
TAG=$1; B=$2; N=${3:-4}
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for i in $(seq $N); do
  for v in A B; do
    so=""; [ $v = B ] && so=$GRAFT_REPO_ROOT/$B
    AIGAR_SO=$so timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pixels \
      --batched-arenas 0 --no-c4 > $O/${TAG}_${v}$i.json 2>/dev/null || { echo "ab $v failed"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/${TAG}_${v}$i.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,2), 'M  %.1f us/step' % (d['ms_per_step']*1e3))"
  done
done
