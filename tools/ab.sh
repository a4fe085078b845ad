#!/bin/bash
# A/B of two library builds on one box (gpurun): alternating short C3 bench runs.
# usage: bash tools/ab.sh TAG SO_B [rounds]   (A = the in-tree libaigar_hip.so)
set -o pipefail
TAG=$1; B=$2; N=${3:-3}
mkdir -p gpurun_out
for i in $(seq $N); do
  for v in A B; do
    if [ $v = A ]; then so=""; else so=$B; fi
    AIGAR_SO=$so timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pixels --batched-arenas 0 --no-c4 $AB_ARGS > gpurun_out/ab_${TAG}_${v}$i.json 2>/dev/null || { echo "bench $v rc=$?"; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab_${TAG}_${v}$i.json').read().strip().splitlines()[-1]);b=d['breakdown_ms_per_step'];print('$v', round(d['value']/1e6,2), 'M/s  ms/step %.4f tick %.4f obs %.4f' % (d['ms_per_step'], b['tick'], b['observe']))"
  done
done
