#!/bin/bash
# Alternating bench runs of the in-tree build (A) and variant builds (B, C, ...):
#   bash tools/abn.sh TAG ROUNDS SO_B [SO_C ...]   (GPU box; extra bench args: $AB_ARGS)
# a variant "env:NAME=VALUE" runs the in-tree build with that variable set instead
set -o pipefail
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out; mkdir -p $O; cd $R
for i in $(seq $N); do
  k=0
  for so in "" "$@"; do
    v=$(printf "\\x$(printf %x $((65 + k)))"); k=$((k + 1))
    envv="AIGAR_SO=${so:+$R/$so}"
    case "$so" in env:*) envv="${so#env:}";; esac
    env "$envv" timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pixels \
      --batched-arenas 0 --no-c4 $AB_ARGS > $O/${TAG}_abn_${v}$i.json 2>/dev/null || { echo "abn $v failed"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/${TAG}_abn_${v}$i.json').read().strip().splitlines()[-1]);b=d['breakdown_ms_per_step'];print('$v', round(d['value']/1e6,2), 'M/s  ms/step %.4f tick %.4f obs %.4f' % (d['ms_per_step'], b['tick'], b['observe']))"
  done
done
