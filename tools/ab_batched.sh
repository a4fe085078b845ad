#!/bin/bash
# A/B of library builds on the batched line (16 C3 arenas stepped together) and the default line:
#   bash tools/ab_batched.sh TAG SO_1 [SO_2 ...]   (in-tree build = "base")
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for i in 1 2; do
  for so in base "$@"; do
    lib=""; [ $so != base ] && lib=$GRAFT_REPO_ROOT/$so
    n=$(basename $so .so)
    AIGAR_SO=$lib timeout -k 10 150 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-pixels \
      --batched-arenas 16 --no-c4 > $O/${TAG}_${n}_$i.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/${TAG}_${n}_$i.json').read().strip().splitlines()[-1]);b=d['batched'];print('%-16s' % '$n', 'c3 %.2f M' % (d['value']/1e6), 'obs %.4f' % d['breakdown_ms_per_step']['observe'], '| batched %.2f M' % (b['value']/1e6), 'obs frac %.3f' % b['roofline_k_observe']['frac'])"
  done
done
