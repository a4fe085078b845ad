#!/bin/bash
# SQ instruction / wait counters for the observation kernel (one pass, 8 SQ slots),
# on the bench's profile run (the C3 graph replays); AIGAR_SO picks another build.
# usage (GPU box): [AIGAR_SO=ab/x.so] bash tools/pmc_sq.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_observe" --output-format csv \
  -d $R/gpurun_out/pmcsq_${TAG} -o run -- python3 $R/bench.py --profile-run --steps 30 --warmup 10 \
  > $R/gpurun_out/pmcsq_${TAG}.log 2>&1) || { echo "pmc failed rc=$?"; exit 1; }
python3 - $R/gpurun_out/pmcsq_${TAG}/run_counter_collection.csv <<'PY' | tee $R/gpurun_out/pmcsq_${TAG}.txt
import csv, sys, collections
v = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "k_observe<double, true" not in r["Kernel_Name"]:
        continue
    v[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
tot = collections.defaultdict(float)
for d in v.values():
    for k, x in d.items():
        tot[k] += x
w = tot["SQ_WAVES"]
print("k_observe<double, true>: %d dispatches, %.0f waves each" % (len(v), w / max(1, len(v))))
for k in sorted(tot):
    if k != "SQ_WAVES":
        print("  %-20s per wave %10.1f" % (k, tot[k] / max(1.0, w)))
PY
