#!/bin/bash
# round 6, v4: the whole GPU suite at exact float tolerance (no -x: every failure listed),
# then glibc trig vs correctly rounded trig (A/B), then the k_observe cost split
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/r06_v4_pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/r06_v4_pytest_gpu.log | tail -25
[ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "suite rc=$rc"; exit 1; }
bash tools/gpu.sh r06_v4 ab:tools/var/lib_crtrig.so:3 || exit 1
bash tools/obs_split.sh r06_v4 tools/var/lib_obsstop2.so tools/var/lib_obsstop3.so tools/var/lib_obsstop4.so tools/var/lib_obsnostore.so
