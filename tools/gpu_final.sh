#!/bin/bash
# Round-end measurement on the GPU box: full GPU suite, rocprofv3 kernel traces
# (random and greedy populations), PMC bytes of every step kernel, then the
# default bench (which reads the PMC summary written here).
# usage (GPU box): bash tools/gpu_final.sh TAG      e.g. r03_v2
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest_gpu.log | head; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --profile-run --steps 200 --warmup 20 > $R/gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof_greedy -o run -- python3 $R/bench.py --profile-run --steps 100 --warmup 20 --policy greedy > $R/gpurun_out/${TAG}_prof_greedy.log 2>&1 || { echo "prof greedy rc=$?"; exit 1; }
cd $R
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv > gpurun_out/${TAG}_c3_kernel_summary.txt || exit 1
python3 tools/prof_summary.py gpurun_out/${TAG}_prof_greedy/run_kernel_stats.csv > gpurun_out/${TAG}_greedy_kernel_summary.txt || exit 1
bash tools/pmc.sh $TAG || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE gpurun_out/${TAG}_pmc_c3.json > gpurun_out/${TAG}_pmc_c3.txt || exit 1
cp gpurun_out/${TAG}_pmc_c3.json profiles/${TAG}_pmc_c3.json
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { echo "bench rc=$?"; tail gpurun_out/${TAG}_bench_default.err; exit 1; }
cat gpurun_out/${TAG}_c3_kernel_summary.txt | head -14
echo done
