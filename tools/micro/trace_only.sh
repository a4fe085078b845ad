R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_exp2 -o run -- python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline > $R/gpurun_out/prof_exp2.log 2>&1 || exit 1
echo done
