#!/bin/bash
# One parameterised GPU-box pass (replaces the per-iteration gpu_iter*/gpu_probe*/gpu_r3 scripts).
#   bash tools/gpu.sh TAG STEP [STEP ...]
# Steps run in order; the first failure ends the pass (no GPU step runs after a failed one).
#   suite[:targets]   pytest -m gpu (targets comma-separated; default: tests)
#   bench             default bench line (N = 1)              -> gpurun_out/TAG_bench.json
#   quick             bench without side lines / cpu baseline  -> gpurun_out/TAG_quick.json
#   prof              rocprofv3 kernel trace of the timed graph region (random population)
#   prof_greedy       the same with the Greedy population
#   pmc               FETCH_SIZE / WRITE_SIZE passes of every step kernel + summary
#   c4time            tools/c4_tile_timing.py 8 40 (per-tile phases, serialized)
#   c4prof            rocprofv3 kernel trace of tools/c4_tile_timing.py 8 20
#   c4solo            tools/c4_solo.py 8 200 (each tile alone, aigar_tile_run graph, loopback exchange)
#   gloo:N            bench.py --gpus N rehearsal (N ranks sharing the card over gloo)
#   ab:SO_B[:rounds]  alternating bench runs of the in-tree build against SO_B (extra bench args: $AB_ARGS)
#   ppdiag            tools/pp_diag.py on tools/var/lib_ppdiag.so (why the parallel pp pass fell back)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out
mkdir -p $O; cd $R
fail() { echo "$1 rc=$2"; [ -n "$3" ] && tail -30 "$3"; exit 1; }
prof() {  # name, extra bench / script args...
  local nm=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/${TAG}_$nm -o run -- python3 "$@" > $O/${TAG}_$nm.log 2>&1) || fail "$nm" $? $O/${TAG}_$nm.log
  python3 tools/prof_summary.py $O/${TAG}_$nm/run_kernel_stats.csv > $O/${TAG}_${nm}_summary.txt || fail "summary" $?
  head -16 $O/${TAG}_${nm}_summary.txt
}
for S in "$@"; do
  case $S in
    suite*)
      T=tests; [ "$S" != suite ] && T=$(echo ${S#suite:} | tr , ' ')
      timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread \
        > $O/${TAG}_pytest_gpu.log 2>&1 || { rc=$?; grep -E "FAILED|ERROR|^E  " $O/${TAG}_pytest_gpu.log | head -20; fail suite $rc; }
      tail -1 $O/${TAG}_pytest_gpu.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || fail bench $? $O/${TAG}_bench.err
      tail -c 400 $O/${TAG}_bench.json ;;
    quick)
      timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pixels --batched-arenas 0 \
        > $O/${TAG}_quick.json 2> $O/${TAG}_quick.err || fail quick $? $O/${TAG}_quick.err
      python3 -c "import json;d=json.loads(open('$O/${TAG}_quick.json').read().strip().splitlines()[-1]);b=d['breakdown_ms_per_step'];print('quick %.2f M/s ms/step %.4f tick %.4f obs %.4f' % (d['value']/1e6, d['ms_per_step'], b['tick'], b['observe']))" ;;
    prof) prof prof $R/bench.py --profile-run --steps 200 --warmup 20 ;;
    prof_greedy) prof prof_greedy $R/bench.py --profile-run --steps 100 --warmup 20 --policy greedy ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${TAG}_$C \
          -o run -- python3 $R/bench.py --profile-run --steps 30 --warmup 10 > $O/pmc_${TAG}_$C.log 2>&1) || fail "pmc $C" $?
      done
      python3 tools/pmc_summary.py $O/pmc_${TAG}_FETCH_SIZE $O/pmc_${TAG}_WRITE_SIZE $O/${TAG}_pmc_c3.json \
        > $O/${TAG}_pmc_c3.txt || fail pmc_summary $?
      head -20 $O/${TAG}_pmc_c3.txt ;;
    c4time)
      timeout -k 10 300 python -u tools/c4_tile_timing.py 8 40 > $O/${TAG}_c4_tiles.json 2> $O/${TAG}_c4_tiles.err \
        || fail c4time $? $O/${TAG}_c4_tiles.err
      python3 -c "import json;d=json.load(open('$O/${TAG}_c4_tiles.json'));print('max tile %.1f us' % d['max_tile_total_us'], d['untiled_us']); [print(r) for r in d['per_tile_us']]" ;;
    c4prof) prof c4prof $R/tools/c4_tile_timing.py 8 20 ;;
    c4solo)
      timeout -k 10 300 python -u tools/c4_solo.py 8 200 > $O/${TAG}_c4_solo.json 2> $O/${TAG}_c4_solo.err \
        || fail c4solo $? $O/${TAG}_c4_solo.err
      python3 -c "import json;d=json.load(open('$O/${TAG}_c4_solo.json'));print('solo max tile %.1f us, untiled %.1f us' % (d['max_tile_us_per_step'], d['untiled_us_per_step'])); [print(r) for r in d['per_tile']]" ;;
    gloo:*)
      N=${S#gloo:}
      AIGAR_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
        --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 50 --warmup 10 \
        --no-cpu-baseline --no-pixels --batched-arenas 0 > $O/${TAG}_gloo$N.json 2> $O/${TAG}_gloo$N.err \
        || fail "gloo $N" $? $O/${TAG}_gloo$N.err
      tail -c 300 $O/${TAG}_gloo$N.json ;;
    ab:*)
      IFS=: read -r _ B N <<< "$S"; N=${N:-3}
      for i in $(seq $N); do
        for v in A B; do
          so=""; [ $v = B ] && so=$R/$B
          AIGAR_SO=$so timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pixels \
            --batched-arenas 0 --no-c4 $AB_ARGS > $O/${TAG}_ab_${v}$i.json 2>/dev/null || fail "ab $v" $?
          python3 -c "import json;d=json.loads(open('$O/${TAG}_ab_${v}$i.json').read().strip().splitlines()[-1]);b=d['breakdown_ms_per_step'];print('$v', round(d['value']/1e6,2), 'M/s  ms/step %.4f tick %.4f obs %.4f' % (d['ms_per_step'], b['tick'], b['observe']))"
        done
      done ;;
    ppdiag)
      timeout -k 10 300 python -u tools/pp_diag.py > $O/${TAG}_ppdiag.txt 2>&1 || fail ppdiag $? $O/${TAG}_ppdiag.txt
      cat $O/${TAG}_ppdiag.txt ;;
    *) fail "unknown step $S" 2 ;;
  esac
done
echo done
