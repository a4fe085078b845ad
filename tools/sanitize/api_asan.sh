#!/bin/bash
# Host-side ASan / UBSan build of libaigar_hip plus its C-ABI driver.
#   bash tools/sanitize/api_asan.sh build   # here (hipcc cross-compiles)
#   bash tools/sanitize/api_asan.sh run     # GPU box
set -eo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$R/tools/sanitize/bin
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer"
if [ "$1" = build ]; then
  mkdir -p $OUT
  hipcc -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 $SAN \
    $R/aigar_amd/csrc/tick.hip $R/aigar_amd/csrc/obs.hip $R/aigar_amd/csrc/api.hip -o $OUT/libaigar_hip_asan.so
  hipcc -O1 -g -std=c++17 $SAN $R/tools/sanitize/api_asan.cpp -L$OUT -laigar_hip_asan -Wl,-rpath,$OUT -o $OUT/api_asan
  echo built
else
  mkdir -p $R/gpurun_out
  ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 UBSAN_OPTIONS=print_stacktrace=1 \
    timeout -k 10 300 $OUT/api_asan > $R/gpurun_out/api_asan.log 2>&1
  tail -5 $R/gpurun_out/api_asan.log
fi
