#!/bin/bash
# Build the HIP library from the working tree into another file (A/B runs):
# bash tools/build_variant.sh OUT.so [extra hipcc flags...]
set -e
OUT=$1; shift
cd "$(dirname "$0")/../aigar_amd/csrc"
python3 - "$OUT" "$@" <<'PY'
import os, subprocess, sys
sys.path.insert(0, os.path.abspath("../.."))
from aigar_amd import _build
out = os.path.abspath(os.path.join("../..", sys.argv[1])) if not os.path.isabs(sys.argv[1]) else sys.argv[1]
subprocess.check_call(["hipcc"] + _build.FLAGS + sys.argv[2:] + _build.SOURCES + ["-o", out])
print(out)
PY
