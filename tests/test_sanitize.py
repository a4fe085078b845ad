"""CPU sanitizer run of the oracle: oracle.c built with
AddressSanitizer + UndefinedBehaviorSanitizer (no recovery) and driven through
every entry point the parity tests use by tools/sanitize/oracle_asan.c.  The
host half of the HIP library gets the same treatment on the GPU box
(tools/sanitize/api_asan.sh; its last log: profiles/r02_api_asan.log)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_oracle_is_clean_under_asan_and_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_asan")
    subprocess.check_call(["gcc", "-O1", "-g", "-std=gnu11", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-ffp-contract=off",
                           "-fno-builtin-sin", "-fno-builtin-cos", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "oracle", "oracle.c"),
                           os.path.join(ROOT, "tools", "sanitize", "oracle_asan.c"), "-o", exe, "-lm"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "clean" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
