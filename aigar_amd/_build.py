"""Build libaigar_hip.so (gfx950) in-tree with hipcc."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SO = os.path.join(HERE, "libaigar_hip.so")
SOURCES = ["tick.hip", "obs.hip", "api.hip"]
HEADERS = ["aigar_sem.h", "aigar_dev.h", "aigar_math.h", "aigar_trig.h", "aigar_wave.h", "aigar_glibc_pow_tables.h",
           "aigar_trig_tables.h", "aigar_glibc_trig.h", "aigar_glibc_trig_tables.h", "pixels.inc", "obs_wide.inc", os.path.join("..", "..", "include", "aigar.h")]
ARCH = os.environ.get("AIGAR_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: no FMA contraction, every fp64 operation rounds like the
# reference's Python floats.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "--offload-arch=" + ARCH,
         "-Wall", "-Wno-unused-result", "-Wno-unused-variable", "-Wno-unused-function"]


def stale():
    if not os.path.exists(SO):
        return True
    t = os.path.getmtime(SO)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(p) > t for p in deps)


def build(force=False, verbose=False):
    if not force and not stale():
        return SO
    cmd = ["hipcc"] + FLAGS + [os.path.join(CSRC, s) for s in SOURCES] + ["-o", SO + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(SO + ".tmp", SO)
    return SO


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
