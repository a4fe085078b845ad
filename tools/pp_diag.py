"""Why the parallel playerPlayerOverlap pass fell back to the serial one (diagnostics
build, -DAIGAR_PP_DIAG): per world, 60 greedy ticks; counts of ticks with too few /
too many pending players, closures over the player / cell caps or not settling,
conflicting closures, parallel ticks, and the closure sizes (players 0..7+).
Counters accumulate over the process (the second world's line includes the first's)."""
import os, sys, ctypes as C
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
# build: bash tools/build_variant.sh tools/var/lib_ppdiag.so -DAIGAR_PP_DIAG
os.environ["AIGAR_SO"] = os.path.join(ROOT, "tools", "var", "lib_ppdiag.so")
import torch
from aigar_amd import _lib
from oracle_lib import make_config
import parity
from test_gpu_full_size import c3
import bench
for world in ("c3_t600", "c3_t50"):
    g = _lib.Stepper(c3())
    if world == "c3_t50":
        z = np.load(os.path.join(ROOT, "data", "c3_t50.npz")); g.load_state({k: z[k] for k in z.files})
    else:
        g.load_state(parity.load_snapshot(world))
    L = _lib.load()
    for t in range(60):
        g.policy_greedy(True)
        g.step(1)
    g.sync()
    out = (C.c_ulonglong * 16)()
    L.aigar_debug_ppdiag(out)
    v = list(out)
    print(world, "nw<min %d nw>max %d ovf_pl %d ovf_cells %d noconv %d bad %d par %d | closure npl hist %s" % (
        v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[8:16]), g.counters())
    g.close()
