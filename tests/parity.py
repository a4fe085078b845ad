"""Shared helpers for GPU-vs-oracle parity (test infrastructure)."""
import os

import numpy as np

from aigar_amd import _abi
from oracle_lib import Oracle, golden_state, make_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

# float tolerance: north_star allows 1e-5 on float positions / masses, but the
# device's pow, atan2, sin and cos are glibc's bit for bit (aigar_math.h,
# aigar_glibc_trig.h) and every other operation is a correctly rounded IEEE one
# in the reference's order, so states and observations are compared EXACTLY
# (AIGAR_FTOL overrides, for diagnostics); events / indices / ordering always are.
FTOL = float(os.environ.get("AIGAR_FTOL", "0"))


def philox_dict(z, prefix, seed=7):
    """Golden (reference) snapshot re-keyed for the Philox world stream."""
    d = golden_state(z, prefix)
    d["rng_mode"] = _abi.RNG_PHILOX
    d["philox_key"] = np.array([seed, 0x9E3779B9], np.uint64)
    d["ctr_pellet"] = 0
    d["ctr_virus"] = 0
    return d


def golden_config(z, arenas=1):
    return make_config(n_arenas=arenas, bots=int(z["n_players"]), field_size=int(z["size"]),
                       virus=bool(z["virus_enabled"]), max_pellets=float(z["max_pellets"]),
                       max_viruses=float(z["max_viruses"]), channels=int(z["obs_channels"]),
                       extras=int(z["obs_extras"]), rng_mode=_abi.RNG_PHILOX,
                       grid_squares=int(z["grid_squares"]) if "grid_squares" in z.files else 11)


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def load_snapshot(name):
    """A matured world written by tools/mature.py (data/<name>.npz) as a state dict."""
    z = np.load(os.path.join(ROOT, "data", name + ".npz"))
    return {k: z[k] for k in z.files}


def diff_states(a, b, ftol=FTOL):
    """Return a list of human-readable differences (empty == parity)."""
    out = []
    for k in ("seq_next", "tick", "ctr_pellet", "ctr_virus", "n_cells", "n_pellets", "n_blobs", "n_viruses", "n_dead"):
        if int(a[k]) != int(b[k]):
            out.append("%s: %s != %s" % (k, a[k], b[k]))
    if out:
        return out
    for k in ("players_i", "cells_i", "pellets_seq", "blobs_i", "viruses_i", "dead", "pellets_col", "blobs_col"):
        if k not in a or k not in b:  # (colour owners: optional)
            continue
        if not np.array_equal(a[k], b[k]):
            idx = np.argwhere(np.asarray(a[k]) != np.asarray(b[k]))
            out.append("%s differs at %s: %s vs %s" % (k, idx[:3].tolist(), np.asarray(a[k])[tuple(idx[0])],
                                                       np.asarray(b[k])[tuple(idx[0])]))
    for k in ("players_f", "cells_f", "pellets_f", "blobs_f", "viruses_f"):
        x, y = np.asarray(a[k]), np.asarray(b[k])
        if x.shape != y.shape:
            out.append("%s shape %s vs %s" % (k, x.shape, y.shape))
            continue
        if x.size and not np.allclose(x, y, rtol=0, atol=ftol):
            dd = np.abs(x - y)
            i = np.unravel_index(np.argmax(dd), dd.shape)
            out.append("%s max abs diff %.3g at %s: %r vs %r" % (k, dd[i], i, x[i], y[i]))
    return out


def max_float_diff(a, b):
    m = 0.0
    for k in ("cells_f", "pellets_f", "blobs_f", "viruses_f"):
        x, y = np.asarray(a[k]), np.asarray(b[k])
        if x.shape == y.shape and x.size:
            m = max(m, float(np.max(np.abs(x - y))))
    return m


def obs_close(x, y, tol=FTOL):
    nx, ny = np.isnan(x), np.isnan(y)
    if not np.array_equal(nx, ny):
        return False
    return bool(np.allclose(np.nan_to_num(x), np.nan_to_num(y), rtol=0, atol=tol))


def synthetic_commands(rng, st_players_alive, n, size, p_split=0.0, p_eject=0.0):
    cmd = np.zeros((n, 4))
    cmd[:, 0] = rng.random(n) * size
    cmd[:, 1] = rng.random(n) * size
    cmd[:, 2] = rng.random(n) < p_split
    cmd[:, 3] = rng.random(n) < p_eject
    return cmd


def run_pair(gpu, orc, ticks, cmd_fn, check_every=1, obs=False, ftol=FTOL):
    """Step GPU and oracle side by side; return (first failure message or None, stats)."""
    stats = {"events": 0, "max_float_diff": 0.0, "ticks": 0}
    for t in range(ticks):
        cmd = cmd_fn(t)
        gpu.set_commands(cmd)
        orc.set_commands(cmd)
        gpu.step(1)
        orc.step(1)
        eg, eo = gpu.events(), orc.events()
        if not np.array_equal(eg, eo):
            n = min(len(eg), len(eo))
            bad = next((i for i in range(n) if not np.array_equal(eg[i], eo[i])), n)
            return ("tick %d: event log differs at #%d (gpu %d events, oracle %d): gpu %s oracle %s"
                    % (t, bad, len(eg), len(eo), eg[bad:bad + 3].tolist(), eo[bad:bad + 3].tolist())), stats
        stats["events"] += len(eo)
        if (t + 1) % check_every == 0 or t == ticks - 1:
            sg, so = gpu.get_state(), orc.get_state()
            dif = diff_states(sg, so, ftol)
            if dif:
                return "tick %d: state differs: %s" % (t, "; ".join(dif[:4])), stats
            stats["max_float_diff"] = max(stats["max_float_diff"], max_float_diff(sg, so))
        if obs:
            og, oo = gpu.observe(), orc.observe()
            # every bot is compared: the device pow is glibc's, bit for bit (aigar_math.h), so
            # the fov sizes (and with them the cols == 12 quirk) must be identical
            fg, fo = gpu.player_stats()[:, 4], orc.player_stats()[:, 4]
            if not np.array_equal(fg, fo, equal_nan=True):
                i = int(np.argwhere(~((fg == fo) | (np.isnan(fg) & np.isnan(fo))))[0][0])
                return "tick %d: fov size differs at bot %d: %r vs %r" % (t, i, fg[i], fo[i]), stats
            if not obs_close(og, oo, ftol):
                bad = np.argwhere(~np.isclose(np.nan_to_num(og), np.nan_to_num(oo), rtol=0, atol=ftol))
                r0 = tuple(bad[0])
                return "tick %d: observation differs at bot %d col %d: %r vs %r (%d cells)" % (
                    t, r0[0], r0[1], og[r0], oo[r0], len(bad)), stats
        stats["ticks"] = t + 1
    return None, stats
