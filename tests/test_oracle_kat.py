"""Known-answer tests for the numeric primitives the oracle restates."""
import ctypes as C
import os

import numpy as np

from oracle_lib import lib


def _u32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def test_mt19937_randint_and_random_match_numpy(golden_dir):
    z = np.load(os.path.join(golden_dir, "kat_rng.npz"))
    L = lib()
    key = z["mt_key"].astype(np.uint32).copy()
    pos = C.c_int(int(z["mt_pos"]))
    got = [L.oracle_mt_randint(_u32p(key), C.byref(pos), lo, hi) for lo, hi in zip(z["lo"], z["hi"])]
    assert np.array_equal(np.array(got), z["val"])
    r = [L.oracle_mt_random(_u32p(key), C.byref(pos)) for _ in range(len(z["random"]))]
    assert np.array_equal(np.array(r), z["random"])
    assert np.array_equal(key, z["end_key"]) and pos.value == int(z["end_pos"])


def test_mt19937_seed_matches_numpy():
    L = lib()
    for s in (0, 1, 12345, 2**32 - 1):
        key = np.zeros(624, np.uint32)
        pos = C.c_int(0)
        L.oracle_mt_seed(s, _u32p(key), C.byref(pos))
        st = np.random.RandomState(s).get_state(legacy=True)
        assert np.array_equal(key, st[1]) and pos.value == st[2]


def test_pairwise_sum_round3_deg2rad(golden_dir):
    z = np.load(os.path.join(golden_dir, "kat_numeric.npz"))
    L = lib()
    a, off = z["sum_in"], z["sum_off"]
    for i in range(len(off) - 1):
        seg = np.ascontiguousarray(a[off[i]:off[i + 1]])
        assert L.oracle_np_sum(seg.ctypes.data_as(C.POINTER(C.c_double)), len(seg)) == z["sum_out"][i]
    got = np.array([L.oracle_py_round3(float(v)) for v in z["round_in"]])
    assert np.array_equal(got, z["round_out"]) and np.array_equal(np.signbit(got), np.signbit(z["round_out"]))
    assert np.array_equal(np.arange(360) * (np.pi / 180.0), z["deg2rad"])


def test_philox4x64_matches_numpy():
    L = lib()
    rng = np.random.default_rng(3)
    for _ in range(50):
        key = rng.integers(0, 2**64, size=2, dtype=np.uint64)
        ctr = rng.integers(0, 2**63, size=4, dtype=np.uint64)
        raw = np.random.Philox(key=key, counter=ctr).random_raw(4)
        c2 = ctr.copy()
        c2[0] += np.uint64(1)
        out = np.zeros(4, np.uint64)
        p = lambda x: x.ctypes.data_as(C.POINTER(C.c_uint64))  # noqa: E731
        L.oracle_philox(p(c2), p(key), p(out))
        assert np.array_equal(raw, out)
