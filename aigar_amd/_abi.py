"""ctypes mirror of include/aigar.h (the C-ABI of libaigar_hip.so).

Only plain structs and numpy conversion helpers live here; loading the HIP
library is in `_lib.py`.
"""
import ctypes as C

import numpy as np

ABI_VERSION = 5

RNG_PHILOX = 0
RNG_MT19937 = 1

OBS_PELLET, OBS_SELF, OBS_WALL, OBS_ENEMY, OBS_ALL, OBS_VIRUS = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
OBS_SELF_SLF, OBS_SELF_LF, OBS_ENEMY_SLF, OBS_ENEMY_LF = 0x40, 0x80, 0x100, 0x200
OBS_SIMPLE = 0x400  # GRID_VIEW_ENABLED = False: getSimpleStateRepresentation, 12 values
EX_LAST_FOV, EX_FOV, EX_MASS, EX_LAST_ACT, EX_2LAST_ACT = 0x1, 0x2, 0x4, 0x8, 0x10

EV_MERGE, EV_VIRUS_EAT_BLOB, EV_VIRUS_SPLIT, EV_CELL_EAT_VIRUS, EV_EXPLODE = 1, 2, 3, 4, 5
EV_CELL_EAT_PELLET, EV_CELL_EAT_BLOB, EV_CELL_EAT_CELL, EV_PLAYER_DEATH, EV_RESPAWN = 6, 7, 8, 9, 10

FLAG_EVENTS = 0x1
TILE_OWNED_ONLY = 0x1
TILE_FORCE = 0x2  # a 1 x 1 tiled handle (the whole field one tile: the one-GPU test of the exchange path)


POLICY_NONE, POLICY_RANDOM, POLICY_GREEDY = 0, 1, 2
ROLE_NN, ROLE_GREEDY, ROLE_RANDOM = 0, 1, 2
ROLES = {"NN": ROLE_NN, "Greedy": ROLE_GREEDY, "Random": ROLE_RANDOM}


class EnvParams(C.Structure):
    """aigar_env_params (include/aigar.h): the device Greedy / Random bots of a mixed population."""
    _fields_ = [("greedy_split", C.c_int32), ("random_skip", C.c_int32), ("random_split", C.c_int32),
                ("random_eject", C.c_int32), ("salt", C.c_uint64)]


class RunParams(C.Structure):
    """aigar_run_params (include/aigar.h): the policy replayed inside aigar_run's step graph."""
    _fields_ = [("policy", C.c_int32), ("greedy_split", C.c_int32), ("p_split", C.c_double),
                ("p_eject", C.c_double), ("seed", C.c_uint64)]


class RewardParams(C.Structure):
    """aigar_reward_params (include/aigar.h); defaults of networkParameters.py:50,69-72."""
    _fields_ = [("mass_as_reward", C.c_int32), ("pad", C.c_int32), ("reward_term", C.c_double),
                ("death_term", C.c_double), ("death_factor", C.c_double), ("reward_scale", C.c_double)]

    @classmethod
    def from_parameters(cls, p=None):
        g = (lambda n, dflt: getattr(p, n, dflt)) if p is not None else (lambda n, dflt: dflt)
        return cls(int(bool(g("MASS_AS_REWARD", False))), 0, float(g("REWARD_TERM", 0)), float(g("DEATH_TERM", -40)),
                   float(g("DEATH_FACTOR", 1.5)), float(g("REWARD_SCALE", 2)))


class Config(C.Structure):
    _fields_ = [
        ("n_arenas", C.c_int32), ("bots_per_arena", C.c_int32), ("field_size", C.c_int32),
        ("virus_enabled", C.c_int32), ("max_pellets", C.c_double), ("max_viruses", C.c_double),
        ("grid_squares", C.c_int32), ("obs_channels", C.c_uint32), ("obs_extras", C.c_uint32),
        ("rng_mode", C.c_int32), ("device", C.c_int32), ("pellet_cap", C.c_int32),
        ("blob_cap", C.c_int32), ("virus_cap", C.c_int32), ("event_cap", C.c_int32), ("flags", C.c_int32),
        ("tile_x", C.c_int32), ("tile_y", C.c_int32), ("tile_id", C.c_int32), ("tile_halo", C.c_int32),
        ("tile_cap", C.c_int32), ("tile_flags", C.c_int32),
    ]


_PD = C.POINTER(C.c_double)
_PI = C.POINTER(C.c_int64)


class State(C.Structure):
    _fields_ = [
        ("n_players", C.c_int32), ("field_size", C.c_int32), ("virus_enabled", C.c_int32), ("rng_mode", C.c_int32),
        ("seq_next", C.c_int64), ("tick", C.c_int64),
        ("max_pellets", C.c_double), ("max_viruses", C.c_double),
        ("philox_key", C.c_uint64 * 2), ("ctr_pellet", C.c_uint64), ("ctr_virus", C.c_uint64),
        ("mt_key", C.c_uint32 * 624), ("mt_pos", C.c_int32),
        ("n_cells", C.c_int32), ("n_pellets", C.c_int32), ("n_blobs", C.c_int32), ("n_viruses", C.c_int32),
        ("n_dead", C.c_int32),
        ("players_f", _PD), ("players_i", _PI), ("cells_f", _PD), ("cells_i", _PI),
        ("pellets_f", _PD), ("pellets_seq", _PI), ("blobs_f", _PD), ("blobs_i", _PI),
        ("viruses_f", _PD), ("viruses_i", _PI), ("dead", _PI),
        ("pellets_col", _PI), ("blobs_col", _PI),
    ]


# snapshot record layouts: name -> (count field, columns, dtype)
LAYOUT = {
    "players_f": ("n_players", 2, np.float64), "players_i": ("n_players", 5, np.int64),
    "cells_f": ("n_cells", 9, np.float64), "cells_i": ("n_cells", 4, np.int64),
    "pellets_f": ("n_pellets", 4, np.float64), "pellets_seq": ("n_pellets", 0, np.int64),
    "blobs_f": ("n_blobs", 8, np.float64), "blobs_i": ("n_blobs", 3, np.int64),
    "viruses_f": ("n_viruses", 8, np.float64), "viruses_i": ("n_viruses", 3, np.int64),
    "dead": ("n_dead", 0, np.int64),
    # optional: colour owners (player index, -1: own colour); absent from older snapshots
    "pellets_col": ("n_pellets", 0, np.int64), "blobs_col": ("n_blobs", 0, np.int64),
}
OPTIONAL = ("pellets_col", "blobs_col")
SCALARS = ("n_players", "field_size", "virus_enabled", "rng_mode", "seq_next", "tick",
           "max_pellets", "max_viruses", "ctr_pellet", "ctr_virus", "mt_pos")


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def state_to_struct(d):
    """numpy snapshot dict -> (State, keepalive list)."""
    st = State()
    keep = []
    for name, (cnt, cols, dt) in LAYOUT.items():
        if name in OPTIONAL and name not in d:
            continue  # (NULL: the library takes -1)
        a = np.ascontiguousarray(d[name], dtype=dt)
        n = a.shape[0] if a.ndim else 0
        if cols:
            a = a.reshape(n, cols)
        keep.append(a)
        if cnt != "n_players":
            setattr(st, cnt, n)
        setattr(st, name, _ptr(a, C.c_double if dt == np.float64 else C.c_int64))
    for k in SCALARS:
        if k in d:
            setattr(st, k, float(d[k]) if k.startswith("max_") else int(d[k]))
    st.n_players = int(d["players_f"].shape[0])
    if "philox_key" in d:
        st.philox_key[0], st.philox_key[1] = int(d["philox_key"][0]), int(d["philox_key"][1])
    if "mt_key" in d:
        C.memmove(st.mt_key, np.ascontiguousarray(d["mt_key"], np.uint32).ctypes.data, 624 * 4)
    return st, keep


def alloc_state(counts):
    """Allocate arrays for a State whose counts were filled by a NULL-array query."""
    st = State()
    C.memmove(C.byref(st), C.byref(counts), C.sizeof(State))
    arrays = {}
    for name, (cnt, cols, dt) in LAYOUT.items():
        n = getattr(st, cnt)
        a = np.zeros((n, cols) if cols else (n,), dtype=dt)
        arrays[name] = a
        setattr(st, name, _ptr(a, C.c_double if dt == np.float64 else C.c_int64))
    return st, arrays


def struct_to_dict(st, arrays):
    d = dict(arrays)
    for k in SCALARS + ("n_cells", "n_pellets", "n_blobs", "n_viruses", "n_dead"):
        d[k] = getattr(st, k)
    d["philox_key"] = np.array([st.philox_key[0], st.philox_key[1]], np.uint64)
    d["mt_key"] = np.frombuffer(bytes(st.mt_key), dtype=np.uint32).copy()
    return d


def obs_len(grid_squares, channels, extras):
    if channels & OBS_SIMPLE:
        return 12
    g = grid_squares or 11
    n = bin(channels & 0x3FF).count("1")
    e = (1 if extras & EX_LAST_FOV else 0) + (1 if extras & EX_FOV else 0) + (1 if extras & EX_MASS else 0) \
        + (4 if extras & EX_LAST_ACT else 0) + (4 if extras & EX_2LAST_ACT else 0)
    return g * g * n + e
