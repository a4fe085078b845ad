"""The C-ABI library loads and exports every entry point include/aigar.h declares
(CPU-only: no compute call needs a GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from aigar_amd import _abi, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "aigar.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(aigar_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for need in ("aigar_create", "aigar_reset", "aigar_set_commands", "aigar_step", "aigar_observe",
                 "aigar_get_state", "aigar_load_state", "aigar_get_events", "aigar_sync", "aigar_last_error"):
        assert need in names


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    syms = subprocess.check_output(["nm", "-D", "--defined-only", _lib.SO_PATH]).decode()
    exported = set(re.findall(r" T (aigar_\w+)", syms))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    assert L.aigar_abi_version() == _abi.ABI_VERSION


def test_struct_layouts_match_header():
    # sizes of the ctypes mirrors vs a C compile of the header
    src = '#include "%s"\n#include <stdio.h>\n#include <stddef.h>\nint main(){printf("%%zu %%zu %%zu %%zu %%zu\\n", ' \
          'sizeof(aigar_config), sizeof(aigar_state), offsetof(aigar_state, players_f), ' \
          'sizeof(aigar_reward_params), sizeof(aigar_run_params));return 0;}' % HEADER
    exe = "/tmp/aigar_hdr_check"
    subprocess.run(["gcc", "-x", "c", "-", "-o", exe], input=src.encode(), check=True)
    cfg, st, off, rp, run = map(int, subprocess.check_output([exe]).split())
    assert rp == C.sizeof(_abi.RewardParams)
    assert run == C.sizeof(_abi.RunParams)
    assert cfg == C.sizeof(_abi.Config)
    assert st == C.sizeof(_abi.State)
    assert off == _abi.State.players_f.offset


def test_create_fails_loudly_without_device_or_with_bad_config():
    L = _lib.load()
    cfg = _abi.Config()
    cfg.n_arenas, cfg.bots_per_arena, cfg.rng_mode = 1, 4, _abi.RNG_MT19937
    h = C.c_void_p()
    assert L.aigar_create(C.byref(cfg), C.byref(h)) < 0
    assert b"PHILOX" in L.aigar_last_error()
    cfg.rng_mode, cfg.grid_squares = _abi.RNG_PHILOX, 128  # (42 / 84: the CNN grid view; at most 127)
    assert L.aigar_create(C.byref(cfg), C.byref(h)) < 0
    assert b"grid_squares" in L.aigar_last_error()


def test_obs_len_formula():
    assert _abi.obs_len(11, _abi.OBS_PELLET, _abi.EX_FOV | _abi.EX_MASS) == 123  # networkParameters default
    ch = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
          | _abi.OBS_ENEMY_LF)
    ex = _abi.EX_LAST_FOV | _abi.EX_FOV | _abi.EX_MASS | _abi.EX_LAST_ACT
    assert _abi.obs_len(11, ch, ex) == 854  # C3 (virus + split), SURVEY.md §8a25
    assert _abi.obs_len(84, ch, 0) == 7 * 84 * 84  # CNN grid view (bot.py:284): the grids alone
    assert _abi.obs_len(11, _abi.OBS_SIMPLE, ex) == 12  # getSimpleStateRepresentation (bot.py:511-547)
