"""CPU tests of the Python facade (aigar_amd/model.py): hash footprints,
parameter -> observation mapping, API guards.  No device calls."""
import math
import types

import numpy as np
import pytest

from aigar_amd import _abi
from aigar_amd import model as M


def ids_for_area(pos, radius, size, bucket=20):
    """spatialHashTable.getIdsForArea (spatialHashTable.py:70-83) restated with
    Python loops: the set of (bucket x, bucket y) an object/area touches."""
    cell_left = max(0, pos[0] - radius)
    cell_top = max(0, pos[1] - radius)
    bucket_left = int(cell_left - cell_left % bucket)
    bucket_top = int(cell_top - cell_top % bucket)
    limit_x = int(min(size, pos[0] + radius + 1))
    limit_y = int(min(size, pos[1] + radius + 1))
    return {(x // bucket, y // bucket) for x in range(bucket_left, limit_x, bucket)
            for y in range(bucket_top, limit_y, bucket)}


def test_footprint_matches_reference_hash_ids():
    rng = np.random.default_rng(3)
    size = 333
    pts = [(0.0, 0.0, 1.78), (332.9, 332.9, 5.0), (19.999, 40.0, 0.1), (20.0, 20.0, 0.0), (333.0, 10.0, 3.0),
           (100.0, 100.0, 84.6)]
    pts += [tuple(v) for v in np.c_[rng.uniform(-5, size + 5, 300), rng.uniform(-5, size + 5, 300),
                                    rng.uniform(0, 60, 300)]]
    for x, y, r in pts:
        want = ids_for_area((x, y), r, size)
        x0, x1, y0, y1 = (int(v) for v in M._footprint(np.float64(x), np.float64(y), np.float64(r), size))
        got = {(bx, by) for bx in range(x0, x1 + 1) for by in range(y0, y1 + 1)}
        assert got == want, (x, y, r)


def test_in_area_is_hash_then_box():
    rng = np.random.default_rng(5)
    size = 400
    x, y = rng.uniform(0, size, 500), rng.uniform(0, size, 500)
    r = np.sqrt(rng.choice([1.0, 2.0, 3.0, 14.4, 100.0], 500) / math.pi)
    for fx, fy, fs in [(200.0, 200.0, 52.3), (5.0, 390.0, 80.0), (399.0, 1.0, 35.0)]:
        q = ids_for_area((fx, fy), fs / 2, size)
        want = []
        for i in range(500):
            near = bool(ids_for_area((x[i], y[i]), r[i], size) & q)
            h = fs / 2
            inside = not (x[i] + r[i] < fx - h or x[i] - r[i] > fx + h or y[i] + r[i] < fy - h or y[i] - r[i] > fy + h)
            want.append(near and inside)
        assert np.array_equal(M._in_area(x, y, r, size, (fx, fy), fs), np.array(want))


def reference_like_parameters(virus, split, eject, n_bots):
    """networkParameters.py:74-102 derivation for the given switches."""
    p = types.SimpleNamespace()
    multi = n_bots > 1
    p.VIRUS_SPAWN, p.ENABLE_SPLIT, p.ENABLE_EJECT = virus, split, eject
    p.PELLET_GRID = True
    p.SELF_GRID = split or virus
    p.SELF_GRID_LF = split
    p.SELF_GRID_SLF = False
    p.WALL_GRID = multi
    p.VIRUS_GRID = virus
    p.ENEMY_GRID = multi
    p.ENEMY_GRID_LF = split
    p.ENEMY_GRID_SLF = False
    p.SIZE_GRID = False
    p.ALL_PLAYER_GRID = False
    p.USE_FOVSIZE, p.USE_LAST_FOVSIZE, p.USE_TOTALMASS = True, split, True
    p.USE_LAST_ACTION, p.USE_SECOND_LAST_ACTION = split, False
    p.GRID_SQUARES_PER_FOV = 11
    p.NUM_OF_GRIDS = sum([p.PELLET_GRID, p.SELF_GRID, p.WALL_GRID, p.VIRUS_GRID, p.ENEMY_GRID, p.SIZE_GRID,
                          p.SELF_GRID_LF, p.SELF_GRID_SLF, p.ENEMY_GRID_LF, p.ENEMY_GRID_SLF, p.ALL_PLAYER_GRID])
    p.EXTRA_INPUT = p.USE_FOVSIZE + p.USE_TOTALMASS + p.USE_LAST_ACTION * 4 + p.USE_SECOND_LAST_ACTION * 4 + \
        p.USE_LAST_FOVSIZE
    p.STATE_REPR_LEN = 121 * p.NUM_OF_GRIDS + p.EXTRA_INPUT
    p.FRAME_SKIP_RATE = 7
    p.RESET_LIMIT = 20000
    return p


@pytest.mark.parametrize("virus,split,eject,n", [(False, False, False, 1), (False, False, False, 256),
                                                 (True, True, True, 4096), (True, False, False, 16)])
def test_obs_masks_reproduce_state_repr_len(virus, split, eject, n):
    p = reference_like_parameters(virus, split, eject, n)
    ch, ex, g = M.obs_masks(p)
    L = g * g * bin(ch).count("1") + sum({_abi.EX_LAST_FOV: 1, _abi.EX_FOV: 1, _abi.EX_MASS: 1,
                                          _abi.EX_LAST_ACT: 4, _abi.EX_2LAST_ACT: 4}[b] for b in
                                         (1, 2, 4, 8, 16) if ex & b)
    assert L == p.STATE_REPR_LEN
    assert _abi.obs_len(g, ch, ex) == p.STATE_REPR_LEN


def test_obs_masks_state_variants():
    """GRID_VIEW_ENABLED = False -> getSimpleStateRepresentation (12 values);
    CNN_REPR without CNN_P_REPR -> the grid view alone at CNN_INPUT_DIM_* squares."""
    p = reference_like_parameters(True, True, False, 16)
    p.GRID_VIEW_ENABLED = False
    ch, ex, g = M.obs_masks(p)
    assert ch == _abi.OBS_SIMPLE and _abi.obs_len(g, ch, ex) == 12
    p.GRID_VIEW_ENABLED = True
    p.CNN_REPR, p.CNN_P_REPR = True, False
    p.CNN_USE_L1, p.CNN_USE_L2, p.CNN_INPUT_DIM_1, p.CNN_INPUT_DIM_2 = False, True, 42, 84
    ch, ex, g = M.obs_masks(p)
    assert g == 84 and ex == 0 and _abi.obs_len(g, ch, ex) == p.NUM_OF_GRIDS * 84 * 84


def test_unsupported_paths_fail_loudly():
    p = reference_like_parameters(False, False, False, 2)
    p.SIZE_GRID = True
    with pytest.raises(NotImplementedError):
        M.obs_masks(p)
    f = M.Field(False)
    with pytest.raises(RuntimeError):
        f.initialize()
    pl = M.Player("x")
    f.addPlayer(pl)
    with pytest.raises(NotImplementedError):
        M.Bot(pl, f, "Smart")


def test_cell_view_predicates():
    a = M.Cell("player", [0.0, 0.0, 40.0, math.sqrt(40 / math.pi), 0, 0, 0, 0], 5, 0, None, -1.0)
    b = M.Cell("pellet", [1.0, 1.0, 1.0, math.sqrt(1 / math.pi)], 9, 0)
    assert a.canEat(b) and not b.canEat(a)
    assert a.overlap(b) and b.overlap(a)
    assert a.canSplit() and a.canEject() and a.canMerge() and not a.justEjected()
    assert a.isInFov([10.0, 10.0], 20.0) and not a.isInFov([30.0, 30.0], 10.0)


def test_colours_follow_the_reference_rules():
    # Player.randomizeColor (player.py:38-41): bytes, sum <= 600; deterministic per (seed, player)
    cols = [M.player_color(i, 3) for i in range(500)]
    assert all(all(0 <= v <= 255 for v in c) and sum(c) <= 600 for c in cols)
    assert cols == [M.player_color(i, 3) for i in range(500)]
    assert len(set(cols)) > 450 and M.player_color(0, 3) != M.player_color(0, 4)
    # pellets: three randint(50, 200) values (cell.py:31); viruses green (field.py:274)
    pc = [M.pellet_color(s) for s in range(2000)]
    assert all(all(50 <= v < 200 for v in c) for c in pc)
    assert M.VIRUS_COLOR == (0, 255, 0)
    p = M.Player("p")
    assert p.getColor() == M.player_color(-1, 0) or sum(p.getColor()) <= 600


def test_init_parameters_keeps_the_world_options():
    """Model.initParameters (model.py:79-84) rebuilds the Field; the
    options given to the Model (field size, counts, event recording) must survive."""
    from aigar_amd.model import Model
    m = Model(False, False, None, seed=3, field_size=500, max_pellets=200.0, max_viruses=4.0, record_events=True)
    m.createPlayer("p0")
    m.initParameters(types.SimpleNamespace(VIRUS_SPAWN=True, RESET_LIMIT=77))
    f = m.field
    assert (f.field_size, f.max_pellets, f.max_viruses, f.record_events, f.seed) == (500, 200.0, 4.0, True, 3)
    assert f.virusEnabled and m.resetLimit == 77 and len(f.players) == 1
