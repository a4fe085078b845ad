"""GPU parity of the pixel observation (RGBGenerator.get_cnn_inputRGB,
rgbGenerator.py:95-110) against the CPU oracle's restatement (oracle.c
pixels_one).  Byte work: the RGB frames must be bit-exact.  pygame is absent
here, so parity with pygame itself is unpinned (the oracle follows the
published SDL_gfx algorithms); this test pins the HIP kernel to the oracle.
"""
import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu

_lib = pytest.importorskip("aigar_amd._lib")

CH = _abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY


def pair(cfg, seed):
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(seed)
    o.reset(seed)
    return g, o


def step_both(g, o, ticks, seed, bots, ps=0.0, pe=0.0):
    rng = np.random.default_rng(seed)
    size = g.get_state()["field_size"]
    err, _ = parity.run_pair(g, o, ticks, lambda t: parity.synthetic_commands(rng, None, bots, size, ps, pe))
    assert err is None, err


def assert_frames_equal(fg, fo):
    bad = np.argwhere(np.any(fg != fo, axis=-1))
    assert bad.size == 0, "%d pixels differ, first (player, x, y) %s: gpu %s oracle %s" % (
        len(bad), tuple(bad[0]), fg[tuple(bad[0])], fo[tuple(bad[0])])


@pytest.mark.parametrize("bots,ticks,seed,side,kw", [
    (1, 0, 1, 42, dict(max_pellets=100, field_size=1000)),
    (1, 200, 1, 84, dict(max_pellets=100, field_size=1000)),
    (32, 60, 2, 42, dict(p_split=0.05, p_eject=0.05)),
    (32, 60, 2, 41, dict(p_split=0.05, p_eject=0.05)),                    # odd side: byte-store path
    (32, 60, 3, 84, dict(virus=True, max_viruses=40, p_split=0.05, p_eject=0.05)),
    (48, 120, 4, 42, dict(field_size=120, p_split=0.05, p_eject=0.05)),   # crowded: big cells, deaths
    (256, 20, 5, 42, dict(max_pellets=10000, field_size=1200)),           # C2
    (8, 30, 6, 42, dict(field_size=100, max_pellets=1500)),                # >255 small objects per frame
    (8, 30, 7, 84, dict(field_size=100, max_pellets=1500, p_split=0.1)),
])
def test_pixels_match_oracle(bots, ticks, seed, side, kw):
    kw = dict(kw)
    ps, pe = kw.pop("p_split", 0.0), kw.pop("p_eject", 0.0)
    virus = kw.pop("virus", False)
    cfg = make_config(bots=bots, virus=virus, channels=CH, extras=0, **kw)
    g, o = pair(cfg, seed)
    if ticks:
        step_both(g, o, ticks, seed, bots, ps, pe)
    for cseed in (0, 12345):
        fg, fo = g.observe_pixels(side, cseed), o.pixels(side, cseed)
        assert fg.shape == fo.shape == (bots, side, side, 3)
        assert_frames_equal(fg, fo)
    if ticks == 0:  # cells enter the player hash only at the first tick (field.py:121-132)
        return
    # the frames are not trivially white: the own cell is drawn
    alive = g.player_stats()[:, 0] > 0
    assert np.all(np.any(fg[alive] != 255, axis=(1, 2, 3)))


def test_pixels_gray_is_weighted_average():
    cfg = make_config(bots=16, virus=True, max_viruses=10, channels=CH, extras=0)
    g, o = pair(cfg, 9)
    step_both(g, o, 30, 9, 16, 0.05, 0.0)
    rgb = g.observe_pixels(42, 3)
    gray = g.observe_pixels(42, 3, rgb=False)
    gray32 = g.observe_pixels(42, 3, out=np.zeros((16, 42, 42), np.float32))
    alive = g.player_stats()[:, 0] > 0
    ref = np.average(rgb.astype(np.float64), axis=-1, weights=[0.298, 0.587, 0.114])
    assert np.array_equal(gray[alive], ref[alive])
    assert np.array_equal(gray32[alive], ref[alive].astype(np.float32))
    assert np.all(np.isnan(gray[~alive]))


def test_pixels_on_device_matches_host():
    torch = pytest.importorskip("torch")
    cfg = make_config(bots=64, channels=CH, extras=0)
    g = _lib.Stepper(cfg)
    g.reset(21)
    host = g.observe_pixels(42, 0)
    dev = torch.zeros((64, 42, 42, 3), dtype=torch.uint8, device="cuda")
    g.observe_pixels(42, 0, out=dev)
    g.sync()
    assert np.array_equal(dev.cpu().numpy(), host)


def test_pixels_rejects_bad_side():
    g = _lib.Stepper(make_config(bots=2, channels=CH, extras=0))
    g.reset(0)
    with pytest.raises(RuntimeError):
        g.observe_pixels(85, 0)


def test_rgb_generator_facade():
    """aigar_amd.model.RGBGenerator (rgbGenerator.py:10-110) over a Model: frames equal the oracle's."""
    from aigar_amd import model as M
    from test_facade import reference_like_parameters
    params = reference_like_parameters(virus=True, split=True, eject=False, n_bots=6)
    params.CNN_P_RGB, params.CNN_USE_L1, params.CNN_INPUT_DIM_1 = True, True, 42
    mdl = M.Model(False, False, params, seed=11, field_size=200, max_viruses=4)
    for _ in range(6):
        mdl.createBot("Random")
    mdl.initialize()
    field = mdl.getField()
    orc = Oracle(field._config())
    orc.reset(11)
    gen = M.RGBGenerator(field, params)
    for _ in range(20):
        mdl.takeBotActions()
        cmd = field._cmd.copy()
        field.update()
        orc.set_commands(cmd)
        orc.step(1)
    want = orc.pixels(42, 11)
    for p in mdl.getPlayers():
        if p.getIsAlive():
            assert np.array_equal(gen.get_cnn_inputRGB(p), want[p.index])
    params.CNN_P_RGB = False
    gray = M.RGBGenerator(field, params).get_cnn_inputRGB(mdl.getPlayers()[0])
    assert gray.shape == (42, 42, 1)
    orc.close()


def test_blob_colours_follow_the_ejecting_player():
    """Ejected blobs carry their player's colour (field.py:141, cell.py:219) and
    keep it as the pellets they become (addPellet(blob), field.py:110): the
    colour owners in the state equal the oracle's and the ejecting player's
    index, and the frames that show them equal the oracle's."""
    cfg = make_config(bots=4, virus=False, channels=CH, extras=0, field_size=300, max_pellets=50)
    g, o = pair(cfg, 3)
    st = g.get_state()
    cf = np.array(st["cells_f"])
    ci = np.array(st["cells_i"])
    k = int(np.argmax(ci[:, 0] == 1))  # player 1's first cell: heavy enough to eject for a while
    cf[k, 2] = 400.0
    cf[k, 3] = np.sqrt(400.0 / np.pi)
    st["cells_f"] = cf
    g.load_state(st)
    o.load_state(st)
    n = cfg.bots_per_arena
    ejected = pelleted = False
    for t in range(40):
        cmd = np.zeros((n, 4))
        cmd[:, 0] = cmd[:, 1] = 150.0
        cmd[1, 0], cmd[1, 3] = 10.0, 1.0 if t < 8 else 0.0  # player 1 ejects towards the left wall
        g.set_commands(cmd)
        o.set_commands(cmd)
        g.step(1)
        o.step(1)
        sg, so = g.get_state(), o.get_state()
        dif = parity.diff_states(sg, so)
        assert not dif, (t, dif)
        if len(sg["blobs_col"]):
            assert set(np.asarray(sg["blobs_col"]).tolist()) <= {1}, sg["blobs_col"]
            ejected = True
        if 1 in set(np.asarray(sg["pellets_col"]).tolist()):
            pelleted = True
        if ejected and t % 5 == 0:
            for cseed in (0, 7):
                assert_frames_equal(g.observe_pixels(42, cseed), o.pixels(42, cseed))
    assert ejected and pelleted
    assert set(np.asarray(sg["pellets_col"]).tolist()) <= {-1, 1}
    for cseed in (0, 7):
        assert_frames_equal(g.observe_pixels(42, cseed), o.pixels(42, cseed))
    g.close()
    o.close()
