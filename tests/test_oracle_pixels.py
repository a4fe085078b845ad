"""CPU checks of the oracle's pixel-observation restatement (oracle.c
pixels_one; RGBGenerator.get_cnn_inputRGB, rgbGenerator.py:95-110).  pygame is
absent, so these are properties of the SDL_gfx algorithms, not pinned vectors."""
import numpy as np

from oracle_lib import Oracle, make_config


def test_lone_player_frame():
    o = Oracle(make_config(bots=1, field_size=1000, max_pellets=0))
    o.reset(3)
    o.step(1)  # player cells enter the player hash (and so the FOV) at the first tick (field.py:121-132)
    for side in (42, 84):
        f = o.pixels(side, 0)[0]
        assert f.shape == (side, side, 3)
        c = side // 2
        # the own cell sits at the FOV centre and is not white; the corners are
        assert np.any(f[c, c] != 255)
        for x, y in ((0, 0), (0, side - 1), (side - 1, 0), (side - 1, side - 1)):
            assert np.all(f[x, y] == 255)
        # a lone circle is mirror-symmetric about its centre row/column (within the 1-pixel
        # centre offset of integer truncation): the drawn mask's extents match
        drawn = np.any(f != 255, axis=-1)
        xs, ys = np.nonzero(drawn)
        assert abs((xs.max() - c) - (c - xs.min())) <= 1 and abs((ys.max() - c) - (c - ys.min())) <= 1


def test_colour_seed_changes_colours_not_shapes():
    o = Oracle(make_config(bots=8, max_pellets=300, field_size=200))
    o.reset(5)
    a, b = o.pixels(42, 0), o.pixels(42, 99)
    assert not np.array_equal(a, b)
    assert np.array_equal(np.all(a == 255, axis=-1), np.all(b == 255, axis=-1))
