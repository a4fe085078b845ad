"""GPU: the reference-shaped facade (aigar_amd/model.py) driven like the
reference's Model, checked against the oracle stepping the same commands."""
import math

import numpy as np
import pytest

from aigar_amd import model as M
from oracle_lib import Oracle
import parity
from test_facade import ids_for_area, reference_like_parameters

pytestmark = pytest.mark.gpu


def brute_in_fov(objs_f, size, fov_pos, fov_size, member=None):
    """getNearbyObjectsInArea + isInFov restated with Python loops over a state array."""
    q = ids_for_area(fov_pos, fov_size / 2, size)
    h = fov_size / 2
    out = []
    for k, f in enumerate(objs_f):
        if member is not None and not member[k]:
            continue
        x, y, r = f[0], f[1], f[3]
        if not (ids_for_area((x, y), r, size) & q):
            continue
        if x + r < fov_pos[0] - h or x - r > fov_pos[0] + h or y + r < fov_pos[1] - h or y - r > fov_pos[1] + h:
            continue
        out.append(k)
    return out


def test_model_update_matches_oracle_and_getters():
    np.random.seed(4)
    params = reference_like_parameters(virus=True, split=True, eject=True, n_bots=12)
    params.FRAME_SKIP_RATE = 3
    model = M.Model(False, False, params, seed=11, field_size=260, max_viruses=8)
    for _ in range(10):
        model.createBot("Random")
    nn = [model.createBot("NN"), model.createBot("NN")]
    model.initialize()
    field = model.getField()
    orc = Oracle(field._config())
    orc.reset(11)
    dif = parity.diff_states(field.stepper.get_state(), orc.get_state())
    assert not dif, dif
    for t in range(60):
        for b in nn:  # an external learner's actions
            b.currentAction = list(np.random.random(4))
        model.takeBotActions()
        cmd = field._cmd.copy()
        field.update()
        orc.set_commands(cmd)
        orc.step(1)
        st, so = field._snapshot(), orc.get_state()
        dif = parity.diff_states(st, so)
        assert not dif, "tick %d: %s" % (t, dif)
        stats = orc.player_stats()
        size = field.getWidth()
        for p in model.getPlayers():
            s = stats[p.index]
            assert p.getIsAlive() == bool(s[0] > 0)
            if not p.getIsAlive():
                assert p.getCells() == []
                continue
            assert abs(p.getTotalMass() - s[1]) <= 1e-9
            assert abs(p.getFovSize() - s[4]) <= 1e-9 * s[4]
            own = [c for c in p.getCells()]
            assert len(own) == int(st["players_i"][p.index][4])
            fp, fs = p.getFovPos(), p.getFovSize()
            want = brute_in_fov(so["pellets_f"], size, fp, fs)
            got = [c.getId() for c in field.getPelletsInFov(fp, fs)]
            assert got == [int(so["pellets_seq"][k]) for k in want]
            vm = np.asarray(so["viruses_i"])[:, 2] != 0 if len(so["viruses_i"]) else None
            want_v = brute_in_fov(so["viruses_f"], size, fp, fs, vm)
            assert [c.getId() for c in field.getVirusesInFov(fp, fs)] == \
                sorted(int(so["viruses_i"][k][1]) for k in want_v)
            enemies = field.getEnemyPlayerCellsInFov(p)
            assert all(c.getPlayer() is not p for c in enemies)
            assert [c.getId() for c in enemies] == sorted(c.getId() for c in enemies)
        # NN bots: the reference's [1, L] state row for live players, None for dead ones
        obs_o = orc.observe()
        for b in nn:
            r = b.getStateRepresentation()
            if not b.getPlayer().getIsAlive():
                assert r is None
                continue
            assert r.shape == (1, params.STATE_REPR_LEN)
            og = field._state_row(b.player.index)
            assert np.array_equal(r[0], og)
            assert field._player_stats()[b.player.index][4] == stats[b.player.index][4]  # (glibc pow on the device)
            assert parity.obs_close(og, obs_o[b.player.index])
    orc.close()
    model.resetModel()
    assert model.counter == 0 and field.getWidth() == 260


def test_greedy_model_matches_oracle_greedy():
    """Model with Greedy bots: the facade's batched device moves equal the oracle's greedy policy."""
    params = reference_like_parameters(virus=True, split=True, eject=False, n_bots=24)
    params.ENABLE_GREEDY_SPLIT = True
    model = M.Model(False, False, params, seed=5, field_size=400, max_viruses=10)
    for _ in range(24):
        model.createBot("Greedy")
    model.initialize()
    field = model.getField()
    orc = Oracle(field._config())
    orc.reset(5)
    for t in range(50):
        model.takeBotActions()
        orc.policy_greedy(True)
        cmd = field._cmd.copy()
        assert np.array_equal(cmd, orc.commands()), "tick %d" % t
        for b in model.getBots():  # the reference objects see the same commands
            assert b.getPlayer().getCommandPoint() == [cmd[b.player.index, 0], cmd[b.player.index, 1]]
        field.update()
        orc.step(1)
        assert not parity.diff_states(field._snapshot(), orc.get_state())
    orc.close()
