"""GPU: the facade's NN bots drive the device unchanged (SURVEY.md §8f rank 2,
bot.py:166-233): a learner object with the reference's `decideMove(state)`
interface plays NN bots among Greedy and Random bots through `Model.update()`.

Checked against the oracle driven by the same commands: every tick's events
and the world; every NN state the learner saw equals the oracle's observation
of that bot computed at the same ticks (the device observes only the bots that
are not skipping a frame, so the last-frame history advances exactly as the
reference's per-bot getGridStateRepresentation calls make it); every reward
the bots accumulated equals bot.py:654-667 evaluated on the oracle's players;
the Greedy bots' commands equal the oracle's Greedy bots'."""
import types

import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle
import parity

pytestmark = pytest.mark.gpu
model = pytest.importorskip("aigar_amd.model")


class StubLearner:
    """decideMove(state) -> (extra, action): a fixed function of the state (the
    reference's learners, actorCritic.py:938 / qLearning.py:217, have this shape)."""
    discrete = False

    def __str__(self):
        return "Stub"

    def reset(self):
        pass

    def decideMove(self, state):
        v = float(np.nansum(state))
        frac = lambda k: (v * k) % 1.0  # noqa: E731
        return None, [frac(0.37), frac(0.71), frac(0.13), frac(0.97)]


def params():
    return types.SimpleNamespace(
        VIRUS_SPAWN=True, ENABLE_SPLIT=True, ENABLE_EJECT=True, ENABLE_GREEDY_SPLIT=True, GRID_VIEW_ENABLED=True,
        CNN_REPR=False, PELLET_GRID=True, SELF_GRID=True, WALL_GRID=True, ENEMY_GRID=True, VIRUS_GRID=True,
        SELF_GRID_LF=True, ENEMY_GRID_LF=True, EXTRA_INPUT=True, USE_FOVSIZE=True, USE_TOTALMASS=True,
        USE_LAST_ACTION=True, USE_SECOND_LAST_ACTION=True, USE_LAST_FOVSIZE=True, GRID_SQUARES_PER_FOV=11,
        FRAME_SKIP_RATE=3, GATHER_EXP=True, MASS_AS_REWARD=False, REWARD_TERM=0.0, DEATH_TERM=-40.0,
        DEATH_FACTOR=1.5, REWARD_SCALE=2.0, ALGORITHM="CACLA", RESET_LIMIT=20000)


def test_nn_bots_through_model_update_match_oracle():
    p = params()
    np.random.seed(4)  # Random bots draw from numpy, as the reference's
    m = model.Model(False, False, p, seed=4, field_size=300, max_viruses=10, record_events=True)
    kinds = ["NN"] * 6 + ["Greedy"] * 5 + ["Random"] * 5
    bots = [m.createBot(k, StubLearner() if k == "NN" else None) for k in kinds]
    m.initialize()
    n = len(bots)
    o = Oracle(m.field.stepper.cfg)
    o.load_state(m.field.stepper.get_state())
    nn = [b for b in bots if b.type == "NN"]
    seen = {b.player.index: [] for b in nn}

    def actions():  # Model.update -> Field._set_actions: the NN bots' current / last actions
        cur, prev = np.zeros((n, 4)), np.zeros((n, 4))
        for b in nn:
            for arr, act in ((cur, b.currentAction), (prev, b.lastAction)):
                if act is not None:
                    arr[b.player.index, :len(act)] = list(act)[:4]
        return cur, prev

    for t in range(80):
        before = {b.player.index: b.oldState for b in nn}
        stats0 = o.player_stats()
        cur, prev = actions()
        m.field.stepper.set_actions(cur, prev)
        o.set_actions(cur, prev)
        for b in nn:  # bot.py:654-667 on the oracle's players == the bot's own getReward
            i = b.player.index
            if b.lastMass is not None:
                alive = stats0[i, 0] > 0
                want = ((stats0[i, 1] - b.lastMass) if alive else (-1 * b.lastMass * p.DEATH_FACTOR + p.DEATH_TERM))
                assert b.getReward() == pytest.approx(want * p.REWARD_SCALE - p.REWARD_TERM, abs=1e-9), (t, i)
        m.takeBotActions()
        o.policy_greedy(True)  # (the oracle's Greedy moves, for comparison; commands are replaced below)
        greedy_cmd = o.commands()
        for b in nn:  # the NN bots that computed a state this tick, against the oracle's
            i = b.player.index
            if b.oldState is not None and b.oldState is not before[i]:
                row = o.observe_one(i)
                assert parity.obs_close(b.oldState.reshape(-1), row), "tick %d bot %d: state differs" % (t, i)
                seen[i].append(t)
        cmd = m.field._cmd.copy()
        for b in bots:
            if b.type == "Greedy" and stats0[b.player.index, 0] > 0:
                assert np.array_equal(cmd[b.player.index], greedy_cmd[b.player.index]), "tick %d greedy" % t
        m.field.update()
        o.set_commands(cmd)
        o.step(1)
        assert np.array_equal(m.field.events(), o.events()), "tick %d: events differ" % t
    assert all(len(v) >= 15 for v in seen.values()), seen
    # every NN bot computed its state every FRAME_SKIP_RATE + 1 ticks while alive
    for i, ticks in seen.items():
        gaps = set(np.diff(ticks).tolist())
        assert 4 in gaps, (i, ticks[:10])
    dif = parity.diff_states(m.field.stepper.get_state(), o.get_state())
    assert not dif, dif
    # experiences: (state, action, reward, next state, raw action) tuples, rewards per bot.py:654-667
    for b in nn:
        assert len(b.experiences) >= 10
        for s, a, r, s2, raw in b.experiences:
            assert s.shape == (1, m.field.stepper.obs_len) and len(a) == 4 and np.isfinite(r)
    o.close()


def test_cnn_pixel_state_representation():
    """CNN_REPR + CNN_P_REPR (bot.py:276-282): the state is the pixel frame of
    RGBGenerator.get_cnn_inputRGB (grayscale, CNN_P_RGB False) normalised as
    (rgb - 255) / 100; with CNN_LAST_GRID the reference concatenates with a None
    last grid on the first frame and raises -- the facade raises the same way."""
    p = params()
    p.CNN_REPR, p.CNN_P_REPR, p.CNN_P_RGB, p.CNN_LAST_GRID = True, True, False, False
    p.CNN_USE_L1, p.CNN_INPUT_DIM_1 = True, 42
    m = model.Model(False, False, p, seed=2, field_size=300)
    bots = [m.createBot("NN", StubLearner()) for _ in range(8)]
    m.initialize()
    s = bots[0].getStateRepresentation()
    frames = m.field.observe_pixels_all(42, rgb=False)
    want = (frames[bots[0].player.index][..., None] - 255) / 100
    assert s.shape == (42, 42, 1) and np.array_equal(s, want)
    for _ in range(10):
        m.update()
    assert all(b.oldState is not None and b.oldState.shape == (42, 42, 1) for b in bots if b.player.getIsAlive())
    p.CNN_LAST_GRID = True
    b = model.Bot(bots[1].player, m.field, "NN", StubLearner(), p, m.rgbGenerator)
    with pytest.raises(ValueError):
        b.getStateRepresentation()


@pytest.mark.parametrize("variant", ["simple", "cnn_grid"])
def test_state_variants_through_the_facade(variant):
    """Bot.getStateRepresentation for GRID_VIEW_ENABLED = False (a 12-value list,
    bot.py:296-297, 511-547) and for the CNN over the grid view (CNN_REPR without
    CNN_P_REPR: [NUM_OF_GRIDS, 84, 84], bot.py:284), equal to the oracle's states
    of the same bots in the same world."""
    p = params()
    if variant == "simple":
        p.GRID_VIEW_ENABLED = False
    else:
        p.CNN_REPR, p.CNN_P_REPR = True, False
        p.CNN_USE_L1, p.CNN_USE_L2, p.CNN_INPUT_DIM_1, p.CNN_INPUT_DIM_2 = False, True, 42, 84
    m = model.Model(False, False, p, seed=6, field_size=300, max_viruses=10)
    bots = [m.createBot("Greedy") for _ in range(10)]
    m.initialize()
    o = Oracle(m.field.stepper.cfg)
    o.load_state(m.field.stepper.get_state())
    for t in range(12):
        m.update()
        o.set_commands(_commands(m.field.stepper.get_state()))  # the commands the tick ran with
        o.step(1)
    want = o.observe()
    for b in bots:
        s = b.getStateRepresentation()
        i = b.player.index
        if not b.player.getIsAlive():
            assert s is None
            continue
        if variant == "simple":
            assert isinstance(s, list) and len(s) == 12
            got = np.array(s)
        else:
            assert s.shape == (7, 84, 84)
            got = s.reshape(-1)
        assert parity.obs_close(got[None], want[i][None]), (variant, i)
    o.close()


def _commands(st):
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]].astype(np.float64)
