"""GPU: the reference's collector loop drives the fast facade unchanged.

`performModelSteps` (/root/reference/src/aigar.py:795-887) is replayed call for
call on `aigar_amd.model.Model`: createModelPlayers (NN, Greedy, Random bots,
aigar.py:767-780), initialize, the desynchronisation updates and resetBots
(:833-838), then windows of FRAME_SKIP_RATE + 2 updates, each followed by
getNNBots / getExperiences / resetBots (:845-852) and the learners'
setNetworkWeights (:870-871), and at RESET_LIMIT getMassOverTime /
resetMassList / resetModel (:876-887).  A stub learner (decideMove of a fixed
function of the state, the shape of actorCritic.py:938) checks every state it
is handed against the oracle's observation of that bot at that moment; the
oracle runs in lockstep on the commands each tick ran with, and every tick's
events and (periodically) the world are compared."""
import types

import numpy as np
import pytest

from oracle_lib import Oracle
import parity

pytestmark = pytest.mark.gpu
model = pytest.importorskip("aigar_amd.model")


def params():
    return types.SimpleNamespace(
        VIRUS_SPAWN=True, ENABLE_SPLIT=True, ENABLE_EJECT=False, ENABLE_GREEDY_SPLIT=True, GRID_VIEW_ENABLED=True,
        CNN_REPR=False, PELLET_GRID=True, SELF_GRID=True, WALL_GRID=True, ENEMY_GRID=True, VIRUS_GRID=True,
        SELF_GRID_LF=True, ENEMY_GRID_LF=True, SELF_GRID_SLF=True, EXTRA_INPUT=True, USE_FOVSIZE=True,
        USE_TOTALMASS=True, USE_LAST_ACTION=True, USE_SECOND_LAST_ACTION=False, USE_LAST_FOVSIZE=True,
        GRID_SQUARES_PER_FOV=11, FRAME_SKIP_RATE=3, GATHER_EXP=True, MASS_AS_REWARD=False, REWARD_TERM=0.0,
        DEATH_TERM=-40.0, DEATH_FACTOR=1.5, REWARD_SCALE=2.0, ALGORITHM="CACLA", RESET_LIMIT=40,
        NUM_COLLECTORS=2, NUM_NN_BOTS=4, NUM_GREEDY_BOTS=4, NUM_RANDOM_BOTS=4, VIEW_ENABLED=False)


class CheckingLearner:
    """decideMove(state) -> (raw action, action); checks the state against the oracle."""
    discrete = False

    def __init__(self, check):
        self.check, self.index, self.weights, self.states = check, None, None, 0

    def __str__(self):
        return "AC"

    def reset(self):
        pass

    def decideMove(self, state):
        self.check(self.index, state)
        self.states += 1
        v = float(np.nansum(state))
        a = [(v * k) % 1.0 for k in (0.37, 0.71, 0.13, 0.97)]
        return list(a), a

    def setNetworkWeights(self, w):
        self.weights = w


def _commands(st):
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]].astype(np.float64)


def test_perform_model_steps_call_sequence_matches_oracle():
    p = params()
    np.random.seed(12)  # the Random bots draw from numpy's global stream, as the reference's
    m = model.Model(False, False, p, seed=12, field_size=320, max_viruses=10, record_events=True)
    box = {}

    def check(i, state):  # the oracle's observation of bot i at this moment of the tick
        want = box["o"].observe_one(i)
        assert parity.obs_close(np.asarray(state).reshape(-1), want), "tick %d bot %d: state differs" % (
            box["t"], i)

    learners = []
    for _ in range(p.NUM_NN_BOTS):  # createModelPlayers (aigar.py:767-780)
        ln = CheckingLearner(check)
        learners.append(ln)
        m.createBot("NN", ln, p)
    for _ in range(p.NUM_GREEDY_BOTS):
        m.createBot("Greedy", None, p)
    for _ in range(p.NUM_RANDOM_BOTS):
        m.createBot("Random", None, p)
    m.initialize()
    for b in m.getNNBots():
        b.getLearningAlg().index = b.getPlayer().index
    assert m.getNNBot() is m.getNNBots()[0] and m.getVirusEnabled() and m.getParameters() is p
    o = Oracle(m.field.stepper.cfg)
    o.load_state(m.field.stepper.get_state())
    box["o"], box["t"] = o, 0
    st = m.field.stepper
    # the device calls the facade makes that change observation inputs go to the oracle too
    dev_set_actions, dev_reset_bots = st.set_actions, st.reset_bots
    st.set_actions = lambda cur=None, prev=None: (dev_set_actions(cur, prev), o.set_actions(cur, prev))[0]
    st.reset_bots = lambda mask=None: (dev_reset_bots(mask), o.reset_bots(mask))[0]
    resets = [0]
    dev_reset = m.field.reset

    def field_reset():
        dev_reset()
        o.reset(m.field.seed + 7919 * m.field._resets)  # Field.reset's seed (model.py)
        resets[0] += 1
    m.field.reset = field_reset

    def update():  # model.update() + the oracle on the commands the tick ran with
        m.update()
        o.set_commands(_commands(st.get_state()))
        o.step(1)
        assert np.array_equal(m.field.events(), o.events()), "tick %d: events differ" % box["t"]
        box["t"] += 1

    process_num, step = 2, 0
    for _ in range((process_num - 1) * int(p.RESET_LIMIT / p.NUM_COLLECTORS)):  # desynchronisation
        update()
        step += 1
    m.resetBots()
    windows, masses = 0, []
    while windows < 14:
        for _ in range(p.FRAME_SKIP_RATE + 2):
            update()
            step += 1
        all_experience_lists = [bot.getExperiences() for bot in m.getNNBots()]
        m.resetBots()
        for lst in all_experience_lists:  # aigar.py:858-862: one experience per window (a live bot)
            assert len(lst) <= 1
        for bot in m.getNNBots():
            bot.getLearningAlg().setNetworkWeights({"w": windows})
        windows += 1
        if step > p.RESET_LIMIT - p.FRAME_SKIP_RATE + 2:
            for bot in m.getNNBots():
                masses.append(bot.getMassOverTime())
                bot.resetMassList()
                assert bot.getMassOverTime() == []
            m.resetModel()
            step = 0
            dif = parity.diff_states(st.get_state(), o.get_state())
            assert not dif, dif
    dif = parity.diff_states(st.get_state(), o.get_state())
    assert not dif, dif
    assert resets[0] >= 2, resets
    assert all(ln.states >= 10 for ln in learners), [ln.states for ln in learners]
    assert all(len(ms) > 0 for ms in masses)
    top = m.getTopTenPlayers()
    tm = [pl.getTotalMass() for pl in top]
    assert len(top) == 10 and tm == sorted(tm, reverse=True)
    assert len(m.getPellets()) == st.get_state()["n_pellets"] and len(m.getPlayerCells()) == st.get_state()["n_cells"]
    o.close()


def test_public_state_parts_equal_get_state_representation():
    """getGridStateRepresentation / getAdditionalFeatures (bot.py:302-497) read
    the same device observation getStateRepresentation flattens."""
    p = params()
    m = model.Model(False, False, p, seed=3, field_size=300, max_viruses=10)
    bots = [m.createBot("NN", None, p) for _ in range(6)]
    m.initialize()
    for _ in range(5):
        m.update()
    b = bots[2]
    s = b.getStateRepresentation()
    g, ex = b.getGridStateRepresentation(), b.getAdditionalFeatures()
    assert g.shape == (8, 11, 11) and len(ex) == 1 + 1 + 1 + 4
    assert np.array_equal(np.concatenate([g.reshape(-1), ex])[None], s)
    with pytest.raises(NotImplementedError):
        b.getSimpleStateRepresentation()
    assert b.getGridSquaresPerFov() == 11
