"""GPU: learner-facing glue -- set_command_point for external actions, the
reference's getReward, and the vectorised environment built on them --
against the oracle and a direct restatement of bot.py:654-667."""
import types

import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu
_lib = pytest.importorskip("aigar_amd._lib")


def set_command_point(stats, act):
    """bot.py:550-577 for 4-element actions, from (alive, mass, fov x, fov y, fov size)."""
    cmd = np.zeros((len(act), 4))
    for i, (s, a) in enumerate(zip(stats, act)):
        if not s[0] > 0:
            continue  # dead: no command (the caller keeps the old one)
        x, y, size = int(s[2]), int(s[3]), s[4]
        left, top = x - int(size / 2), y - int(size / 2)
        cmd[i] = (left + a[0] * int(size), top + a[1] * int(size), a[2] > 0.5, a[3] > 0.5)
    return cmd


def get_reward(alive, mass, last, p):
    """bot.py:654-667 (MASS_AS_REWARD False); None -> NaN."""
    if np.isnan(last):
        return np.nan
    r = (-1 * last * p.DEATH_FACTOR + p.DEATH_TERM) if not alive else mass - last
    return r * p.REWARD_SCALE - p.REWARD_TERM


def test_actions_and_rewards_match_reference_formulas():
    cfg = make_config(bots=40, field_size=150, channels=_abi.OBS_PELLET | _abi.OBS_ENEMY, extras=0x1F)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(9)
    o.reset(9)
    prm = types.SimpleNamespace(REWARD_TERM=0.0, DEATH_TERM=-40.0, DEATH_FACTOR=1.5, REWARD_SCALE=2.0)
    last = np.full(40, np.nan)
    rng = np.random.default_rng(9)
    for t in range(80):
        stats = o.player_stats()
        act = rng.random((40, 4))
        act[:, 2:] = act[:, 2:] > 0.9
        g.apply_actions(act, enable_split=True, skipping=False, record=True)
        cmd = set_command_point(stats, act)
        alive = stats[:, 0] > 0
        o_cmd = o.commands()
        cmd[~alive] = o_cmd[~alive]  # dead players keep their old command (makeMove returns)
        o.set_commands(cmd)
        gs = g.get_state()
        assert np.array_equal(np.c_[gs["players_f"], gs["players_i"][:, 2:4]], cmd), "tick %d" % t
        g.step(1)
        o.step(1)
        stats = o.player_stats()
        want = np.array([get_reward(stats[i, 0] > 0, stats[i, 1], last[i], prm) for i in range(40)])
        got = g.rewards(prm, update_last=True)
        assert parity.obs_close(got, want, 1e-9), "rewards at tick %d" % t
        last = np.where(stats[:, 0] > 0, stats[:, 1], last)
    assert not parity.diff_states(g.get_state(), o.get_state())
    g.close()
    o.close()


def test_vec_env_runs_on_device_tensors():
    import torch
    from aigar_amd.env import AgarVecEnv
    p = types.SimpleNamespace(VIRUS_SPAWN=True, ENABLE_SPLIT=True, PELLET_GRID=True, SELF_GRID=True, WALL_GRID=True,
                              ENEMY_GRID=True, VIRUS_GRID=True, SELF_GRID_LF=True, ENEMY_GRID_LF=True,
                              USE_FOVSIZE=True, USE_TOTALMASS=True, USE_LAST_ACTION=True, USE_LAST_FOVSIZE=True,
                              GRID_SQUARES_PER_FOV=11, EXTRA_INPUT=True, FRAME_SKIP_RATE=3)
    env = AgarVecEnv(64, p, field_size=600, max_viruses=10)
    obs = env.reset(3)
    assert obs.shape == (64, 7 * 121 + 7) and obs.is_cuda
    was_alive = ~torch.isnan(obs[:, 0])
    for _ in range(10):
        act = torch.rand((64, 4), dtype=torch.float64, device="cuda")
        obs, rew, alive, done = env.step(act)
        assert not done.any()
        assert rew.shape == (64,) and alive.dtype == torch.bool and torch.isfinite(rew).all()
        # the observation's last-action extras are the action just taken (bot.py:316-319);
        # a player dead when the action came keeps its old one (makeMove returns, bot.py:257)
        live = (alive & was_alive).nonzero().flatten()
        assert torch.equal(obs[live, 7 * 121 + 3:7 * 121 + 7], act[live])
        was_alive = alive
    env.close()


def test_vec_env_decision_graph_matches_separate_calls():
    """AgarVecEnv.step (one aigar_env_step graph replay per decision) == the same
    decision issued as apply_actions / step / rewards / observe calls."""
    import torch
    from aigar_amd.env import AgarVecEnv
    p = types.SimpleNamespace(VIRUS_SPAWN=True, ENABLE_SPLIT=True, PELLET_GRID=True, SELF_GRID=True, WALL_GRID=True,
                              ENEMY_GRID=True, VIRUS_GRID=True, SELF_GRID_LF=True, ENEMY_GRID_LF=True,
                              USE_FOVSIZE=True, USE_TOTALMASS=True, USE_LAST_ACTION=True, USE_LAST_FOVSIZE=True,
                              GRID_SQUARES_PER_FOV=11, EXTRA_INPUT=True, FRAME_SKIP_RATE=7)
    a, b = AgarVecEnv(48, p, field_size=300, max_viruses=8), AgarVecEnv(48, p, field_size=300, max_viruses=8)
    oa, ob = a.reset(5), b.reset(5)
    assert torch.equal(torch.nan_to_num(oa, nan=-7.0), torch.nan_to_num(ob, nan=-7.0))
    gen = torch.Generator(device="cuda").manual_seed(5)
    for t in range(12):
        act = torch.rand((48, 4 if t % 3 else 3), dtype=torch.float64, device="cuda", generator=gen)
        oa, ra, la, _ = a.step(act)
        ob, rb, lb = b.step_calls(act)
        torch.cuda.synchronize()
        assert torch.equal(torch.nan_to_num(oa, nan=-7.0), torch.nan_to_num(ob, nan=-7.0)), t
        assert torch.equal(ra, rb), t
        assert torch.equal(la, lb), t
    assert parity.diff_states(a.stepper.get_state(), b.stepper.get_state(), ftol=0.0) == []
    a.close()
    b.close()


def _params(**kw):
    base = dict(VIRUS_SPAWN=True, ENABLE_SPLIT=True, ENABLE_EJECT=False, ENABLE_GREEDY_SPLIT=True, PELLET_GRID=True,
                SELF_GRID=True, WALL_GRID=True, ENEMY_GRID=True, VIRUS_GRID=True, SELF_GRID_LF=True,
                ENEMY_GRID_LF=True, USE_FOVSIZE=True, USE_TOTALMASS=True, USE_LAST_ACTION=True,
                USE_LAST_FOVSIZE=True, GRID_SQUARES_PER_FOV=11, EXTRA_INPUT=True, FRAME_SKIP_RATE=3)
    base.update(kw)
    return types.SimpleNamespace(**base)


def test_mixed_population_graph_matches_separate_calls():
    """NN bots among Greedy and Random bots (aigar.py:767-780): the decision graph
    (learner actions for the NN players, device Greedy / Random moves every tick,
    NN observations only) == the same decision as separate calls."""
    import torch
    from aigar_amd.env import AgarVecEnv
    p = _params()
    roles = ["NN"] * 16 + ["Greedy"] * 16 + ["Random"] * 16
    a = AgarVecEnv(48, p, field_size=300, max_viruses=8, roles=roles, seed=3)
    b = AgarVecEnv(48, p, field_size=300, max_viruses=8, roles=roles, seed=3)
    oa, ob = a.reset(5), b.reset(5)
    nn = torch.zeros(48, dtype=torch.bool, device="cuda")
    nn[:16] = True
    assert torch.equal(torch.nan_to_num(oa[nn], nan=-7.0), torch.nan_to_num(ob[nn], nan=-7.0))
    gen = torch.Generator(device="cuda").manual_seed(5)
    for t in range(15):
        act = torch.rand((48, 4), dtype=torch.float64, device="cuda", generator=gen)
        oa, ra, la, _ = a.step(act)
        ob, rb, lb = b.step_calls(act)
        torch.cuda.synchronize()
        assert torch.equal(torch.nan_to_num(oa[nn], nan=-7.0), torch.nan_to_num(ob[nn], nan=-7.0)), t
        assert torch.equal(ra, rb) and torch.equal(la, lb), t
    assert parity.diff_states(a.stepper.get_state(), b.stepper.get_state(), ftol=0.0) == []
    a.close()
    b.close()


def test_mixed_population_matches_oracle():
    """Each role against the reference's rules driven on the oracle: NN players
    through set_command_point (bot.py:550-577), Greedy players' commands equal
    the oracle's Greedy bots' (bot.py:579-633), Random players hold a Philox-drawn
    action for FRAME_SKIP_RATE moves (bot.py:243-249); the worlds stay equal."""
    from aigar_amd import _lib as L
    from oracle_lib import lib as oracle_c
    import ctypes as C
    p = _params(FRAME_SKIP_RATE=4)
    n = 36
    roles = np.array([0] * 12 + [1] * 12 + [2] * 12, np.uint8)
    cfg = make_config(bots=n, field_size=260, virus=True, max_viruses=10, channels=_abi.OBS_PELLET, extras=0x3)
    g, o = L.Stepper(cfg), Oracle(cfg)
    g.reset(8)
    o.reset(8)
    g.set_roles(roles)
    salt = 99
    g.env_config(greedy_split=True, random_skip=4, random_split=True, random_eject=False, salt=salt)
    key = np.array(o.get_state()["philox_key"], np.uint64)
    held = np.zeros((n, 4))
    t_rand = np.zeros(n, np.int64)
    rng = np.random.default_rng(8)
    OC = oracle_c()
    for t in range(60):
        stats = o.player_stats()
        act = rng.random((n, 4))
        g.apply_actions(act, enable_split=True, skipping=False, record=True)
        g.policy_greedy(True, (roles == 1).astype(np.uint8))
        g.policy_random_bots()
        o.policy_greedy(True)
        cmd = o.commands()  # Greedy players: the oracle's greedy moves
        alive = stats[:, 0] > 0
        nn_cmd = set_command_point(stats, act)
        for i in range(n):
            if roles[i] == 0 and alive[i]:
                cmd[i] = nn_cmd[i]
            elif roles[i] == 2 and alive[i]:
                if t_rand[i] % 4 == 0:
                    ctr = np.array([i, 9, t_rand[i], salt], np.uint64)
                    u = np.zeros(4, np.uint64)
                    OC.oracle_philox(ctr.ctypes.data_as(C.POINTER(C.c_uint64)), key.ctypes.data_as(C.POINTER(C.c_uint64)),
                                     u.ctypes.data_as(C.POINTER(C.c_uint64)))
                    held[i] = [(int(v) >> 11) * (1.0 / 9007199254740992.0) for v in u]
                    held[i, 3] = 0.0
                t_rand[i] += 1
                cmd[i] = set_command_point(stats[i:i + 1], held[i:i + 1])[0]
        gs = g.get_state()
        got = np.c_[gs["players_f"], gs["players_i"][:, 2:4]]
        live = np.nonzero(alive)[0]
        assert np.array_equal(got[live], cmd[live]), "tick %d: %s" % (t, np.argwhere(got[live] != cmd[live])[:3])
        o.set_commands(got)
        g.step(1)
        o.step(1)
        assert np.array_equal(g.events(), o.events()), "tick %d" % t
    assert parity.diff_states(g.get_state(), o.get_state()) == []
    g.close()
    o.close()


def test_reset_limit_and_desynchronised_arenas():
    """RESET_LIMIT episodes (aigar.py:876-887) with desynchronised arenas
    (aigar.py:833-837): before the first decision arena a has played a *
    int(R / N) ticks of its own world; an episode ends after the decision in which
    the arena's tick count passes R - FRAME_SKIP_RATE + 2, with a fresh world and
    fresh bots."""
    import torch
    from aigar_amd.env import AgarVecEnv
    p = _params(FRAME_SKIP_RATE=1, RESET_LIMIT=16)
    env = AgarVecEnv(32, p, n_arenas=4, field_size=250, max_viruses=6, seed=1)
    env.reset(2)
    assert [env.stepper.get_state(a)["tick"] for a in range(4)] == [0, 4, 8, 12]
    w = [env.stepper.get_state(a) for a in range(4)]
    assert len({int(x["n_pellets"]) for x in w} | {int(x["seq_next"]) for x in w}) > 1  # different game stages
    ends = []
    for t in range(20):
        act = torch.rand((128, 4), dtype=torch.float64, device="cuda")
        obs, rew, alive, done = env.step(act)
        arenas = sorted(set((done.nonzero().flatten() // 32).tolist()))
        ends.append(arenas)
        for a in arenas:
            st = env.stepper.get_state(a)
            assert st["tick"] == 0 and st["n_cells"] == 32  # a fresh world, every player respawned
            assert not torch.isnan(obs[a * 32:(a + 1) * 32, 0]).any()  # the new episode's first states
    # 2 ticks per decision; arena a starts at 4a ticks and ends when its count passes 16 - 1 + 2 = 17
    for a in range(4):
        hits = [t for t, e in enumerate(ends) if a in e]
        first = (17 - 4 * a) // 2  # the decision index t with 4a + 2 (t + 1) > 17 first
        assert hits == [h for h in (first, first + 9, first + 18) if h < 20], (a, hits)
    # an explicit reset restarts the timers and the desynchronisation
    env.reset(3)
    assert list(env.age) == [0, 4, 8, 12]
    env.close()
