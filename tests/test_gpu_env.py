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
        obs, rew, alive = env.step(act)
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
        oa, ra, la = a.step(act)
        ob, rb, lb = b.step_calls(act)
        torch.cuda.synchronize()
        assert torch.equal(torch.nan_to_num(oa, nan=-7.0), torch.nan_to_num(ob, nan=-7.0)), t
        assert torch.equal(ra, rb), t
        assert torch.equal(la, lb), t
    assert parity.diff_states(a.stepper.get_state(), b.stepper.get_state(), ftol=0.0) == []
    a.close()
    b.close()
