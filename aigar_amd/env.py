"""Vectorised environment for learners (NN-bot glue).

Replaces the reference's per-bot NN plumbing -- Bot.move_NN / updateRewards /
updateFrameSkip / updateValues (bot.py:166-233) driven by
`aigar.py:performModelSteps` (aigar.py:795-887) -- with batched device calls:
every player is an NN bot whose action comes from the learner as one
[n_players, n_act] tensor.  All tensors stay on the GPU (torch-ROCm).

Per decision (`step`): the action is applied through set_command_point and
held for FRAME_SKIP_RATE + 1 ticks with split/eject dropped on the skipped
ticks; the reward is the reference's cumulative reward over the window
(getReward each tick against the lastMass of the previous decision); the
observation is Bot.getStateRepresentation of every player (NaN rows for dead
players, where the reference returns None).
"""
import numpy as np

from . import _abi
from ._lib import Stepper
from .model import obs_masks


class AgarVecEnv:
    def __init__(self, n_players, parameters=None, n_arenas=1, virus=None, field_size=0, max_pellets=-1.0,
                 max_viruses=-1.0, device=0, torch_stream=True):
        import torch
        self.torch = torch
        self.parameters = parameters
        g = (lambda n, dflt: getattr(parameters, n, dflt)) if parameters is not None else (lambda n, dflt: dflt)
        ch, ex, gsq = obs_masks(parameters)
        virus = bool(g("VIRUS_SPAWN", False)) if virus is None else bool(virus)
        if not virus:
            ch &= ~_abi.OBS_VIRUS
        c = _abi.Config()
        c.n_arenas, c.bots_per_arena, c.field_size = n_arenas, n_players, field_size
        c.virus_enabled = int(virus)
        c.max_pellets, c.max_viruses = float(max_pellets), float(max_viruses)
        c.grid_squares, c.obs_channels, c.obs_extras = gsq, ch, ex
        c.rng_mode, c.device = _abi.RNG_PHILOX, device
        self.stepper = Stepper(c)
        self.dev = torch.device("cuda", device)
        if torch_stream:
            self.stepper.set_stream(torch.cuda.current_stream(self.dev).cuda_stream)
        self.NP = self.stepper.NP
        self.skip = int(g("FRAME_SKIP_RATE", 0))
        self.enable_split = bool(g("ENABLE_SPLIT", False))
        self.reward_params = _abi.RewardParams.from_parameters(parameters)
        self.obs = torch.empty((self.NP, self.stepper.obs_len), dtype=torch.float64, device=self.dev)
        self._r = torch.empty(self.NP, dtype=torch.float64, device=self.dev)
        self._act = {}  # n_act -> persistent action buffer (the decision graph is keyed by its address)

    def reset(self, seed=0):
        """Field.reset + NN bots' reset (lastMass = None, history grids cleared)."""
        self.stepper.reset(seed)
        return self.observe()

    def observe(self):
        """A fresh tensor: the device buffer is rewritten by the next decision, so
        (s, a, r, s') tuples must not alias it (self.obs is that buffer)."""
        self.stepper.observe(self.obs)
        return self.obs.clone()

    def step(self, actions):
        """actions: [n_players, 2..4] tensor/array in [0, 1] -> (obs, reward, alive).
        The whole decision (skip + 1 ticks, rewards, observation) is one graph replay."""
        torch = self.torch
        act = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions), device=self.dev)
        n = int(act.shape[1])
        buf = self._act.get(n)
        if buf is None:
            buf = self._act[n] = torch.empty((self.NP, n), dtype=torch.float64, device=self.dev)
        buf.copy_(act)
        self.stepper.env_step(buf, self._r, self.obs, self.enable_split, self.skip, self.reward_params)
        alive = ~torch.isnan(self.obs[:, 0])
        return self.obs.clone(), self._r.clone(), alive

    def step_calls(self, actions):
        """The same decision as separate calls (apply_actions / step / rewards / observe)."""
        torch = self.torch
        act = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions), device=self.dev)
        act = act.to(device=self.dev, dtype=torch.float64).contiguous()
        reward = torch.zeros(self.NP, dtype=torch.float64, device=self.dev)
        for k in range(self.skip + 1):
            if k > 0:  # updateRewards on the skipped frames (bot.py:166-168)
                self.stepper.rewards(self.reward_params, update_last=False, out=self._r)
                reward += torch.nan_to_num(self._r)
            self.stepper.apply_actions(act, self.enable_split, skipping=k > 0, record=k == 0)
            self.stepper.step(1)
        self.stepper.rewards(self.reward_params, update_last=True, out=self._r)
        reward += torch.nan_to_num(self._r)
        obs = self.observe()
        alive = ~torch.isnan(obs[:, 0])
        return obs, reward, alive

    def close(self):
        self.stepper.close()
