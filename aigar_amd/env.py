"""Vectorised environment for learners (NN-bot glue).

Replaces the reference's per-bot NN plumbing -- Bot.move_NN / updateRewards /
updateFrameSkip / updateValues (bot.py:166-233) driven by
`aigar.py:performModelSteps` (aigar.py:795-887) -- with batched device calls:
the NN players' actions come from the learner as one [n_players, n_act]
tensor.  All tensors stay on the GPU (torch-ROCm).

Populations (aigar.py:767-780 trains NN bots among Greedy and Random bots):
`roles` gives every player of an arena "NN", "Greedy" or "Random".  The Greedy
bots (bot.py:579-633) and the Random bots (bot.py:243-249: a new random action
every FRAME_SKIP_RATE moves) move on the device every tick; the learner's
actions apply to the NN players only, and only they are observed.

Per decision (`step`): the NN actions go through set_command_point and are held
for FRAME_SKIP_RATE + 1 ticks with split/eject dropped on the skipped ticks;
the reward is the reference's cumulative reward over the window (getReward
each tick against the lastMass of the previous decision); the observation is
Bot.getStateRepresentation of every NN player (NaN rows for dead players, where
the reference returns None).

Episodes (aigar.py:833-837, 876-887): an arena's episode ends after the
decision in which its tick count passes RESET_LIMIT - FRAME_SKIP_RATE + 2 (the
reference's collector test); the arena is then reset (Model.resetModel + the
bots' reset) and reported in `done`.  With several arenas the game stages are
desynchronised the way the reference desynchronises its collectors: before the
first decision arena k has played k * int(RESET_LIMIT / n_arenas) ticks of its
own world with its own population (the NN players on random actions during
that warm-up, the reference's untrained networks), then every bot is reset
(Model.resetBots).
"""
import numpy as np

from . import _abi
from ._lib import Stepper
from .model import obs_masks


class AgarVecEnv:
    def __init__(self, n_players, parameters=None, n_arenas=1, virus=None, field_size=0, max_pellets=-1.0,
                 max_viruses=-1.0, device=0, torch_stream=True, roles=None, reset_limit=None, desync=True, seed=0):
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
        self.NP, self.A, self.B = self.stepper.NP, n_arenas, n_players
        self.skip = int(g("FRAME_SKIP_RATE", 0))
        self.enable_split = bool(g("ENABLE_SPLIT", False))
        self.reward_params = _abi.RewardParams.from_parameters(parameters)
        self.seed = int(seed)
        # roles: per player of one arena (repeated in every arena) or of all arenas
        if roles is None:
            roles = ["NN"] * n_players
        roles = [_abi.ROLES[r] if isinstance(r, str) else int(r) for r in roles]
        if len(roles) == n_players:
            roles = roles * n_arenas
        if len(roles) != self.NP:
            raise ValueError("roles: %d entries for %d players per arena x %d arenas" % (len(roles), n_players,
                                                                                          n_arenas))
        self.roles = np.array(roles, np.uint8)
        self.stepper.set_roles(self.roles)
        self.stepper.env_config(greedy_split=bool(g("ENABLE_GREEDY_SPLIT", False)), random_skip=max(1, self.skip),
                                random_split=self.enable_split, random_eject=bool(g("ENABLE_EJECT", False)),
                                salt=self.seed)
        self.nn = torch.as_tensor(self.roles == _abi.ROLE_NN, device=self.dev)
        self._nn_u8 = self.nn.to(torch.uint8)
        self._mixed = bool((self.roles != _abi.ROLE_NN).any())
        self.reset_limit = int(g("RESET_LIMIT", 20000) if reset_limit is None else reset_limit)
        self.desync = bool(desync) and self.reset_limit > 0 and n_arenas > 1
        self.age = np.zeros(n_arenas, np.int64)
        self._resets = 0
        self.obs = torch.empty((self.NP, self.stepper.obs_len), dtype=torch.float64, device=self.dev)
        self._mask = torch.zeros(self.NP, dtype=torch.uint8, device=self.dev)  # (persistent: read on the stepper's stream)
        self._r = torch.empty(self.NP, dtype=torch.float64, device=self.dev)
        self._act = {}  # n_act -> persistent action buffer (the decision graph is keyed by its address)

    def reset(self, seed=None):
        """Field.reset + every bot's reset (lastMass = None, history grids cleared);
        with several arenas, the desynchronising warm-up (aigar.py:833-837)."""
        seed = self.seed if seed is None else int(seed)
        self.stepper.reset(seed)
        self.age[:] = 0
        self._resets = 0
        if self.desync:
            self._desynchronise(seed)
        return self.observe()

    def _desynchronise(self, seed):
        """Arena k plays k * int(R / N) ticks from a fresh world before the first
        decision (collector k + 1 of aigar.py:833-837): all arenas are stepped
        together for (N - 1) * int(R / N) ticks and arena k gets its fresh world when
        k * int(R / N) of them are left; then Model.resetBots for every arena."""
        per = self.reset_limit // self.A
        total = (self.A - 1) * per
        has_g, has_r = bool((self.roles == _abi.ROLE_GREEDY).any()), bool((self.roles == _abi.ROLE_RANDOM).any())
        greedy = self.torch.as_tensor(self.roles == _abi.ROLE_GREEDY, device=self.dev).to(self.torch.uint8)
        gsplit = bool(getattr(self.parameters, "ENABLE_GREEDY_SPLIT", False)) if self.parameters is not None else False
        for t in range(total + 1):
            for a in range(self.A):
                if t > 0 and total - a * per == t:
                    self.stepper.reset_arena(a, seed + 104729 * (a + 1))
            if t == total:
                break
            # NN players: random points in their view (an untrained network's moves);
            # Greedy / Random bots: their own device policies
            self.stepper.policy_random(0.0, 0.0, seed ^ 0x5DEECE66D)
            if has_g:
                self.stepper.policy_greedy(gsplit, greedy)
            if has_r:
                self.stepper.policy_random_bots()
            self.stepper.step(1)
        for a in range(self.A):  # Model.resetBots: every bot of every arena (the world goes on)
            self.stepper.load_state(self.stepper.get_state(a), a)
        self.age[:] = np.arange(self.A) * per

    def episode_over(self):
        """Arenas whose episode is over: the collector's test step > RESET_LIMIT -
        FRAME_SKIP_RATE + 2 (aigar.py:876)."""
        return self.age > self.reset_limit - self.skip + 2

    def observe(self):
        """A fresh tensor: the device buffer is rewritten by the next decision, so
        (s, a, r, s') tuples must not alias it (self.obs is that buffer)."""
        self.stepper.observe(self.obs, mask=self._nn_u8 if self._mixed else None)
        return self.obs.clone()

    def _episode_ends(self):
        """Reset the arenas that reached RESET_LIMIT; returns the per-player done mask."""
        torch = self.torch
        done = torch.zeros(self.NP, dtype=torch.bool, device=self.dev)
        if self.reset_limit <= 0:
            return done
        self.age += self.skip + 1
        ended = np.nonzero(self.episode_over())[0]
        if not len(ended):
            return done
        mask = np.zeros(self.NP, np.uint8)
        for a in ended:
            self._resets += 1
            self.stepper.reset_arena(int(a), self.seed + 7919 * self._resets)
            self.age[a] = 0
            mask[a * self.B:(a + 1) * self.B] = 1
        done[torch.as_tensor(mask.astype(bool), device=self.dev)] = True
        # the new episodes' first states (NN players of the reset arenas)
        nn_reset = (mask & (self.roles == _abi.ROLE_NN)).astype(np.uint8)
        self._mask.copy_(torch.as_tensor(nn_reset))
        self.stepper.observe(self.obs, mask=self._mask)
        return done

    def step(self, actions):
        """actions: [n_players, 2..4] tensor/array in [0, 1] (rows of non-NN players are
        ignored) -> (obs, reward, alive, done).  The decision (skip + 1 ticks, every
        bot's moves, rewards, NN observations) is one graph replay."""
        torch = self.torch
        act = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions), device=self.dev)
        n = int(act.shape[1])
        buf = self._act.get(n)
        if buf is None:
            buf = self._act[n] = torch.empty((self.NP, n), dtype=torch.float64, device=self.dev)
        buf.copy_(act)
        self.stepper.env_step(buf, self._r, self.obs, self.enable_split, self.skip, self.reward_params)
        reward = self._r.clone()
        done = self._episode_ends()
        alive = ~torch.isnan(self.obs[:, 0]) & self.nn
        return self.obs.clone(), reward, alive, done

    def step_calls(self, actions):
        """The same decision as separate calls (apply_actions / Greedy bots / Random
        bots / step / rewards / observe); without the episode bookkeeping."""
        torch = self.torch
        act = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions), device=self.dev)
        act = act.to(device=self.dev, dtype=torch.float64).contiguous()
        reward = torch.zeros(self.NP, dtype=torch.float64, device=self.dev)
        greedy = torch.as_tensor(self.roles == _abi.ROLE_GREEDY, device=self.dev).to(torch.uint8)
        has_g, has_r = bool((self.roles == _abi.ROLE_GREEDY).any()), bool((self.roles == _abi.ROLE_RANDOM).any())
        gsplit = bool(getattr(self.parameters, "ENABLE_GREEDY_SPLIT", False)) if self.parameters is not None else False
        for k in range(self.skip + 1):
            if k > 0:  # updateRewards on the skipped frames (bot.py:166-168)
                self.stepper.rewards(self.reward_params, update_last=False, out=self._r)
                reward += torch.nan_to_num(self._r)
            self.stepper.apply_actions(act, self.enable_split, skipping=k > 0, record=k == 0)
            if has_g:
                self.stepper.policy_greedy(gsplit, greedy)
            if has_r:
                self.stepper.policy_random_bots()
            self.stepper.step(1)
        self.stepper.rewards(self.reward_params, update_last=True, out=self._r)
        reward += torch.nan_to_num(self._r)
        obs = self.observe()
        alive = ~torch.isnan(obs[:, 0]) & self.nn
        return obs, reward, alive

    def close(self):
        self.stepper.close()
