import os, sys, types
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT]
import torch
from aigar_amd.env import AgarVecEnv
p = types.SimpleNamespace(VIRUS_SPAWN=True, ENABLE_SPLIT=True, PELLET_GRID=True, SELF_GRID=True, WALL_GRID=True,
                          ENEMY_GRID=True, VIRUS_GRID=True, SELF_GRID_LF=True, ENEMY_GRID_LF=True,
                          USE_FOVSIZE=True, USE_TOTALMASS=True, USE_LAST_ACTION=True, USE_LAST_FOVSIZE=True,
                          GRID_SQUARES_PER_FOV=11, EXTRA_INPUT=True, FRAME_SKIP_RATE=3)
env = AgarVecEnv(64, p, field_size=600, max_viruses=10)
obs = env.reset(3)
for it in range(10):
    act = torch.rand((64, 4), dtype=torch.float64, device="cuda")
    obs, rew, alive = env.step(act)
    live = alive.nonzero().flatten()
    a = obs[live, 7 * 121 + 3:7 * 121 + 7]
    bad = (a != act[live]).any(dim=1).nonzero().flatten()
    if len(bad):
        for b in bad.tolist():
            i = live[b].item()
            print("step", it, "player", i, "obs", obs[i, 7 * 121:].tolist(), "act", act[i].tolist())
print("done")
