#!/usr/bin/env python3
"""Learner-loop throughput: AgarVecEnv decisions at C3
size with the reference's NN-bot frame skipping (FRAME_SKIP_RATE = 7,
networkParameters.py:33), one graph replay per decision (env.step) against the
same decision as separate calls (env.step_calls).  Prints one JSON line."""
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from aigar_amd.env import AgarVecEnv
    p = types.SimpleNamespace(VIRUS_SPAWN=True, ENABLE_SPLIT=True, PELLET_GRID=True, SELF_GRID=True, WALL_GRID=True,
                              ENEMY_GRID=True, VIRUS_GRID=True, SELF_GRID_LF=True, ENEMY_GRID_LF=True,
                              USE_FOVSIZE=True, USE_TOTALMASS=True, USE_LAST_ACTION=True, USE_LAST_FOVSIZE=True,
                              GRID_SQUARES_PER_FOV=11, EXTRA_INPUT=True, FRAME_SKIP_RATE=7)
    bots, n = 4096, 40
    out = {"workload": "C3 AgarVecEnv: 4096 NN bots, field 4800, 100k pellets, viruses, FRAME_SKIP_RATE 7",
           "ticks_per_decision": p.FRAME_SKIP_RATE + 1}
    for name in ("step", "step_calls"):
        env = AgarVecEnv(bots, p, field_size=4800, max_pellets=100000.0)
        env.reset(1)
        act = torch.rand((bots, 4), dtype=torch.float64, device="cuda")
        f = getattr(env, name)
        for _ in range(5):
            f(act)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            f(act)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[name] = {"decisions_per_s": n / dt, "ms_per_decision": dt / n * 1e3,
                     "env_steps_per_s": bots * n * (p.FRAME_SKIP_RATE + 1) / dt}
        env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
