#!/usr/bin/env python3
"""Time the reference's own Python src/model on bench.py's workload.

CONTAINER-ONLY (the reference cannot travel to the GPU box): this imports the
read-only reference through the golden harness (tools/golden/gen_golden.py:
pygame stub, canonical-order shim), loads bench.py's start world
(data/c3_t50.npz, the C3 headline world: 4096 bots, field 4800, 100k pellets,
1152 viruses) into the reference's objects, and drives it with bench.py's
synthetic policy (a uniform point of each bot's FOV through the reference's
own Bot.set_command_point, split p = 2.5e-3, eject p = 1e-2).  One step =
the policy for every bot + Field.update() (field.py:85-92) + the grid
observation of every bot (Bot.getStateRepresentation, bot.py:272-299), the
same step bench.py times on the GPU.  One warm-up step, then --steps timed
steps, one core (the reference is single-threaded).

Writes profiles/<tag>_ref_python_c3.json, which bench.py quotes as
cpu_baseline.reference_python.

usage: python tools/golden/ref_cpu_bench.py [--steps 3] [--tag r05]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (container-only harness)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--tag", default="r05")
    ap.add_argument("--world", default="data/c3_t50.npz")
    ap.add_argument("--shim", action="store_true",
                    help="time with the golden harness's canonical-order shim and event observers (default: the "
                         "reference's own code paths, nothing wrapped)")
    args = ap.parse_args()
    ref = G.import_reference()
    rec = G.Recorder()
    if args.shim:
        G.install_shims(ref, rec)
    sc = dict(G.SCENARIOS["c3_4096"])
    n = sc["n"]
    ref.field.SIZE_INCREASE_PER_PLAYER = 75
    params = G.make_params(ref, n, sc["virus"], sc["split"], sc["eject"])
    model = ref.model.Model(False, False, params)
    G.tracemalloc.stop()
    for i in range(n):
        model.createPlayer("P%d" % i)
    t0 = time.perf_counter()
    field = G.load_world(ref, rec, model, os.path.join(ROOT, args.world))
    load_s = time.perf_counter() - t0
    np.random.seed(1234)
    bots = [ref.bot.Bot(p, field, "NN", None, params) for p in field.players]
    rng = np.random.default_rng(1234)
    L = params.STATE_REPR_LEN

    def step():
        t_a = time.perf_counter()
        G.bench_commands(field, bots, rng, sc)
        t_b = time.perf_counter()
        field.update()
        t_c = time.perf_counter()
        for b in bots:
            b.getStateRepresentation()
        t_d = time.perf_counter()
        return t_b - t_a, t_c - t_b, t_d - t_c

    step()  # warm-up
    pol, tick, obs = [], [], []
    for _ in range(args.steps):
        a, b, c = step()
        pol.append(a)
        tick.append(b)
        obs.append(c)
    per_step = float(np.mean(np.array(pol) + np.array(tick) + np.array(obs)))
    out = {
        "value": n / per_step, "unit": "env-steps/s", "cores": 1, "kind": "reference",
        "workload": "c3: %s loaded into the reference (4096 bots, field 4800, 100k pellets, 1152 viruses, "
                    "split + eject), bench.py's random policy via Bot.set_command_point (p_split 2.5e-3, "
                    "p_eject 1e-2), Field.update + getStateRepresentation (L = %d) for every bot" % (args.world, L),
        "sample": "%d timed steps after 1 warm-up step%s" % (
            args.steps, ", golden harness shims installed" if args.shim else ", reference code unwrapped"),
        "ms_per_step": per_step * 1e3,
        "ms_policy": float(np.mean(pol)) * 1e3, "ms_field_update": float(np.mean(tick)) * 1e3,
        "ms_observe_all_bots": float(np.mean(obs)) * 1e3,
        "tick_only_env_steps_per_s": n / float(np.mean(tick)),
        "host": {"cpu": cpu_model(), "os_cpu_count": os.cpu_count(), "python": platform.python_version(),
                 "numpy": np.__version__, "where": "build container (the reference cannot travel to the GPU box)"},
        "load_s": load_s,
        "script": "tools/golden/ref_cpu_bench.py",
    }
    path = os.path.join(ROOT, "profiles", "%s_ref_python_c3.json" % args.tag)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
