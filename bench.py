#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the agar.io stepper (BASELINE.json metric).

One step = one synthetic-population policy pass + Field.update() for the
whole arena + the grid observation for every bot.
env-steps = bots x steps.  Default workload = BASELINE.json configs[2] (C3):
4096 bots, 100k pellets, 1152 viruses, split + eject on, field 4800, on one
MI355X, started from the matured tick-50 world of data/c3_t50.npz (the
survey's warm distribution: mean cell mass 17.4, max ~54; tools/mature.py).
For N > 1 (launched by torch.distributed.run, one rank per GPU) `value` is the
metric's own world: ONE C3 arena (4096 bots x 100k pellets) tiled 2-D over the
N ranks (BASELINE configs[3], C4: each rank one tile, the tiles' eat-phase
messages and observation-history hand-offs all-gathered over RCCL / xGMI, each
bot observed by one tile; strong scaling, no host round trip per tick).  The
timed region is bracketed by barrier + synchronize and the max over ranks is
taken.  Beside it, "replicas" times every rank stepping its own C3 arena
(independent replicas, weak scaling, no collective in the data path).

The timed steps are issued with aigar_run: each step (policy + tick +
observation) is one hipGraph replay.  The per-phase breakdown and the roofline
kernel's duration come from the following steps issued as separate calls.

Prints ONE JSON line (rank 0).  Extra objects: "roofline" for the dominant
kernel (k_observe, HIP-event timed live on the stepper's stream) and
"cpu_baseline" (the C oracle, i.e. a single-thread CPU port of the reference,
timed on a bounded sample of the same workload on this host).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from aigar_amd import _abi, replicas  # noqa: E402

# the reference's own Python src/model on THIS workload (bench.py's start world and policy,
# Field.update + the observation of every bot, one core), timed in the build container by
# tools/golden/ref_cpu_bench.py: the reference itself cannot travel to the GPU box, so its
# committed figure is quoted beside the C-port baseline
def reference_python(workload):
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_ref_python_%s.json" % workload)))
    if not files:
        return None
    d = json.load(open(files[-1]))
    keep = ("value", "unit", "cores", "kind", "workload", "sample", "ms_per_step", "ms_field_update",
            "ms_observe_all_bots", "host")
    out = {k: d[k] for k in keep if k in d}
    out["source"] = os.path.relpath(files[-1], ROOT)
    return out


SNAPSHOTS = {"c3": "c3_t50"}  # matured start worlds (tools/mature.py)
# The c3_t50 world was matured by Greedy bots (the survey's warm distribution);
# under the random policy its first ~25 ticks carry ~3x the steady
# playerPlayerOverlap work while the Greedy clusters scatter
# (profiles/r04_v32_early_steps.txt: k_spawn_plan 36 -> 16 -> 10 us over steps
# 0-5, 15-25, 25+).  The random population therefore first plays this many
# untimed ticks from the snapshot -- part of setting up the world, like the load
# -- so that warm-up and timed steps run its steady state whatever --warmup is.
SETTLE_TICKS = 30

# C3 observation config: VIRUS_SPAWN + ENABLE_SPLIT (networkParameters.py:76-96)
C3_CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
         | _abi.OBS_ENEMY_LF)
C3_EX = _abi.EX_LAST_FOV | _abi.EX_FOV | _abi.EX_MASS | _abi.EX_LAST_ACT

MULTI_CH = _abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY
WORKLOADS = {
    # name: (bots per arena, field, pellets, virus, p_split, p_eject, channels, extras, arenas per GPU)
    "c3": (4096, 4800, 100000.0, True, 2.5e-3, 1e-2, C3_CH, C3_EX, 1),
    "c2": (256, 1200, 10000.0, False, 0.0, 0.0, MULTI_CH, _abi.EX_FOV | _abi.EX_MASS, 1),
    # C5: 64 arenas x 512 bots over 8 GPUs = 8 arenas per GPU
    "c5": (512, 1697, 43200.0, False, 0.0, 0.0, MULTI_CH, _abi.EX_FOV | _abi.EX_MASS, 8),
}


def make_cfg(name, device=0, flags=0, arenas=None):
    bots, field, pellets, virus, _, _, ch, ex, arenas0 = WORKLOADS[name]
    arenas = arenas0 if arenas is None else arenas
    c = _abi.Config()
    c.n_arenas, c.bots_per_arena, c.field_size = arenas, bots, field
    c.virus_enabled = int(virus)
    c.max_pellets, c.max_viruses = pellets, -1.0
    c.grid_squares, c.obs_channels, c.obs_extras = 11, ch, ex
    c.rng_mode, c.device, c.flags = _abi.RNG_PHILOX, device, flags
    return c


def obs_bytes_per_bot(L, p_fov, c_fov, v_fov, n_cells=1.2):
    """Algorithmic HBM bytes k_observe moves per bot:
    own cells (x, y, m, r + list slot), visible pellet records (x, y, m, seq = 32 B),
    visible cells (x, y, m, r, flags = 36 B), viruses (x, y, m, r, seq, flags = 44 B),
    history grids read+write (2 x 2 x 121 x 8 B), output row (L x 8 B)."""
    return n_cells * 33 + p_fov * 32 + c_fov * 36 + v_fov * 44 + 2 * 2 * 121 * 8 + L * 8


def pmc_traffic(kernel_prefix, workload):
    """HBM-side bytes per launch of the kernel (kernel_prefix "_step": per env
    step, all the step's kernels) from the newest committed PMC summary
    (profiles/r*_pmc_<workload>.json, written by tools/gpu.sh TAG pmc +
    tools/pmc_summary.py on the same bench command).  None if absent."""
    import glob
    import re

    def version(f):  # profiles/r01_v18_pmc_c3.json -> (1, 18): numeric, not lexicographic
        m = re.search(r"r(\d+)_v(\d+)_pmc", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_%s.json" % workload)), key=version)
    if not files:
        return None, None
    data = json.load(open(files[-1]))
    for k, v in data.items():
        if kernel_prefix in k and "traffic_bytes" in v:
            return float(v["traffic_bytes"]), os.path.relpath(files[-1], ROOT)
    return None, None


def cpu_baseline(name, budget_s=12.0, seed=1, policy="random"):
    """Single-thread C oracle (CPU port of the reference) on the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle  # test infrastructure: the checker / CPU baseline only
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = WORKLOADS[name]
    bots *= arenas
    cfg = make_cfg(name, flags=0)
    o = Oracle(cfg)
    o.reset(seed)
    rng = np.random.default_rng(seed)
    start = "reset(%d)" % seed
    snap = SNAPSHOTS.get(name)
    path = os.path.join(ROOT, "data", "%s.npz" % snap) if snap else None
    if path and os.path.exists(path) and arenas == 1:  # the GPU line's start world (start_world)
        z = np.load(path)
        o.load_state({k: z[k] for k in z.files})
        start = "data/%s.npz" % snap

    def commands():
        st = o.player_stats()
        cmd = np.zeros((bots, 4))
        fx, fy, fs = st[:, 2], st[:, 3], st[:, 4]
        ok = st[:, 0] > 0
        x, y = np.trunc(np.nan_to_num(fx)), np.trunc(np.nan_to_num(fy))
        half, size = np.trunc(np.nan_to_num(fs) / 2), np.trunc(np.nan_to_num(fs))
        cmd[:, 0] = np.where(ok, x - half + rng.random(bots) * size, -1)
        cmd[:, 1] = np.where(ok, y - half + rng.random(bots) * size, -1)
        cmd[:, 2] = rng.random(bots) < ps
        cmd[:, 3] = rng.random(bots) < pe
        return cmd

    def act():
        if policy == "greedy":
            o.policy_greedy(True)
        else:
            o.set_commands(commands())

    if policy == "random" and snap and start != "reset(%d)" % seed:
        for _ in range(SETTLE_TICKS):  # (untimed, as the GPU line: the random population settles)
            act()
            o.step(1)
        start += " + %d untimed random-policy ticks" % SETTLE_TICKS
    for _ in range(2):  # warm-up
        act()
        o.step(1)
        o.observe()
    n, t0 = 0, time.perf_counter()
    while True:
        act()
        o.step(1)
        o.observe()
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    o.close()
    return {"value": bots * n / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": "%s world from %s, %d steps (%s policy + Field.update + obs for all %d bots) after 2 warm-up "
                      "steps, oracle/oracle.c single thread, %.1f s" % (name.upper(), start, n, policy, bots, dt)}


def _c5_arena_worker(args):
    """One process of the C5 CPU baseline: a 512-bot arena stepped by the oracle."""
    seed, budget_s = args
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle
    bots, field, pellets, virus, ps, pe, ch, ex, _ = WORKLOADS["c5"]
    o = Oracle(make_cfg("c5", arenas=1))
    o.reset(seed)
    rng = np.random.default_rng(seed)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        cmd = np.zeros((bots, 4))
        cmd[:, 0] = rng.random(bots) * field
        cmd[:, 1] = rng.random(bots) * field
        o.set_commands(cmd)
        o.step(1)
        o.observe()
        n += 1
    dt = time.perf_counter() - t0
    o.close()
    return bots * n, dt


def cpu_baseline_c5(budget_s=12.0):
    """SURVEY.md §8d C5 CPU baseline: min(64, cores) processes, one 512-bot arena
    each (the reference's own mp.Pool pattern, aigar.py:549), aggregate env-steps/s."""
    import multiprocessing as mp
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    nproc = max(1, min(64, cores, 16))  # (the GPU box grants 16 CPUs per GPU)
    with mp.get_context("spawn").Pool(nproc) as pool:
        res = pool.map(_c5_arena_worker, [(1000 + k, budget_s) for k in range(nproc)])
    rate = sum(u / dt for u, dt in res)
    return {"value": rate, "unit": "env-steps/s", "cores": nproc, "kind": "port",
            "sample": "C5: %d processes x one 512-bot arena (field 1697, 43,200 pellets), random commands + "
                      "Field.update + obs, oracle/oracle.c, %.0f s each" % (nproc, budget_s)}


def batched(name, arenas, policy, ps, pe, seed, device, steps=20, warmup=5):
    """The same per-arena workload, `arenas` independent arenas stepped by the
    same launches (batched-env mode, SURVEY.md §8e C5 pattern): what one MI355X
    sustains when it is given enough work to fill it.  Reported beside `value`."""
    import torch
    from aigar_amd import _lib
    bots = WORKLOADS[name][0] * arenas
    stp = _lib.Stepper(make_cfg(name, device=device, arenas=arenas))
    stp.set_stream(torch.cuda.current_stream().cuda_stream)
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    start = start_world(stp, name, seed + 1, arenas)
    run = lambda n: stp.run(n, policy, obs, p_split=ps, p_eject=pe, seed=seed, greedy_split=True)
    run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # k_observe over all arenas' bots in one launch: its roofline at this size
    stp.profile(True)
    for _ in range(10):
        stp.observe(obs)
    torch.cuda.synchronize()
    obs_ms, obs_n = stp.kernel_time("observe")
    stp.profile(False)
    stp.sync()
    per_bot, reads_bot, alive = obs_bytes(stp, WORKLOADS[name][1], arenas)
    obs_s = obs_ms / max(1, obs_n) / 1e3
    stp.close()
    return {"arenas": arenas, "bots": bots, "value": bots * steps / dt, "unit": "env-steps/s",
            "ms_per_step": dt / steps * 1e3, "steps": steps, "start": start,
            "roofline_k_observe": {"bytes_per_launch": int(per_bot * alive), "avg_launch_ms": obs_s * 1e3,
                                   "achieved": round(per_bot * alive / obs_s / 1e9, 2), "peak": 8000.0,
                                   "unit": "GB/s", "frac": per_bot * alive / obs_s / 1e9 / 8000.0,
                                   "reads": {"bytes_per_launch": int(reads_bot * alive),
                                             "frac": reads_bot * alive / obs_s / 1e9 / 8000.0}}}


def obs_bytes(stp, field, arenas):
    """Algorithmic bytes of one k_observe launch from the stepper's current
    world: (per alive bot, of which reads, alive bots)."""
    st = stp.get_state()
    stats = stp.player_stats()
    alive = int(np.sum(stats[:, 0] > 0))
    fs = np.nan_to_num(stats[:, 4])
    area = float(np.mean((fs + 2.0) ** 2))  # FOV box incl. object radii
    dens_p = st["n_pellets"] / float(field * field * arenas)
    dens_c = st["n_cells"] / float(field * field * arenas)
    dens_v = st["n_viruses"] / float(field * field * arenas)
    ncell = st["n_cells"] / max(1, alive)
    per_bot = obs_bytes_per_bot(stp.obs_len, dens_p * area, dens_c * area, dens_v * area, n_cells=ncell)
    reads_bot = per_bot - stp.obs_len * 8 - 2 * 121 * 8  # minus the output row and the history writes
    return per_bot, reads_bot, alive


def start_world(stp, name, seed, arenas):
    """Reset, or load the workload's matured snapshot into every arena."""
    snap = SNAPSHOTS.get(name)
    path = os.path.join(ROOT, "data", "%s.npz" % snap) if snap else None
    if path is None or not os.path.exists(path):
        stp.reset(seed)
        return "reset(seed %d)" % seed
    z = np.load(path)
    d = {k: z[k] for k in z.files}
    stp.reset(seed)
    for a in range(arenas):
        stp.load_state(d, a)
    return "data/%s.npz (tick %d, mean cell mass %.2f, max %.1f)" % (
        snap, int(d["tick"]), float(d["cells_f"][:, 2].mean()), float(d["cells_f"][:, 2].max()))


def tick_bytes(st, alive, field, n_eaten):
    """Algorithmic HBM bytes of one Field.update (SURVEY.md §8d formula, fp64
    records): every cell record read and written (88 B), the pellet / enemy-cell
    candidates each cell's overlap tests read (32 B / 88 B, expected counts from
    the densities over the cell's hash box), the eaten and respawned pellet
    records (32 B each), and the cell hash (4 B per bucket + 4 B per cell)."""
    n_c = st["n_cells"]
    if n_c == 0:
        return 0.0
    r = np.sqrt(np.asarray(st["cells_f"])[:, 2] / np.pi)
    box = float(np.mean((2 * r + 20.0) ** 2))
    k_p = st["n_pellets"] / float(field * field) * box
    k_e = n_c / float(field * field) * box
    H = int(np.ceil(field / 20.0)) ** 2
    return 2 * 88 * n_c + n_c * k_p * 32 + n_c * k_e * 88 + 2 * n_eaten * 32 + 4 * H + 4 * n_c


def c4_leg(args, name, rank, world, local, seed, dist, backend):
    """BASELINE configs[3]: ONE C3 arena tiled over the N ranks (aigar_amd/tiles.py),
    each rank one tile.  On the nccl backend (the production path) every step is
    aigar_tile_run: policy + Field.update with the eat-phase messages (and the
    observation-history hand-offs) all-gathered by RCCL over xGMI + the observation
    of this tile's bots, captured as ONE hipGraph per step (no Python, no host round
    trip per tick).  On gloo (the 1-GPU rehearsal: N ranks sharing one card, which
    RCCL cannot do) the exchange goes through TorchTransport, staged through host
    memory.  Strong scaling: the same 4096 bots whatever N.  The passes are
    device-decided: first with no extra pass; if a tick needed one (device error
    bit), the world is reloaded and timed again with one extra gated pass per tick.
    world == 1 (AIGAR_C4_SELFTEST): the whole field as one forced tile over a
    1-rank communicator -- the same code path on the one GPU of a test box."""
    import torch
    from aigar_amd import _lib, tiles
    tx, ty = tiles.tile_grid(world)
    # 512 records per message (the random population's owned outcomes per tick and tile are
    # a few dozen; an overflow is a device error, not a silent loss) and 16 hand-off slots:
    # a 48 KB first-pass message per tile
    cfg = tiles.tile_config(make_cfg(name, device=local, arenas=1), tx, ty, rank, cap=512 if world > 1 else 4096,
                            flags=_abi.TILE_FORCE if world == 1 else 0)
    stp = _lib.Stepper(cfg)
    rccl = backend == "nccl"
    if rccl:
        stp.set_stream(torch.cuda.current_stream().cuda_stream)
        tiles.rccl_comm(stp, dist)
        tr = None
    else:
        tr = tiles.TorchTransport.for_stepper(stp, staged=True)
    bots, field, pellets, virus, ps, pe, ch, ex, _ = WORKLOADS[name]
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    steps, warm = args.steps, args.warmup

    def run(n, extra):
        if rccl:
            stp.tile_run(n, "random", obs, p_split=ps, p_eject=pe, seed=args.seed, extra_passes=extra)
        else:
            for _ in range(n):
                tiles.tiled_tick([stp], tr, "random", ps, pe, args.seed, [obs], extra_passes=extra)

    dev = "cuda" if backend == "nccl" else None
    for extra in (0, 1):
        start = start_world(stp, name, seed, 1)  # every tile loads the same world and keeps its held pellets
        try:
            run(warm, extra)
            torch.cuda.synchronize()
            stp.sync()
            replicas.barrier(dist)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(steps, extra)
            torch.cuda.synchronize()
            replicas.barrier(dist)
            el = time.perf_counter() - t0
            stp.sync()  # raises on a device error (every tile raises alike: the undone count is global)
            break
        except RuntimeError as e:
            if extra == 1 or "device error bits" not in str(e):
                raise
    el = replicas.max_over_ranks(dist, el, device=dev)
    graphed = stp.tile_run_graphed() if rccl else False
    # per-tile breakdown: the next steps as separate launches, HIP events on the tile's stream
    nb = min(steps, 30)
    stp.profile(True)
    if tr is not None:
        tr.reset_timing()
    run(nb, extra)
    torch.cuda.synchronize()
    names = ("tile_begin", "exchange", "tile_apply", "tile_resume", "tile_end", "observe")
    br = {k: stp.kernel_time(k) for k in names}
    stp.profile(False)
    ex_ms = br["exchange"][0] / max(1, br["exchange"][1]) if rccl else tr.avg_exchange_ms()
    stp.sync()
    observed = int(np.sum(stp.tile_observers() == rank))
    info = stp.tile_info()
    stp.close()
    per_tile = {"tile": rank, "bots_observed": observed,
                "ms_per_step": {k: v[0] / nb for k, v in br.items() if v[1]},
                "exchange_ms_per_pass": ex_ms,
                "note": "separate launches with HIP events (the timed steps replay one graph): tile_begin = "
                        "policy + updateViruses .. playerVirusOverlap + the first eat pass and the hand-off plan; "
                        "tile_end = playerPlayerOverlap .. spawnStuff; observe = this tile's bots"}
    tiles_all = [per_tile]
    if dist is not None:
        tiles_all = [None] * world
        dist.all_gather_object(tiles_all, per_tile)
    return {"workload": "C4: one C3 arena (%d bots, %d pellets) tiled %dx%d over %d GPUs, start %s" % (
                bots, int(pellets), tx, ty, world, start),
            "value": bots * steps / el, "unit": "env-steps/s", "scaling": "strong", "steps": steps,
            "ms_per_step": el / steps * 1e3, "eat_passes_per_tick": 1 + extra, "extra_passes": extra,
            "step_graph": graphed,
            "exchange": {"collective": "ncclAllGather inside the step graph (RCCL, xGMI)" if rccl else
                         "all_gather_into_tensor (%s, staged through host memory)" % backend,
                         "rccl_ranks": info["ntiles"] if rccl else 0,  # (the communicator: one rank per tile)
                         "process_group_ranks": world,
                         "bytes_per_rank_first_pass": (1 + info["tcap"]) * 32 + info.get("handoff_bytes", 0),
                         "avg_ms": ex_ms},
            "per_tile": tiles_all}


def launch_ranks(n):
    """`python bench.py --gpus N` (N > 1) outside torch.distributed.run: start the
    N ranks (one process per GPU) the way the driver does, as a CHILD process --
    this process has not touched the GPU and never execs -- with the same
    arguments; rank 0's JSON line reaches stdout through the inherited pipe, and
    the child's exit code is returned (the reference's own multi-process launch is
    an mp.Pool of workers, aigar.py:549-554)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.stdout.flush()
    return subprocess.call(cmd, cwd=ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--arenas", type=int, default=None,
                    help="independent arenas per GPU (default: the workload's own; >1 = batched-env scale sweep)")
    ap.add_argument("--batched-arenas", type=int, default=16,
                    help="also time this many independent arenas of the same workload stepped together on "
                         "the GPU (reported under 'batched', never as 'value'); 0 = skip")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pixels", action="store_true", help="skip the pixel-observation side measurement")
    ap.add_argument("--no-c4", action="store_true",
                    help="N > 1: report the replicas as value instead of the tiled single arena (C4)")
    ap.add_argument("--profile-run", action="store_true",
                    help="only the warm-up and the timed graph replays (for rocprofv3: one call per step)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--policy", default="random", choices=["random", "greedy"],
                    help="synthetic population: Philox random actions, or the reference's Greedy bots "
                         "(bot.py:579-633, ENABLE_GREEDY_SPLIT) on the device")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    import torch
    rank, world, local = replicas.world_from_env()
    if args.gpus != world:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE is %d: launch N > 1 ranks with torch.distributed.run "
                 "(one process per GPU)" % (args.gpus, world))
    dist = None
    # AIGAR_DIST_BACKEND=gloo rehearses the N-rank path with several ranks
    # sharing the GPUs there are (ranks wrap around the visible devices)
    backend = os.environ.get("AIGAR_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:  # one process per GPU, independent replicas (weak scaling)
        dist = replicas.init(backend)
    from aigar_amd import _lib  # raises if libaigar_hip.so is missing: no fallback

    name = args.workload
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = WORKLOADS[name]
    if args.arenas:
        arenas = args.arenas
    bots *= arenas  # players stepped per GPU
    stp = _lib.Stepper(make_cfg(name, device=local, arenas=arenas))
    stream = torch.cuda.current_stream()
    stp.set_stream(stream.cuda_stream)
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    start = start_world(stp, name, replicas.rank_seed(args.seed, rank), arenas)
    salt = args.seed + 7919 * rank  # replicas of one snapshot diverge through their policy draws

    def run(n):  # n whole steps (policy + tick + observation): aigar_run replays its step graph (4 steps per launch)
        stp.run(n, args.policy, obs, p_split=ps, p_eject=pe, seed=salt, greedy_split=True)

    if args.policy == "random" and name in SNAPSHOTS:
        run(SETTLE_TICKS)  # (untimed: the random population settles from the Greedy-matured snapshot)
        start += " + %d untimed random-policy ticks to settle" % SETTLE_TICKS

    def one_step():  # the same step as separate calls, each bracketed by HIP events
        if args.policy == "greedy":
            stp.policy_greedy(True)
        else:
            stp.policy_random(ps, pe, salt)
        stp.step(1)
        stp.observe(obs)

    run(args.warmup)
    torch.cuda.synchronize()
    stp.sync()
    w0 = stp.counters()
    replicas.barrier(dist)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    replicas.barrier(dist)
    t1 = time.perf_counter()
    elapsed = t1 - t0
    stp.sync()  # raises on any device-side capacity error
    elapsed = replicas.max_over_ranks(dist, elapsed, device="cuda" if backend == "nccl" else None)
    value = replicas.job_throughput(bots * args.steps, world, elapsed)
    st = stp.get_state()
    stats = stp.player_stats()
    work = stp.counters()
    ticks_timed = max(1, work["ticks"] - w0["ticks"])
    out = {
        "metric": "env-steps/sec at 4096 bots x 100k pellets; 1/2/4/8 MI355X scaling",
        "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (Philox bot population, %s)" % ("reference Greedy bots on the device" if args.policy == "greedy"
                                                           else "random-action policy"),
        "config": {"workload": "%s: %s%d bots, %d pellets, %s viruses, %s, field %d, obs %d floats/bot; start: %s" % (
            name.upper(), "%d arenas x " % arenas if arenas > 1 else "", bots // arenas, int(pellets),
            "1152" if virus else "no",
            "greedy bots with ENABLE_GREEDY_SPLIT" if args.policy == "greedy" else "split p=%g, eject p=%g" % (ps, pe),
            field, stp.obs_len, start),
                   "policy": args.policy,
                   "parallelism": "replicas%d" % world if world > 1 else "single-gpu"},
    }
    if not args.profile_run:
        # per-phase breakdown and the roofline kernel's duration: the next
        # min(steps, 50) steps issued as separate calls, HIP events on the stepper's stream
        stp.profile(True)
        for _ in range(min(args.steps, 50)):
            one_step()
        torch.cuda.synchronize()
        obs_ms, obs_n = stp.kernel_time("observe")
        tick_ms, tick_n = stp.kernel_time("tick")
        pol_ms, pol_n = stp.kernel_time("policy")
        stp.profile(False)
        stp.sync()
        # roofline of the dominant kernel (k_observe): algorithmic bytes per launch / avg duration
        per_bot, reads_bot, alive = obs_bytes(stp, field, arenas)
        obs_bytes_launch = per_bot * alive
        obs_avg_s = (obs_ms / max(1, obs_n)) / 1e3
        achieved = obs_bytes_launch / obs_avg_s / 1e9
        peak = 8000.0
        traffic, traffic_src = pmc_traffic("k_observe", name)
        step_traffic, step_src = pmc_traffic("_step", name)
        eaten = work["pellets_eaten"] - w0["pellets_eaten"] if "pellets_eaten" in work else 0
        step_bytes = tick_bytes(st, alive, field, eaten / ticks_timed) * arenas + obs_bytes_launch
        out["roofline"] = {
            "bound": "hbm", "kernel": "k_observe", "achieved": round(achieved, 2), "peak": peak, "unit": "GB/s",
            "frac": achieved / peak, "traffic": None if traffic is None else int(traffic),
            "traffic_source": traffic_src, "bytes_per_launch": int(obs_bytes_launch), "avg_launch_ms": obs_avg_s * 1e3,
            "reads": {"bytes_per_launch": int(reads_bot * alive),
                      "frac": reads_bot * alive / obs_avg_s / 1e9 / peak},
            "step": {"bytes_per_step": int(step_bytes), "frac": step_bytes / (elapsed / args.steps) / 1e9 / peak,
                     "traffic": None if step_traffic is None else int(step_traffic), "traffic_source": step_src,
                     "note": "algorithmic bytes of the whole env step (tick + observation) / ms_per_step; "
                             "traffic: PMC bytes of all the step's kernels per step"}}
        out["breakdown_ms_per_step"] = {"policy": pol_ms / max(1, pol_n), "tick": tick_ms / max(1, tick_n),
                                        "observe": obs_ms / max(1, obs_n)}
    out["world"] = {"pellets": st["n_pellets"], "cells": st["n_cells"], "viruses": st["n_viruses"],
                    "blobs": st["n_blobs"], "alive_bots": int(np.sum(stats[:, 0] > 0)), "tick": int(st["tick"]),
                    "mean_cell_mass": float(np.asarray(st["cells_f"])[:, 2].mean()) if st["n_cells"] else 0.0,
                    "multi_cell_players": int(np.sum(np.asarray(st["players_i"])[:, 4] > 1)),
                    "per_tick_in_timed_region": {k: round((work[k] - w0[k]) / ticks_timed, 3) for k in work
                                                 if k != "ticks"}}
    if not args.profile_run and not args.no_pixels:
        # RGBGenerator.get_cnn_inputRGB for every bot (side 42, uint8 RGB): a side line,
        side, reps = 42, 20  # not part of the env-step metric (the reference's CNN pixel mode is off by default)
        frames = torch.empty((bots, side, side, 3), dtype=torch.uint8, device="cuda")
        stp.observe_pixels(side, 0, out=frames)
        stp.profile(True)
        for _ in range(reps):
            stp.observe_pixels(side, 0, out=frames)
        torch.cuda.synchronize()
        pix_ms, pix_n = stp.kernel_time("observe_pixels")
        stp.profile(False)
        stp.sync()
        pix_s = pix_ms / max(1, pix_n) / 1e3
        out["pixels"] = {"side": side, "dtype": "u8 rgb", "frames_per_s": bots / pix_s, "avg_launch_ms": pix_s * 1e3,
                         "output_GB_s": bots * side * side * 3 / pix_s / 1e9}
    stp.close()
    if not args.profile_run and world == 1 and rank == 0:
        if args.batched_arenas > 1 and not args.arenas:
            out["batched"] = batched(name, args.batched_arenas, args.policy, ps, pe, args.seed, local)
        if args.policy == "random" and name == "c3":  # the same start with the reference's Greedy bots
            out["greedy"] = greedy_side(name, args.seed, local)
    if world == 1 and name == "c3" and os.environ.get("AIGAR_C4_SELFTEST") and not args.profile_run:
        # the C4 code path on one GPU: the whole field as one forced tile over a 1-rank RCCL communicator
        out["c4_selftest"] = c4_leg(args, name, rank, world, local, args.seed, dist, "nccl")
    if not args.no_c4 and world > 1 and name == "c3":
        # the metric's world at N GPUs: one 4096-bot arena tiled over them (value);
        # the replicas measured above become the side line
        c4 = c4_leg(args, name, rank, world, local, args.seed, dist, backend)
        out["replicas"] = {"value": out["value"], "ms_per_step": out["ms_per_step"], "scaling": "weak",
                           "workload": "%d independent C3 arenas, one per GPU" % world}
        out["value"], out["ms_per_step"], out["scaling"] = c4["value"], c4["ms_per_step"], "strong"
        out["config"]["workload"] = c4["workload"]
        out["config"]["parallelism"] = "tiles%dx%d" % replicas_tiles(world)
        out["c4"] = c4
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_run:  # (N = 1 only)
        out["cpu_baseline"] = cpu_baseline(name, args.cpu_budget, policy=args.policy)
        if name == "c3" and args.policy == "random":  # (the file times bench.py's random policy)
            ref_py = reference_python(name)
            if ref_py is not None:
                out["cpu_baseline"]["reference_python"] = ref_py
        if name == "c5":
            out["cpu_baseline_processes"] = cpu_baseline_c5(args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def replicas_tiles(world):
    from aigar_amd import tiles
    return tiles.tile_grid(world)


def greedy_side(name, seed, device, steps=30, warmup=5):
    """Side line: the same matured start stepped with the reference's Greedy bots
    (bot.py:579-633, ENABLE_GREEDY_SPLIT) on the device: bots converge on food and
    chase each other, so the serial phases carry real work."""
    import torch
    from aigar_amd import _lib
    stp = _lib.Stepper(make_cfg(name, device=device))
    stp.set_stream(torch.cuda.current_stream().cuda_stream)
    start_world(stp, name, seed, 1)
    bots = WORKLOADS[name][0]
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    stp.run(warmup, "greedy", obs, greedy_split=True)
    torch.cuda.synchronize()
    w0 = stp.counters()
    t0 = time.perf_counter()
    stp.run(steps, "greedy", obs, greedy_split=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stp.sync()
    w1 = stp.counters()
    stp.close()
    n = max(1, w1["ticks"] - w0["ticks"])
    return {"value": bots * steps / dt, "unit": "env-steps/s", "ms_per_step": dt / steps * 1e3, "steps": steps,
            "serial_work_per_tick": {k: round((w1[k] - w0[k]) / n, 3) for k in w1 if k != "ticks"}}


if __name__ == "__main__":
    main()
