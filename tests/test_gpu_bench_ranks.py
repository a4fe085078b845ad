"""bench.py's N > 1 path with real steppers: two ranks launched the way the
driver launches them (torch.distributed.run, one process per rank), here
sharing the one GPU over the gloo backend (RCCL cannot put two ranks on one
device).  Checks rank 0's JSON line: value = one C3 arena tiled 2 x 1 (C4,
messages all-gathered between the ranks, each bot observed by one tile), and
the replica aggregation in the "replicas" side line.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("launch", ["torchrun", "plain"])
def test_two_rank_bench_line(launch):
    """`torchrun`: the driver's launch; `plain`: `python bench.py --gpus 2`, which
    starts torch.distributed.run itself as a child process."""
    steps = 10
    env = dict(os.environ, AIGAR_DIST_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    tail = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", "3",
            "--no-cpu-baseline", "--no-pixels", "--batched-arenas", "0"]
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + tail
    else:
        cmd = [sys.executable] + tail
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == "tiles2x1"
    # value = the metric's world: ONE 4096-bot arena tiled over the 2 ranks
    assert d["value"] == pytest.approx(4096 * steps / (d["ms_per_step"] * steps / 1e3), rel=1e-6)
    assert d["world"]["alive_bots"] > 4000 and d["world"]["pellets"] > 99000
    rep = d["replicas"]  # side line: both replicas' bots over the max-over-ranks time
    assert rep["scaling"] == "weak"
    assert rep["value"] == pytest.approx(2 * 4096 * steps / (rep["ms_per_step"] * steps / 1e3), rel=1e-6)
    c4 = d["c4"]
    assert c4["scaling"] == "strong" and "tiled 2x1" in c4["workload"]
    assert c4["eat_passes_per_tick"] >= 1 and c4["exchange"]["bytes_per_rank_first_pass"] > 0
    assert c4["value"] > 0 and c4["exchange"]["avg_ms"] > 0
    assert c4["exchange"]["process_group_ranks"] == 2 and c4["exchange"]["rccl_ranks"] == 0  # (gloo: no RCCL)
    # the observation is divided: each tile observed part of the bots, together all the live ones
    obs = [t["bots_observed"] for t in c4["per_tile"]]
    assert len(obs) == 2 and min(obs) > 0 and 4000 < sum(obs) <= 4096, obs
