"""world_size-2 gloo run of the replica plumbing bench.py uses for --gpus N."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from aigar_amd import replicas
    r, w, lr = replicas.world_from_env()
    dist = replicas.init("gloo")
    replicas.barrier(dist)
    elapsed = 1.0 + r  # rank 1 is the slow replica
    t = replicas.max_over_ranks(dist, elapsed)
    q.put((r, w, lr, replicas.rank_seed(1234, r), t, replicas.job_throughput(4096 * 10, w, t)))
    replicas.barrier(dist)
    dist.destroy_process_group()


def test_two_rank_gloo_replicas():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[0] for o in out] == [0, 1] and all(o[1] == 2 for o in out)
    assert out[0][3] != out[1][3]                       # distinct replica worlds
    assert all(o[4] == 2.0 for o in out)                # max over ranks
    assert all(o[5] == pytest.approx(4096 * 10 * 2 / 2.0) for o in out)
