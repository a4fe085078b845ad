"""world_size-2 gloo run of the C4 exchange layer (aigar_amd/tiles.py) on CPU:
the fixed-size tile messages (header, 32-byte records, final-cell bitmap)
all-gathered with the same collective the GPU path runs over RCCL, and the
merge of the tiles' event logs into the reference's global order (eat events
ordered by the eater's priority -- player, cell list position -- then by the
food's turn, whichever tile owned the eater)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


TCAP, BMW = 16, 8  # records per message, bitmap words (512 cells)
PH_PELLET, PH_PP = 3, 5


def _message(rank):
    from aigar_amd import tiles
    r = np.zeros(3, tiles.TILE_REC)
    r[0] = (tiles.TR_PELLET, 0, 1000 + rank, 20.5 + rank, 40.25)  # a pellet kill (seq, position)
    r[1] = (tiles.TR_BLOB, 7 + rank, 500 + rank, 0.0, 0.0)        # a blob kill (slot, seq)
    r[2] = (tiles.TR_CELL, 64 * rank + 3, 10 + rank, 12.5, 1.99)   # an owned cell's outcome (mass, radius)
    return tiles.pack_message(r, undone=rank, tcap=TCAP, bm_words=BMW, final_cells=[64 * rank + 3, 300 + rank])


def _log(rank):
    """raw event rows (key_hi = tick << 8 | phase, key_lo = order, code, a, b): tile 0
    logs the replicated phases, each tile the eat events of the cells it owns."""
    rows = []
    tick = 7
    for prio in ((0, 2) if rank == 0 else (1, 3)):  # players 0, 2 on tile 0; 1, 3 on tile 1
        for t in range(2):
            rows.append(((tick << 8) | PH_PELLET, (prio * 16 << 16) | t, 6, 100 + prio, 1000 + 10 * prio + t))
    if rank == 0:
        rows.append(((tick << 8) | PH_PP, 5, 8, 1, 2))
        rows.append(((tick << 8) | 0, 1, 1, 3, 4))  # a merge, phase 0
    return np.array(rows, np.int64)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from aigar_amd import tiles
    dist.init_process_group("gloo", rank=rank, world_size=world)
    msg = _message(rank)
    tr = tiles.TorchTransport(len(msg), world, "cpu")
    tr.outbox.copy_(torch.from_numpy(msg.copy()))
    tr.exchange()
    inbox = tr.inbox.numpy()
    got = [tiles.unpack_message(inbox[k * len(msg):(k + 1) * len(msg)], TCAP, BMW) for k in range(world)]
    logs = [None] * world
    dist.all_gather_object(logs, _log(rank))
    merged = tiles.merge_events(logs)
    q.put((rank, [(g[0], g[1].tolist(), g[2].tolist()) for g in got], merged.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_tile_exchange():
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
    from aigar_amd import tiles
    for rank, got, merged in out:
        for k, (hdr, recs, final) in enumerate(got):  # slot k of every inbox is tile k's message
            h2, r2, f2 = tiles.unpack_message(_message(k), TCAP, BMW)
            assert hdr == h2 == {"records": 3, "undone": k, "pellet_kills": 1}
            assert recs == r2.tolist() and final == f2.tolist() == [64 * k + 3, 300 + k]
        # merged log: the merge first (phase 0), then the eat events by eater priority 0,1,2,3
        # interleaved across the two tiles, then playerPlayerOverlap
        assert merged[0] == [7, 1, 3, 4]
        eaters = [row[2] for row in merged[1:9]]
        assert eaters == [100, 100, 101, 101, 102, 102, 103, 103]
        assert [row[3] for row in merged[1:9]] == [1000, 1001, 1010, 1011, 1020, 1021, 1030, 1031]
        assert merged[9] == [7, 8, 1, 2]
    assert out[0][2] == out[1][2]  # every rank merges to the same log
