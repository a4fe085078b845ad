"""Replica (weak-scaling) plumbing for multi-GPU runs: one process per GPU,
each stepping its own independent arenas; no collective in the data path
(DESIGN.md §7).  torch.distributed is only used for the barrier around the
timed region and the max-over-ranks of its duration ("nccl" = RCCL on a GPU
node, "gloo" in the CPU tests)."""
import os


def world_from_env():
    """(rank, world_size, local_rank) as set by torch.distributed.run."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend):
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group(backend, init_method="env://")
    return dist


def rank_seed(seed, rank):
    """Distinct, reproducible world seed per replica."""
    return int(seed) + 7919 * int(rank)


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, value, device=None):
    """MAX of a float over all ranks (the job's wall time is its slowest replica)."""
    if dist is None:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_throughput(units_per_rank, world, elapsed_max):
    """Whole-job rate: every rank's units over the slowest rank's time."""
    return units_per_rank * world / elapsed_max
