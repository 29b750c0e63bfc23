"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL on ROCm = "nccl";
gloo on CPU for tests).

Envs are independent, so the vectorised path shards as independent env blocks (seed + rank) with
no data-path collective. A shared policy (BASELINE config 5) adds exactly one collective: the
all-reduce of each flat gradient buffer before the (redundant, bit-identical) optimizer steps.
"""
import os

import torch
import torch.distributed as dist


def env_info():
    """(world_size, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_seed(base_seed, rank):
    """Independent env block of `rank`: Philox key = base seed + rank (bench config 4)."""
    return int(base_seed) + int(rank)


def make_grad_hook(world_size, group=None):
    """Shared-policy gradient averaging: sum over ranks (RCCL ring over xGMI for GPU tensors),
    then / world_size. Deterministic reduction order per backend, identical on every rank."""
    if world_size <= 1:
        return None

    def hook(g):
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
        g.div_(world_size)

    return hook


def broadcast_params(tensors, src=0, group=None):
    """Same initial policy on every rank."""
    for t in tensors:
        dist.broadcast(t, src, group=group)


def max_over_ranks(value, device):
    """Max of a float over ranks (the bench's timed-region wall time)."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()
