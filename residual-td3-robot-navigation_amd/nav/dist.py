"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL on ROCm = "nccl";
gloo on CPU for tests).

Envs are independent, so the vectorised path shards as independent env blocks (seed + rank) with
no data-path collective. A shared policy (BASELINE config 5) adds exactly one collective: the
SUM all-reduce of each flat gradient bucket (twin critics as one bucket per epoch, the actor's on
policy epochs) before the redundant, bit-identical optimizer steps.
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


class GradAllReduce:
    """Shared-policy gradient exchange (BASELINE config 5): ONE in-place SUM all-reduce per flat
    gradient bucket (RCCL over xGMI for GPU tensors, gloo for CPU tensors). The learner divides
    by `world_size` inside its Adam launch (nav_adam_multi's grad_div), as torch DDP's average.
    Every rank receives the same bytes, so the redundant Adam / Polyak steps keep the ranks'
    parameters bit-identical."""

    def __init__(self, world_size, group=None):
        self.world_size = int(world_size)
        self.group = group
        self.calls = 0
        self.bytes = 0

    def __call__(self, bucket):
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=self.group)
        self.calls += 1
        self.bytes += bucket.numel() * bucket.element_size()


def make_grad_hook(world_size, group=None):
    """The learner's grad_hook for a shared policy over `world_size` ranks (None for one)."""
    if world_size <= 1:
        return None
    return GradAllReduce(world_size, group)


def broadcast_params(tensors, src=0, group=None):
    """Same initial policy on every rank."""
    for t in tensors:
        dist.broadcast(t, src, group=group)


def max_over_ranks(value, device):
    """Max of a float over ranks (the bench's timed-region wall time)."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()
