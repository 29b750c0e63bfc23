"""Host cost of the shared-policy learner path (BASELINE config 5) on one GPU (tuning probe).

At 8 ranks each rank runs 65 536 envs and samples B / 8 = 4 096 rows per epoch, so the device
epoch is short and the host's issue of the learner launches can dominate. This times the bench
step (one collect + 2 TD3 epochs, UTD 1) at rank batch 4 096 with an in-process hook that carries
world_size = 8 but moves no data (the collective itself is not timed: it is the driver's 8-GPU
run), against the hook-free learner at the same batch, interleaved, on one box. "hook_overlap" adds
overlap_collect=True (the next collect on a second stream beside the last epoch's all-reduce and
critic Adam step), which here has no collective to hide and shows the cross-stream cost alone.

python tools/shared_policy_host.py [--batch 4096] [--steps 200] [--rounds 3]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "residual-td3-robot-navigation_amd"))

import torch  # noqa: E402


class IdentityHook:
    """grad_hook contract (nav.dist.GradAllReduce) without the collective."""

    def __init__(self, world_size):
        self.world_size = int(world_size)
        self.calls = 0

    def __call__(self, bucket):
        self.calls += 1


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    args = ap.parse_args()
    from nav.trainer import VecTrainer
    arms = {
        "no_hook": VecTrainer(n_envs=65536, batch=args.batch, updates_per_step=2,
                              envs_per_group=1024),
        "hook": VecTrainer(n_envs=65536, batch=args.batch, updates_per_step=2,
                           envs_per_group=1024, grad_hook=IdentityHook(args.world)),
        "hook_overlap": VecTrainer(n_envs=65536, batch=args.batch, updates_per_step=2,
                                   envs_per_group=1024, grad_hook=IdentityHook(args.world),
                                   overlap_collect=True),
    }
    for tr in arms.values():
        for _ in range(10):
            tr.step()
    torch.cuda.synchronize()
    res = {k: [] for k in arms}
    for _ in range(args.rounds):
        for k, tr in arms.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.step()
            torch.cuda.synchronize()
            res[k].append(1e3 * (time.perf_counter() - t0) / args.steps)
    best = {k: min(v) for k, v in res.items()}
    out = {"batch": args.batch, "world_size_carried": args.world, "steps": args.steps,
           "ms_per_step": res, "best_ms": best,
           "hook_overhead": best["hook"] / best["no_hook"] - 1.0,
           "hook_overlap_overhead": best["hook_overlap"] / best["no_hook"] - 1.0,
           "hook_calls": arms["hook"].td3.grad_hook.calls}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
