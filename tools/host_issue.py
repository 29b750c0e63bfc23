"""Host-side issue cost of the bench step (diagnostic): wall time to enqueue K steps without
synchronising vs the synchronised wall time, plus a cProfile of the enqueue loop.

python tools/host_issue.py [--steps 30]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "residual-td3-robot-navigation_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    from nav.trainer import VecTrainer
    tr = VecTrainer(n_envs=65536, hidden=256, n_hidden=2, batch=32768, updates_per_step=2,
                    envs_per_group=1024, device="cuda:0")
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("host issue %.1f us/step, wall %.1f us/step" % (1e6 * (t1 - t0) / args.steps,
                                                         1e6 * (t2 - t0) / args.steps))
    # host queued far ahead: a long GPU sleep first
    torch.cuda._sleep(400_000_000)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print("behind a GPU sleep: host issue %.1f us/step" % (1e6 * (t1 - t0) / args.steps))
    pr = cProfile.Profile()
    torch.cuda._sleep(400_000_000)
    pr.enable()
    for _ in range(10):
        tr.step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
