"""Diagnostic (GPU): candidate-list lengths the indexed demo reward walks at the bench config.
Builds the bench trainer (65 536 envs, CEM demo sets), runs some training steps, then reports the
index size, the per-env candidate count at the env's current cell, its per-wave max (a wave runs
as many trips as its longest list), and the tick time with / without the demo pass.

python tools/demo_index_stats.py [steps]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "residual-td3-robot-navigation_amd"))

import torch  # noqa: E402


def main():
    from nav import prof
    from nav.trainer import VecTrainer
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    tr = VecTrainer(n_envs=65536, hidden=256, n_hidden=2, batch=32768, updates_per_step=2,
                    envs_per_group=1024, device="cuda")
    res = {}
    for phase in range(2):
        for _ in range(steps):
            tr.step()
        torch.cuda.synchronize()
        ix = tr.env.demo_index
        st = tr.env.state.cpu()
        g = torch.arange(tr.n) // tr.env.envs_per_group
        k = ix.cell_of(g, st[:, 0].clamp(0, 99.999), st[:, 1].clamp(0, 99.999))
        cs = ix.cell_start.cpu()
        n = (cs[k + 1] - cs[k]).double()
        wave = n.view(-1, 64).max(1).values
        lens = (cs[1:] - cs[:-1]).double()
        t = prof.KernelTimer(["act_tick", "act", "agent_step"])
        with prof.timing(t):
            for form in (True, False):
                tr.fuse_tick = form
                for _ in range(10):
                    tr.collect()
        tr.fuse_tick = True
        s = t.summary()
        res["after_%d_steps" % ((phase + 1) * steps)] = {
            "index_res": ix.res, "index_total": ix.total, "level1_total": ix.total_l1, "mean_per_cell": ix.mean_candidates,
            "cell_len_p50_p90_max": [float(lens.quantile(q)) for q in (0.5, 0.9)] + [float(lens.max())],
            "env_cand_mean": float(n.mean()), "env_cand_p90": float(n.quantile(0.9)),
            "wave_max_mean": float(wave.mean()), "wave_max_p90": float(wave.quantile(0.9)),
            "us": {k2: round(v["avg_us"], 2) for k2, v in s.items()}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
