"""TEST INFRASTRUCTURE ONLY — the CPU port of bench.py's workload (the `cpu_baseline` leg).

Same per-vector-step work as nav.trainer.VecTrainer, restated on the host: actor forward on torch
CPU fp32 + the act epilogue, the fused env/agent tick from the C oracle (OpenMP over envs, each
group with its demonstration set and the same exact bucketed demo index as the GPU tick), then
`updates` TD3 epochs of the oracle learner (torch CPU). Timed on a bounded number of vector steps
by bench.py; never part of the product path. `single_env_rates` times the reference's single-env
loop pieces on one core.
"""
import ctypes as C
import time

import numpy as np
import torch

from . import oracle as O
from .td3_oracle import TD3Oracle, make_mlp_params


class CPUPort:
    def __init__(self, n_envs, hidden, n_hidden, batch, updates, envs_per_group, seed, speed,
                 angle, demo_pts, demo_off):
        self.n, self.B, self.updates, self.epg = n_envs, batch, updates, envs_per_group
        self.p = O.default_params(seed)
        self.speed = np.ascontiguousarray(speed, np.float32)
        self.angle = np.ascontiguousarray(angle, np.float32)
        self.st = O.VecAgentState(n_envs)
        for e in range(n_envs):
            r, g, _ = O.vec_init_one(self.p, e // envs_per_group)
            self.st.region[e] = r
            self.st.goal[e] = g
        self.st.state[:] = self.st.region[:, [0, 2]] + 0.5 * (self.st.region[:, [1, 3]] -
                                                              self.st.region[:, [0, 2]])
        self.st.plan_index[:] = 5
        self.st.path_length[:] = 50
        self.st.episodes[:] = 5
        self.st.noise_scale[:] = 1.0
        self.st.meta[:] = 4
        self.demo_pts = np.ascontiguousarray(demo_pts, np.float64)
        self.demo_off = np.asarray(demo_off, np.int64)
        # the same exact bucketed demo index the GPU tick uses (O.DemoIndexCPU == brute force,
        # tests/test_oracle_golden.py), one per group
        self.index = [O.DemoIndexCPU(self.demo_pts[self.demo_off[g]:self.demo_off[g + 1]])
                      for g in range(len(self.demo_off) - 1)]
        sizes = lambda di, do: [di] + [hidden] * n_hidden + [do]  # noqa: E731
        self.td3 = TD3Oracle(make_mlp_params(seed, sizes(2, 2), 0.0),
                             make_mlp_params(seed + 1, sizes(4, 1), 0.0),
                             make_mlp_params(seed + 2, sizes(4, 1), 0.0))
        self.cap = max(4 * n_envs, 2 * batch)
        self.rows = np.zeros((self.cap, 8), np.float32)
        self.pos = 0
        self.size = 0
        self.rng = np.random.default_rng(seed)

    def step(self):
        st = self.st
        # act (robot.py:541-569)
        b = st.state - st.goal
        with torch.no_grad():
            res = self.td3.actor.forward(torch.from_numpy(b.astype(np.float32))).numpy()
        z = self.rng.standard_normal((self.n, 2))
        a = np.clip(b + res + (st.noise_scale * 5.0)[:, None] * z, -5.0, 5.0)
        a = np.ascontiguousarray(a)
        ns = np.zeros((self.n, 2))
        L = O.lib()
        G = (self.n + self.epg - 1) // self.epg
        for g in range(G):
            lo, hi = g * self.epg, min(self.n, (g + 1) * self.epg)
            d0, d1 = self.demo_off[g], self.demo_off[g + 1]
            f = lambda arr, t, k=1: arr[lo:].ctypes.data_as(t)  # noqa: E731
            L.orc_vec_agent_step_batch(
                C.byref(self.p), O.ptr(self.speed, O._fp), O.ptr(self.angle, O._fp),
                self.demo_pts[d0:].ctypes.data_as(O._dp), d1 - d0, hi - lo,
                f(st.state, O._dp), f(st.goal, O._dp), f(st.region, O._dp), f(st.hist, O._dp),
                f(st.meta, O._u32p), f(st.plan_index, O._i32p), f(st.path_length, O._i32p),
                f(st.episodes, O._i32p), f(st.noise_scale, O._dp), a[lo:].ctypes.data_as(O._dp),
                ns[lo:].ctypes.data_as(O._dp), O.ptr(self.rows, O._fp), self.cap,
                (self.pos + lo) % self.cap, lo, O.ptr(self.index[g].start, O._i64p),
                O.ptr(self.index[g].cand, O._i32p))
        self.pos = (self.pos + self.n) % self.cap
        self.size = min(self.size + self.n, self.cap)
        # TD3 epochs (robot.py:272-285) on batches with replacement
        if self.size >= self.B:
            for u in range(self.updates):
                i = self.rng.integers(0, self.size, self.B)
                r = self.rows[i]
                batch = (r[:, 0:2], r[:, 2:4], r[:, 4], r[:, 5:7], r[:, 7] > 0.5)
                self.td3.train_critic(batch, self.rng.standard_normal((self.B, 2)).astype(
                    np.float32))
                if u % 2 == 0:
                    j = self.rng.integers(0, self.size, self.B)
                    self.td3.train_actor(self.rows[j, 0:2])
                    self.td3.soft_update()


def time_port(port, budget_s=15.0, max_steps=8):
    """Warm one step, then time whole vector steps until the budget is used."""
    port.step()
    t0 = time.perf_counter()
    k = 0
    while k < max_steps:
        port.step()
        k += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return k, dt


def single_env_rates(speed, angle, demo_pts, seconds=2.0):
    """One env on one core: Environment.step alone (environment.py:122-127) and the
    whole per-step agent tick (step + process_transition with the demo term through the index +
    episode control + replay push), the C restatement looping inside one call, env-steps/s."""
    p = O.default_params()
    sp = np.ascontiguousarray(speed, np.float32)
    an = np.ascontiguousarray(angle, np.float32)
    demo = np.ascontiguousarray(demo_pts, np.float64)
    ix = O.DemoIndexCPU(demo)
    acts = np.ascontiguousarray(np.random.default_rng(3).uniform(-5, 5, (4096, 2)))
    out = {}
    for name, tick in (("env_step_per_s", 0), ("agent_tick_per_s", 1)):
        K, dt = 1 << 14, 0.0
        while True:
            t0 = time.perf_counter()
            O.lib().orc_single_env_run(C.byref(p), O.ptr(sp, O._fp), O.ptr(an, O._fp),
                                       O.ptr(demo, O._dp), len(demo), O.ptr(ix.start, O._i64p),
                                       O.ptr(ix.cand, O._i32p), O.ptr(acts, O._dp), len(acts), K,
                                       tick)
            dt = time.perf_counter() - t0
            if dt > seconds / 4 or K > (1 << 30):
                break
            K *= 4
        out[name] = K / dt
    return out
