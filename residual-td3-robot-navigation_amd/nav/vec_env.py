"""Vectorised Environment + Robot per-step state on one GPU (environment.py, robot.py:413-538).

`VecEnv` owns the structure-of-arrays per-env state as torch tensors (device memory) and drives the
gfx950 kernels of libnavenv.so through the C-ABI. One env = one lane; n envs advance per launch.
"""
import ctypes as C

import torch

from . import config as K
from . import prof
from ._lib import (NavEnvSoa, NavReplay, NavStepOut, lib, params_struct, ptr, require_gpu,
                   stream_handle)


def make_field(speed, angle, device="cuda"):
    """Interleave Environment.dynamics_speed / dynamics_angle ([100,100] float32, x-major) into the
    kernels' [100][100][2] table."""
    s = torch.as_tensor(speed, dtype=torch.float32)
    a = torch.as_tensor(angle, dtype=torch.float32)
    assert s.shape == (100, 100) and a.shape == (100, 100)
    return torch.stack([s, a], dim=-1).contiguous().to(device)


class DemoIndex:
    """Exact bucketed nearest-demo index (nav_demo_index_*): per (group, index cell) the list of
    demonstration points that can be nearest to any state in the cell. Two levels: the 1 x 1
    dynamics cells over every point of the group, then R x R index cells per dynamics cell
    (R = nav_demo_index_res()) over their parent's list. `cell_start` / `cand` are the index-cell
    lists the reward kernels walk. The indexed reward equals the brute-force one bit for bit
    (tests/test_gpu_env.py)."""

    L1_CELLS = 100 * 100

    def __init__(self, demo_xy, demo_off=None, stream=None):
        dev = demo_xy.device
        G = 1 if demo_off is None else demo_off.shape[0] - 1
        m = demo_xy.shape[0] if demo_off is None else 0
        s = stream_handle(stream)
        L = lib()
        self.res = int(L.nav_demo_index_res())
        self.side = 100 * self.res
        self.CELLS = self.side * self.side
        # level 1: dynamics cells over all points
        bound1 = torch.zeros(G * self.L1_CELLS, dtype=torch.float64, device=dev)
        count1 = torch.zeros(G * self.L1_CELLS, dtype=torch.int32, device=dev)
        start1 = torch.zeros(G * self.L1_CELLS + 1, dtype=torch.int64, device=dev)
        L.nav_demo_index_plan(ptr(demo_xy), ptr(demo_off), G, m, ptr(bound1), ptr(count1), s)
        L.nav_demo_index_scan(ptr(count1), G, ptr(start1), s)
        total1 = int(start1[-1].item())
        cand1 = torch.zeros(max(total1, 1), dtype=torch.int32, device=dev)
        L.nav_demo_index_fill(ptr(demo_xy), ptr(demo_off), G, m, ptr(bound1), ptr(start1),
                              ptr(cand1), s)
        # level 2: the query index
        bound = torch.zeros(G * self.CELLS, dtype=torch.float64, device=dev)
        count = torch.zeros(G * self.CELLS, dtype=torch.int32, device=dev)
        self.cell_start = torch.zeros(G * self.CELLS + 1, dtype=torch.int64, device=dev)
        L.nav_demo_index_subplan(ptr(demo_xy), ptr(demo_off), G, ptr(start1), ptr(cand1),
                                 ptr(bound), ptr(count), s)
        L.nav_demo_index_subscan(ptr(count), G, ptr(self.cell_start), s)
        total = int(self.cell_start[-1].item())
        self.cand = torch.zeros(max(total, 1), dtype=torch.int32, device=dev)
        L.nav_demo_index_subfill(ptr(demo_xy), ptr(demo_off), G, ptr(start1), ptr(cand1),
                                 ptr(bound), ptr(self.cell_start), ptr(self.cand), s)
        self.total = total
        self.total_l1 = total1
        self.mean_candidates = total / float(G * self.CELLS)

    def cell_of(self, g, x, y):
        """index cell of state (x, y) of group g (torch tensors), as the kernels compute it"""
        return g * self.CELLS + (x * self.res).long() * self.side + (y * self.res).long()


class ReplayRing:
    """ReplayBuffer (robot.py:58-124) as a device ring of 32-byte rows
    (s0 s1 a0 a1 r s'0 s'1 done, float32)."""

    def __init__(self, capacity, device="cuda"):
        self.capacity = int(capacity)
        self.rows = torch.zeros(self.capacity, 8, dtype=torch.float32, device=device)
        self.position = 0  # next write slot (robot.py:77)
        self.size = 0

    def desc(self):
        return NavReplay(self.rows.data_ptr(), self.capacity)

    def advance(self, n):
        base = self.position
        self.position = (self.position + n) % self.capacity
        self.size = min(self.size + n, self.capacity)
        return base

    def __len__(self):
        return self.size


class VecEnv:
    def __init__(self, n, field, seed=K.RANDOM_SEED, envs_per_group=1, demo_flag=True,
                 device="cuda", init=True, fuse_demo=True, **param_overrides):
        require_gpu()
        self.n = int(n)
        self.device = torch.device(device)
        self.field = field
        self.p = params_struct(seed_lo=seed & 0xFFFFFFFF, seed_hi=(seed >> 32) & 0xFFFFFFFF,
                               **param_overrides)
        self.envs_per_group = int(envs_per_group)
        d, n = self.device, self.n
        f64, i32 = torch.float64, torch.int32
        self.state = torch.zeros(n, 2, dtype=f64, device=d)
        self.goal = torch.zeros(n, 2, dtype=f64, device=d)
        self.region = torch.zeros(n, 4, dtype=f64, device=d)
        self.hist = torch.zeros(5, n, 2, dtype=f64, device=d)
        self.meta = torch.zeros(n, dtype=torch.int32, device=d)  # uint32 bits
        self.plan_index = torch.zeros(n, dtype=i32, device=d)
        self.path_length = torch.zeros(n, dtype=i32, device=d)
        self.episodes = torch.zeros(n, dtype=i32, device=d)
        self.noise_scale = torch.zeros(n, dtype=f64, device=d)
        # per-step outputs
        self.next_state = torch.zeros(n, 2, dtype=f64, device=d)
        self.goal_term = torch.zeros(n, dtype=f64, device=d)
        self.flags = torch.zeros(n, dtype=torch.uint8, device=d)
        self.block_stats = torch.zeros((n + 63) // 64, 8, dtype=torch.float32, device=d)
        self.goal_draws = torch.zeros(n, dtype=i32, device=d)
        self.soa = NavEnvSoa(n, *[t.data_ptr() for t in (
            self.state, self.goal, self.region, self.hist, self.meta, self.plan_index,
            self.path_length, self.episodes, self.noise_scale)])
        self.out = NavStepOut(self.next_state.data_ptr(), self.goal_term.data_ptr(),
                              self.flags.data_ptr(), self.block_stats.data_ptr())
        self.demo_xy = None
        self.demo_off = None
        self.demo_index = None
        # demo reward fused into the tick launch (nav_agent_step_indexed); False keeps the two
        # launches (A/B and the fused-vs-unfused parity test)
        self.fuse_demo = bool(fuse_demo)
        if init:
            self.init(demo_flag)

    # environment.py:28-56 + robot.py:413-438 (vectorised, Philox)
    def init(self, demo_flag=True, stream=None):
        lib().nav_env_init(C.byref(self.p), C.byref(self.soa), self.envs_per_group,
                           int(bool(demo_flag)), ptr(self.goal_draws), stream_handle(stream))

    # environment.py:130-137
    def reset(self, mask=None, uniforms=None, stream=None):
        lib().nav_env_reset(C.byref(self.p), C.byref(self.soa), ptr(mask), ptr(uniforms),
                            stream_handle(stream))
        return self.state

    # environment.py:122-127 (pure Environment.step over all envs)
    def step(self, action, next_state=None, stream=None):
        with prof.region("env_step", float(prof.ENV_STEP_BYTES * self.n)):
            lib().nav_env_step(C.byref(self.p), C.byref(self.soa), ptr(self.field), ptr(action),
                               ptr(next_state), stream_handle(stream))
        return self.state

    # environment.py:122-127 applied K times in one launch (state in registers)
    def step_k(self, actions, next_states=None, stream=None):
        K = actions.shape[0]
        assert actions.shape == (K, self.n, 2) and actions.is_contiguous()
        with prof.region("env_step_k", float(prof.env_step_k_bytes(K, next_states is not None)
                                             * self.n)):
            lib().nav_env_step_k(C.byref(self.p), C.byref(self.soa), ptr(self.field),
                                 ptr(actions), K, ptr(next_states), stream_handle(stream))
        return self.state

    def dynamics(self, state, action, out=None, stream=None):
        out = out if out is not None else torch.empty_like(state)
        lib().nav_dynamics(ptr(self.field), ptr(state), ptr(action), ptr(out), state.shape[0],
                           stream_handle(stream))
        return out

    # demonstration set used by the demo-proximity reward (robot.py:749-757)
    def set_demo(self, demo_xy, demo_off=None, index=True):
        self.demo_xy = torch.as_tensor(demo_xy, dtype=torch.float64).reshape(-1, 2).contiguous()
        self.demo_xy = self.demo_xy.to(self.device)
        self.demo_off = None
        if demo_off is not None:
            self.demo_off = torch.as_tensor(demo_off, dtype=torch.int64).to(self.device)
        self.demo_index = DemoIndex(self.demo_xy, self.demo_off) if index else None

    # one fused training tick (robot.py:443-506, 645-675 + environment.py:122-137)
    def agent_step(self, action, replay, stream=None, reward_out=None):
        base = replay.position
        s = stream_handle(stream)
        rd = replay.desc()
        ix = self.demo_index if (self.demo_xy is not None and self.demo_xy.shape[0] > 0) else None
        if ix is not None and self.fuse_demo:
            # one launch: tick + indexed demo reward (bit-identical to the two-launch path)
            with prof.region("agent_step", float(prof.AGENT_STEP_BYTES * self.n)):
                lib().nav_agent_step_indexed(
                    C.byref(self.p), C.byref(self.soa), ptr(self.field), ptr(action), C.byref(rd),
                    base, C.byref(self.out), ptr(self.demo_xy), ptr(self.demo_off),
                    self.envs_per_group, ptr(ix.cell_start), ptr(ix.cand), ptr(reward_out), s)
            replay.advance(self.n)
            return base
        has_demo = self.demo_xy is not None and self.demo_xy.shape[0] > 0
        with prof.region("agent_step", float(prof.AGENT_STEP_BYTES * self.n)):
            lib().nav_agent_step(C.byref(self.p), C.byref(self.soa), ptr(self.field),
                                 ptr(action), C.byref(rd), base, C.byref(self.out),
                                 int(has_demo), s)
        if has_demo:
            m = self.demo_xy.shape[0] if self.demo_off is None else 0
            m_per = self.demo_xy.shape[0] if self.demo_off is None else \
                self.demo_xy.shape[0] / max(1, self.demo_off.shape[0] - 1)
            ix = self.demo_index
            if ix is not None:
                # algorithmic work: the f64 ops over the candidates actually visited
                with prof.region("demo_reward", prof.demo_flops(self.n, ix.mean_candidates)):
                    lib().nav_demo_reward_indexed(
                        C.byref(self.p), self.n, ptr(self.next_state), ptr(self.goal_term),
                        ptr(self.flags), ptr(self.demo_xy), ptr(self.demo_off),
                        self.envs_per_group, ptr(ix.cell_start), ptr(ix.cand), C.byref(rd), base,
                        ptr(reward_out), ptr(self.block_stats), s)
            else:
                with prof.region("demo_reward", prof.demo_flops(self.n, m_per)):
                    lib().nav_demo_reward(C.byref(self.p), self.n, ptr(self.next_state),
                                          ptr(self.goal_term), ptr(self.flags),
                                          ptr(self.demo_xy), ptr(self.demo_off), m,
                                          self.envs_per_group, C.byref(rd), base,
                                          ptr(reward_out), ptr(self.block_stats), s)
        replay.advance(self.n)
        return base

    # robot.py:541-569 + the training tick above, one launch (nav_act_tick): the actor's action
    # epilogue runs each env's tick in the same workgroup
    def act_tick(self, actor, step, replay, training=True, action_out=None, reward_out=None,
                 noise_z=None, stream=None):
        base = replay.position
        rd = replay.desc()
        a = actor.desc()
        ix = self.demo_index if (self.demo_xy is not None and self.demo_xy.shape[0] > 0) else None
        if self.demo_xy is not None and self.demo_xy.shape[0] > 0 and ix is None:
            raise ValueError("act_tick needs the demo index (set_demo(index=True))")
        flops = prof.mlp_fwd_flops(2, 2, actor.hidden, actor.n_hidden, self.n)
        with prof.region("act_tick", flops):
            lib().nav_act_tick(
                C.byref(self.p), C.byref(a), C.byref(self.soa), ptr(self.field), ptr(noise_z),
                int(step) & 0xFFFFFFFF, 0 if training else 1, C.byref(rd), base,
                C.byref(self.out), ptr(self.demo_xy) if ix else None,
                ptr(self.demo_off) if ix else None, self.envs_per_group,
                ptr(ix.cell_start) if ix else None, ptr(ix.cand) if ix else None,
                ptr(action_out), ptr(reward_out), stream_handle(stream))
        replay.advance(self.n)
        return base

    def stats(self):
        """Sum of the per-block rows: reward (the final pushed reward, demo term included, in
        every launch form: the demo-reward launches rewrite the reward column), done, goal,
        stuck, ended."""
        return self.block_stats.sum(0)[:5].tolist()
