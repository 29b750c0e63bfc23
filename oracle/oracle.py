"""TEST INFRASTRUCTURE ONLY — ctypes view of the C restatement in oracle/nav_oracle.c.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module. It is the
parity checker for the HIP path, never part of it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORC_LIB: another build of the same restatement (make asan-test: the sanitized one)
LIB_PATH = os.environ.get("ORC_LIB") or os.path.join(HERE, "liborc.so")

_dp = C.POINTER(C.c_double)
_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int)
_i32p = C.POINTER(C.c_int32)
_u32p = C.POINTER(C.c_uint32)
_i64p = C.POINTER(C.c_int64)


class Params(C.Structure):
    _fields_ = [
        ("world_size", C.c_double), ("max_action", C.c_double), ("init_region_size", C.c_double),
        ("goal_threshold", C.c_double), ("goal_reward", C.c_double),
        ("stuck_threshold", C.c_double), ("stuck_penalty", C.c_double),
        ("demo_factor", C.c_double), ("noise_decay", C.c_double),
        ("path_length0", C.c_int32), ("path_increase", C.c_int32),
        ("seed_lo", C.c_uint32), ("seed_hi", C.c_uint32), ("max_goal_draws", C.c_int32),
    ]


def build():
    """Compile liborc.so (gcc, seconds). Building the checker is not using it."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_mt_sizeof.restype = C.c_size_t
        L.orc_mt_next32.restype = C.c_uint32
        L.orc_mt_double.restype = C.c_double
        L.orc_mt_gauss.restype = C.c_double
        L.orc_mt_randint.restype = C.c_int64
        L.orc_mt_randint.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
        L.orc_mt_permutation.argtypes = [C.c_void_p, C.c_int64, _i64p]
        L.orc_mt_seed.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_u01.restype = C.c_double
        L.orc_u01.argtypes = [C.c_uint32, C.c_uint32]
        L.orc_philox.argtypes = [_u32p, _u32p, _u32p]
        L.orc_dynamics.argtypes = [_fp, _fp, _dp, _dp, _dp]
        L.orc_step.argtypes = [_fp, _fp, _dp, _dp]
        L.orc_step.restype = C.c_int
        L.orc_reset_u.argtypes = [_dp, C.c_double, C.c_double, _dp]
        L.orc_init_and_goal_mt.argtypes = [C.c_void_p, _dp, _dp, _ip]
        L.orc_init_and_goal_mt.restype = C.c_int
        L.orc_reset_mt.argtypes = [C.c_void_p, _dp, _dp]
        L.orc_norm2.restype = C.c_double
        L.orc_norm2.argtypes = [C.c_double, C.c_double]
        L.orc_demo_min.restype = C.c_double
        L.orc_demo_min.argtypes = [_dp, C.c_int64, C.c_double, C.c_double]
        L.orc_compute_reward.restype = C.c_double
        L.orc_compute_reward.argtypes = [_dp, _dp, _dp, C.c_int64, C.c_int, _ip, C.c_double,
                                         C.c_double, C.c_double]
        L.orc_check_if_stuck.restype = C.c_int
        L.orc_check_if_stuck.argtypes = [_dp, _ip, _ip, _dp, C.c_double]
        L.orc_default_params.argtypes = [C.POINTER(Params)]
        L.orc_vec_init_one.restype = C.c_int
        L.orc_vec_init_one.argtypes = [C.POINTER(Params), C.c_uint32, _dp, _dp]
        L.orc_vec_reset_one.argtypes = [C.POINTER(Params), C.c_uint32, C.c_uint32, _dp, _dp]
        L.orc_vec_noise_one.argtypes = [C.POINTER(Params), C.c_uint32, C.c_uint32, _dp]
        L.orc_vec_agent_tick.restype = C.c_int
        L.orc_vec_agent_tick.argtypes = [C.POINTER(Params), _fp, _fp, _dp, C.c_int64, C.c_uint32,
                                         _dp, _dp, _dp, _dp, _u32p, _i32p, _i32p, _i32p, _dp, _dp,
                                         _dp, _fp, _dp, _dp]
        L.orc_act_epilogue.argtypes = [_dp, _dp, _fp, C.c_double, _dp, C.c_double, _dp]
        L.orc_threads.restype = C.c_int
        L.orc_set_threads.restype = None
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_vec_agent_step_batch.argtypes = [C.POINTER(Params), _fp, _fp, _dp, C.c_int64,
                                               C.c_int64, _dp, _dp, _dp, _dp, _u32p, _i32p, _i32p,
                                               _i32p, _dp, _dp, _dp, _fp, C.c_int64, C.c_int64,
                                               C.c_int64, _i64p, _i32p]
        L.orc_demo_index_res.restype = C.c_int32
        L.orc_demo_index_build.restype = C.c_int64
        L.orc_demo_index_build.argtypes = [_dp, C.c_int64, _i64p, _i32p, C.c_int64]
        L.orc_single_env_run.restype = C.c_double
        L.orc_single_env_run.argtypes = [C.POINTER(Params), _fp, _fp, _dp, C.c_int64, _i64p,
                                         _i32p, _dp, C.c_int64, C.c_int64, C.c_int]
        L.orc_demo_min_idx.restype = C.c_double
        L.orc_demo_min_idx.argtypes = [_dp, C.c_int64, _i64p, _i32p, C.c_double, C.c_double]
        _lib = L
    return _lib


def ptr(a, t):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be C-contiguous"
    return a.ctypes.data_as(t)


class DemoIndexCPU:
    """orc_demo_index_build over one demo set (the CPU port's counterpart of nav's DemoIndex)."""

    def __init__(self, demo):
        self.demo = np.ascontiguousarray(demo, np.float64).reshape(-1, 2)
        m = len(self.demo)
        side = 100 * int(lib().orc_demo_index_res())
        self.start = np.zeros(side * side + 1, np.int64)
        total = lib().orc_demo_index_build(ptr(self.demo, _dp), m, ptr(self.start, _i64p), None, 0)
        self.cand = np.zeros(max(total, 1), np.int32)
        lib().orc_demo_index_build(ptr(self.demo, _dp), m, ptr(self.start, _i64p),
                                   ptr(self.cand, _i32p), total)
        self.total = total

    def min(self, x, y):
        return lib().orc_demo_min_idx(ptr(self.demo, _dp), len(self.demo), ptr(self.start, _i64p),
                                      ptr(self.cand, _i32p), x, y)


def default_params(seed=1707366464):
    p = Params()
    lib().orc_default_params(C.byref(p))
    p.seed_lo = seed & 0xFFFFFFFF
    p.seed_hi = (seed >> 32) & 0xFFFFFFFF
    return p


class LegacyRandomState:
    """numpy RandomState(seed) restated in C: the reference's RNG."""

    def __init__(self, seed):
        self._buf = C.create_string_buffer(lib().orc_mt_sizeof())
        lib().orc_mt_seed(self._buf, seed)

    def next32(self):
        return lib().orc_mt_next32(self._buf)

    def random_sample(self):
        return lib().orc_mt_double(self._buf)

    def gauss(self):
        return lib().orc_mt_gauss(self._buf)

    def randint(self, low, high):
        return lib().orc_mt_randint(self._buf, low, high)

    def permutation(self, n):
        out = np.empty(n, np.int64)
        lib().orc_mt_permutation(self._buf, n, ptr(out, _i64p))
        return out

    def init_and_goal(self):
        region = np.zeros(4); goal = np.zeros(2); side = C.c_int(0)
        draws = lib().orc_init_and_goal_mt(self._buf, ptr(region, _dp), ptr(goal, _dp),
                                           C.byref(side))
        return region, goal, side.value, draws

    def reset(self, region):
        out = np.zeros(2)
        lib().orc_reset_mt(self._buf, ptr(np.ascontiguousarray(region, np.float64), _dp),
                           ptr(out, _dp))
        return out


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr); k = (C.c_uint32 * 2)(*key); o = (C.c_uint32 * 4)()
    lib().orc_philox(c, k, o)
    return list(o)


def dynamics(speed, angle, s, a):
    speed = np.ascontiguousarray(speed, np.float32); angle = np.ascontiguousarray(angle, np.float32)
    s = np.ascontiguousarray(s, np.float64); a = np.ascontiguousarray(a, np.float64)
    out = np.zeros(2)
    lib().orc_dynamics(ptr(speed, _fp), ptr(angle, _fp), ptr(s, _dp), ptr(a, _dp), ptr(out, _dp))
    return out


def step(speed, angle, s, a):
    speed = np.ascontiguousarray(speed, np.float32); angle = np.ascontiguousarray(angle, np.float32)
    s = np.array(s, np.float64); a = np.ascontiguousarray(a, np.float64)
    ok = lib().orc_step(ptr(speed, _fp), ptr(angle, _fp), ptr(s, _dp), ptr(a, _dp))
    return s, ok


def reset_u(region, u0, u1):
    out = np.zeros(2)
    lib().orc_reset_u(ptr(np.ascontiguousarray(region, np.float64), _dp), u0, u1, ptr(out, _dp))
    return out


def norm2(a0, a1):
    return lib().orc_norm2(a0, a1)


def demo_min(demo, x, y):
    demo = np.ascontiguousarray(demo, np.float64).reshape(-1, 2)
    return lib().orc_demo_min(ptr(demo, _dp), len(demo), x, y)


def compute_reward(next_state, goal, demo, demo_flag, goal_thr=5.0, goal_reward=50.0,
                   demo_factor=10.0):
    demo = np.ascontiguousarray(demo, np.float64).reshape(-1, 2)
    gr = C.c_int(0)
    r = lib().orc_compute_reward(ptr(np.ascontiguousarray(next_state, np.float64), _dp),
                                 ptr(np.ascontiguousarray(goal, np.float64), _dp),
                                 ptr(demo, _dp) if len(demo) else None, len(demo), int(demo_flag),
                                 C.byref(gr), goal_thr, goal_reward, demo_factor)
    return r, bool(gr.value)


class StuckHistory:
    def __init__(self):
        self.hist = np.zeros((5, 2)); self.count = C.c_int(0); self.head = C.c_int(0)

    def check(self, s, thr=2.0):
        return bool(lib().orc_check_if_stuck(ptr(self.hist, _dp), C.byref(self.count),
                                             C.byref(self.head),
                                             ptr(np.ascontiguousarray(s, np.float64), _dp), thr))


def vec_init_one(p, sid):
    region = np.zeros(4); goal = np.zeros(2)
    k = lib().orc_vec_init_one(C.byref(p), sid, ptr(region, _dp), ptr(goal, _dp))
    return region, goal, k


def vec_reset_one(p, env, ep, region):
    out = np.zeros(2)
    lib().orc_vec_reset_one(C.byref(p), env, ep, ptr(np.ascontiguousarray(region, np.float64), _dp),
                            ptr(out, _dp))
    return out


def vec_noise_one(p, env, step):
    z = np.zeros(2)
    lib().orc_vec_noise_one(C.byref(p), env, step, ptr(z, _dp))
    return z


def act_epilogue(s, g, residual, sigma, z, max_action=5.0):
    out = np.zeros(2)
    lib().orc_act_epilogue(ptr(np.ascontiguousarray(s, np.float64), _dp),
                           ptr(np.ascontiguousarray(g, np.float64), _dp),
                           ptr(np.ascontiguousarray(residual, np.float32), _fp), sigma,
                           None if z is None else ptr(np.ascontiguousarray(z, np.float64), _dp),
                           max_action, ptr(out, _dp))
    return out


class VecAgentState:
    """Host-side SoA mirror of the device per-env state (oracle layout: hist env-major)."""

    def __init__(self, n):
        self.n = n
        self.state = np.zeros((n, 2)); self.goal = np.zeros((n, 2)); self.region = np.zeros((n, 4))
        self.hist = np.zeros((n, 5, 2)); self.meta = np.zeros(n, np.uint32)
        self.plan_index = np.zeros(n, np.int32); self.path_length = np.zeros(n, np.int32)
        self.episodes = np.zeros(n, np.int32); self.noise_scale = np.zeros(n)

    def tick(self, p, speed, angle, demo, e, action, reset_state=None):
        demo = np.ascontiguousarray(demo, np.float64).reshape(-1, 2)
        ns = np.zeros(2); row = np.zeros(8, np.float32); r = C.c_double(0)
        a = np.ascontiguousarray(action, np.float64)
        rs = None if reset_state is None else np.ascontiguousarray(reset_state, np.float64)
        V = lambda arr, t: arr[e:].ctypes.data_as(t)  # noqa: E731
        flags = lib().orc_vec_agent_tick(
            C.byref(p), ptr(np.ascontiguousarray(speed, np.float32), _fp),
            ptr(np.ascontiguousarray(angle, np.float32), _fp),
            ptr(demo, _dp) if len(demo) else None, len(demo), e,
            V(self.state, _dp), V(self.goal, _dp), V(self.region, _dp), V(self.hist, _dp),
            V(self.meta, _u32p), V(self.plan_index, _i32p), V(self.path_length, _i32p),
            V(self.episodes, _i32p), V(self.noise_scale, _dp), ptr(a, _dp), ptr(ns, _dp),
            ptr(row, _fp), C.byref(r), None if rs is None else ptr(rs, _dp))
        return flags, ns, row, r.value

    def step_batch(self, p, speed, angle, demo, action, rows, base, env0=0):
        demo = np.ascontiguousarray(demo, np.float64).reshape(-1, 2)
        ns = np.zeros((self.n, 2))
        lib().orc_vec_agent_step_batch(
            C.byref(p), ptr(speed, _fp), ptr(angle, _fp), ptr(demo, _dp) if len(demo) else None,
            len(demo), self.n, ptr(self.state, _dp), ptr(self.goal, _dp), ptr(self.region, _dp),
            ptr(self.hist, _dp), ptr(self.meta, _u32p), ptr(self.plan_index, _i32p),
            ptr(self.path_length, _i32p), ptr(self.episodes, _i32p), ptr(self.noise_scale, _dp),
            ptr(np.ascontiguousarray(action, np.float64), _dp), ptr(ns, _dp), ptr(rows, _fp),
            rows.shape[0], base, env0)
        return ns
