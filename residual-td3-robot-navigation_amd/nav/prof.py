"""Per-kernel timing with HIP events on the launch stream, and the algorithmic work counts the
roofline figures use.

`with timing(KernelTimer(...)):` activates a timer; every libnavenv launch site in nav/ wraps its
launch in `region(name, work)`, which records a start/stop event pair on the current stream (the
stream the kernel is launched on) when the timer tracks that name. Nothing is recorded otherwise.
The events are libnavenv's device-scope-release HIP events (nav_event_*): a default HIP event
record costs ~6 us of GPU time (system-scope L2 writeback), which would stretch the timed region.
"""
import contextlib
import ctypes as C
from collections import defaultdict

import torch

# ---- algorithmic bytes per env-step (HBM-bound kernels) ----
# nav_env_step: state r/w (16 + 16) + action (16)
ENV_STEP_BYTES = 48
# nav_agent_step, steady state (history full, no reset): reads state 16, action 16, goal 16,
# meta 4, plan 4, path 4, history 5 x 16 = 80 (140); writes history slot 16, replay row 32,
# state 16, plan 4, meta 4, next_state 16, goal_term 8, flags 1 (97)
AGENT_STEP_BYTES = 237


def env_step_k_bytes(K, with_next):
    """nav_env_step_k per env-step: the action (16), each step's state out (16) if kept, and the
    state read + written once per launch (32 / K)."""
    return 16.0 + (16.0 if with_next else 0.0) + 32.0 / K


def mlp_fwd_flops(d_in, d_out, h, nh, rows):
    return 2.0 * rows * (d_in * h + (nh - 1) * h * h + h * d_out)


def mlp_bwd_flops(d_in, d_out, h, nh, rows, dx=False, edges=False, wo=False):
    """row backward (dy . Wo, (nh-1) hidden GEMMs, dx) plus, with edges, the per-block
    parameter-gradient partials it sums: dW0 (2 d_in h), biases (nh h), dWo (2 d_out h)."""
    f = d_out * h + (nh - 1) * h * h + (h * d_in if dx else 0)
    if edges:
        f += d_in * h + 0.5 * nh * h + (d_out * h if wo else 0)
    return 2.0 * rows * f


def mlp_wgrad_flops(h, nh, rows):
    """hidden x hidden weight gradients only (the edge layers are summed by fwd / bwd)."""
    return 2.0 * rows * (nh - 1) * h * h


def demo_flops(n_env, m):
    # per point: 2 sub, 2 mul, 1 add, 1 min (f64)
    return 6.0 * n_env * m


class KernelTimer:
    """Event pairs around the launches of the named regions (all when names is None). With
    sample_every = n only every n-th launch of each region is bracketed: each event record still
    costs the stream a few microseconds, so the bench's timed region samples its dominant kernel
    instead of stretching every launch; the average per launch is the same kernel's."""

    def __init__(self, names=None, sample_every=1):
        self.names = None if names is None else set(names)
        self.rec = defaultdict(list)
        self.sample_every = max(1, int(sample_every))
        self.seen = defaultdict(int)

    def wants(self, name):
        if self.names is not None and name not in self.names:
            return False
        k = self.seen[name]
        self.seen[name] = k + 1
        return k % self.sample_every == 0

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, lst in self.rec.items():
            ms = [s.elapsed_ms(e) for s, e, _ in lst]
            work = sum(w for _, _, w in lst)
            out[name] = {"launches": len(ms), "total_ms": sum(ms),
                         "avg_us": 1e3 * sum(ms) / len(ms), "work": work,
                         "work_per_launch": work / len(ms)}
        return out


class _Event:
    """A pooled nav_event (hipEventReleaseToDevice), returned to the pool when collected."""
    _pool = []

    def __init__(self):
        from ._lib import lib
        if _Event._pool:
            self.h = _Event._pool.pop()
        else:
            h = C.c_void_p()
            lib().nav_event_create(C.byref(h))
            self.h = h

    def record(self):
        from ._lib import lib, stream_handle
        lib().nav_event_record(self.h, stream_handle())

    def elapsed_ms(self, end):
        from ._lib import lib
        ms = C.c_float()
        lib().nav_event_elapsed_ms(self.h, end.h, C.byref(ms))
        return ms.value

    def __del__(self):
        if getattr(self, "h", None) is not None:
            _Event._pool.append(self.h)
            self.h = None


_active = None


@contextlib.contextmanager
def timing(timer):
    global _active
    prev, _active = _active, timer
    try:
        yield timer
    finally:
        _active = prev


@contextlib.contextmanager
def region(name, work=0.0):
    t = _active
    if t is None or not t.wants(name):
        yield
        return
    s, e = _Event(), _Event()
    s.record()
    try:
        yield
    finally:
        e.record()
        t.rec[name].append((s, e, work))
