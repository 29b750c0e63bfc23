"""ctypes binding of libnavenv.so (include/navenv.h) — the only way this package computes.

Loaded after `import torch` so the library binds torch's already-loaded HIP runtime
(libamdhip64.so.7, same SONAME as /opt/rocm's). There is no fallback: if the library is missing or
a call fails, an exception is raised.
"""
import ctypes as C
import os

import torch  # noqa: F401  (must be loaded first: provides the HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnavenv.so")
_lib_path = LIB_PATH
NAV_EINVAL = -100000
ABI_VERSION = 11

_dp = C.POINTER(C.c_double)
_vp = C.c_void_p


class NavParams(C.Structure):
    _fields_ = [
        ("world_size", C.c_double), ("max_action", C.c_double), ("init_region_size", C.c_double),
        ("goal_threshold", C.c_double), ("goal_reward", C.c_double),
        ("stuck_threshold", C.c_double), ("stuck_penalty", C.c_double),
        ("demo_factor", C.c_double), ("noise_decay", C.c_double),
        ("path_length0", C.c_int32), ("path_increase", C.c_int32),
        ("seed_lo", C.c_uint32), ("seed_hi", C.c_uint32), ("max_goal_draws", C.c_int32),
    ]


class NavEnvSoa(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("state", _vp), ("goal", _vp), ("region", _vp), ("hist", _vp),
        ("meta", _vp), ("plan_index", _vp), ("path_length", _vp), ("episodes", _vp),
        ("noise_scale", _vp),
    ]


class NavStepOut(C.Structure):
    _fields_ = [("next_state", _vp), ("goal_term", _vp), ("flags", _vp), ("block_stats", _vp)]


class NavReplay(C.Structure):
    _fields_ = [("rows", _vp), ("capacity", C.c_int64)]


class NavMlp(C.Structure):
    _fields_ = [
        ("d_in", C.c_int32), ("d_out", C.c_int32), ("hidden", C.c_int32),
        ("hidden_pad", C.c_int32), ("n_hidden", C.c_int32), ("params", _vp), ("packed", _vp),
    ]


# (name, restype, argtypes) for every entry point of include/navenv.h
_P = C.POINTER
SIGNATURES = [
    ("nav_abi_version", C.c_int, []),
    ("nav_default_params", None, [_P(NavParams)]),
    ("nav_mlp_param_count", C.c_int64, [C.c_int32] * 4),
    ("nav_mlp_packed_count", C.c_int64, [C.c_int32] * 2),
    ("nav_mlp_layer_offsets", C.c_int, [_P(NavMlp), C.c_int32, _P(C.c_int64), _P(C.c_int64)]),
    ("nav_env_init", C.c_int, [_P(NavParams), _P(NavEnvSoa), C.c_int32, C.c_int32, _vp, _vp]),
    ("nav_env_reset", C.c_int, [_P(NavParams), _P(NavEnvSoa), _vp, _vp, _vp]),
    ("nav_env_step", C.c_int, [_P(NavParams), _P(NavEnvSoa), _vp, _vp, _vp, _vp]),
    ("nav_dynamics", C.c_int, [_vp, _vp, _vp, _vp, C.c_int64, _vp]),
    ("nav_env_step_k", C.c_int, [_P(NavParams), _P(NavEnvSoa), _vp, _vp, C.c_int32, _vp, _vp]),
    ("nav_agent_step", C.c_int, [_P(NavParams), _P(NavEnvSoa), _vp, _vp, _P(NavReplay),
                                 C.c_int64, _P(NavStepOut), C.c_int32, _vp]),
    ("nav_demo_reward", C.c_int, [_P(NavParams), C.c_int64, _vp, _vp, _vp, _vp, _vp, C.c_int64,
                                  C.c_int32, _P(NavReplay), C.c_int64, _vp, _vp, _vp]),
    ("nav_transition", C.c_int, [_P(NavParams), _P(NavEnvSoa), _vp, _vp, _vp, _P(NavReplay),
                                 C.c_int64, _P(NavStepOut), C.c_int32, _vp]),
    ("nav_check_if_stuck", C.c_int, [_P(NavParams), _P(NavEnvSoa), _vp, _vp, _vp]),
    ("nav_rollout", C.c_int, [_vp, C.c_int64, C.c_int32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("nav_cem_rollout", C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp,
                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("nav_cem_elite", C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp, _vp,
                                _vp, _vp]),
    ("nav_replay_push", C.c_int, [_P(NavReplay), C.c_int64, C.c_int64, _vp, _vp, _vp, _vp, _vp,
                                  _vp]),
    ("nav_demo_index_plan", C.c_int, [_vp, _vp, C.c_int32, C.c_int64, _vp, _vp, _vp]),
    ("nav_demo_index_scan", C.c_int, [_vp, C.c_int32, _vp, _vp]),
    ("nav_demo_index_fill", C.c_int, [_vp, _vp, C.c_int32, C.c_int64, _vp, _vp, _vp, _vp]),
    ("nav_demo_index_res", C.c_int32, []),
    ("nav_fields_generate", C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    ("nav_demo_augment", C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp,
                                   _vp]),
    ("nav_demo_index_subplan", C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, _vp, _vp, _vp]),
    ("nav_demo_index_subscan", C.c_int, [_vp, C.c_int32, _vp, _vp]),
    ("nav_demo_index_subfill", C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("nav_demo_reward_indexed", C.c_int, [_P(NavParams), C.c_int64, _vp, _vp, _vp, _vp, _vp,
                                          C.c_int32, _vp, _vp, _P(NavReplay), C.c_int64, _vp,
                                          _vp, _vp]),
    ("nav_agent_step_indexed", C.c_int, [_P(NavParams), _P(NavEnvSoa), _vp, _vp, _P(NavReplay),
                                         C.c_int64, _P(NavStepOut), _vp, _vp, C.c_int32, _vp,
                                         _vp, _vp, _vp]),
    ("nav_demo_min", C.c_int, [_vp, C.c_int64, _vp, C.c_int64, _vp, _vp]),
    ("nav_compute_reward", C.c_int, [_P(NavParams), C.c_int64, _vp, _vp, _vp, C.c_int64,
                                     C.c_int32, _vp, _vp, _vp]),
    ("nav_act", C.c_int, [_P(NavParams), _P(NavMlp), C.c_int64, _vp, _vp, _vp, _vp, C.c_uint32,
                          C.c_int32, _vp, _vp, _vp]),
    ("nav_act_tick", C.c_int, [_P(NavParams), _P(NavMlp), _P(NavEnvSoa), _vp, _vp, C.c_uint32,
                               C.c_int32, _P(NavReplay), C.c_int64, _P(NavStepOut), _vp, _vp,
                               C.c_int32, _vp, _vp, _vp, _vp, _vp]),
    ("nav_mlp_forward", C.c_int, [_P(NavMlp), C.c_int32, C.c_int64, _vp, C.c_int32, C.c_int32,
                                  _P(_vp), C.c_int32, C.c_int32, C.c_int32, _vp, C.c_float,
                                  C.c_float, C.c_float, C.c_uint32, C.c_uint32, C.c_uint32,
                                  _P(_vp), C.c_uint32, _P(_vp), _vp]),
    ("nav_td3_critic_rows", C.c_int, [_P(NavMlp), _P(NavMlp), _P(NavMlp), _P(NavReplay),
                                      C.c_int64, C.c_int64, _vp, C.c_uint32, C.c_uint32,
                                      C.c_uint32, _vp, C.c_float, C.c_float, C.c_float, C.c_float,
                                      _vp, _P(_vp), _P(_vp), _P(_vp), _P(_vp), C.c_uint32,
                                      _P(_vp), C.c_int32, _P(_vp), C.c_uint32, C.c_int32,
                                      _vp]),
    ("nav_td3_actor_rows", C.c_int, [_P(NavMlp), _P(NavMlp), _P(NavReplay), C.c_int64,
                                     C.c_int64, _vp, C.c_uint32, C.c_uint32, C.c_uint32, _vp,
                                     _vp, _vp, _vp, C.c_uint32, _vp, C.c_uint32, _vp, _vp, _vp,
                                     _vp]),
    ("nav_mlp_mask_count", C.c_int64, [C.c_int32, C.c_int32, C.c_int64]),
    ("nav_mlp_row_blocks", C.c_int64, [C.c_int64]),
    ("nav_mlp_edge_count", C.c_int64, [C.c_int32] * 4),
    ("nav_mlp_hidden_count", C.c_int64, [C.c_int32] * 2),
    ("nav_td3_critic_forward", C.c_int, [_P(NavMlp), C.c_int64, _vp, C.c_int32, C.c_int32, _vp,
                                         _vp, _vp, C.c_float, _P(_vp), _P(_vp), _P(_vp),
                                         _P(_vp), C.c_uint32, _P(_vp), _vp]),
    ("nav_mlp_backward", C.c_int, [_P(NavMlp), C.c_int32, C.c_int64, _P(_vp), C.c_int32, _P(_vp),
                                   _vp, C.c_int32, C.c_int32, _P(_vp), _P(_vp), C.c_uint32,
                                   _P(_vp), _P(_vp), _vp]),
    ("nav_mlp_wgrad", C.c_int, [_P(NavMlp), C.c_int32, C.c_int64, _vp, C.c_int32, C.c_int32,
                                _P(_vp), _P(_vp), _P(_vp), C.c_int32, _P(_vp), _P(_vp), C.c_int32,
                                _vp]),
    ("nav_mlp_wgrad_splits", C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                          C.c_int64]),
    ("nav_grad_reduce", C.c_int, [_P(NavMlp), _vp, C.c_int32, _vp, C.c_int64, _vp, _vp]),
    ("nav_grad_reduce_adam", C.c_int, [_P(NavMlp), C.c_int32, _P(_vp), C.c_int32, _P(_vp),
                                       C.c_int64, _P(_vp), _P(_vp), _P(_vp), C.c_float, C.c_float,
                                       C.c_float, _P(C.c_float), _P(C.c_float), _vp]),
    ("nav_grad_reduce_adam_polyak", C.c_int,
     [_P(NavMlp), C.c_int32, _P(_vp), C.c_int32, _P(_vp), C.c_int64, _P(_vp), _P(_vp), _P(_vp),
      C.c_float, C.c_float, C.c_float, _P(C.c_float), _P(C.c_float), _P(NavMlp), _P(NavMlp),
      _P(NavMlp), C.c_int32, C.c_float, _vp]),
    ("nav_grad_reduce_multi", C.c_int, [_P(NavMlp), C.c_int32, _P(_vp), C.c_int32, _P(_vp),
                                        C.c_int64, _P(_vp), _vp]),
    ("nav_adam_multi", C.c_int, [_P(NavMlp), C.c_int32, _P(_vp), _P(_vp), _P(_vp), C.c_float,
                                 C.c_float, C.c_float, _P(C.c_float), _P(C.c_float), C.c_float,
                                 _vp]),
    ("nav_adam_polyak_multi", C.c_int, [_P(NavMlp), C.c_int32, _P(_vp), _P(_vp), _P(_vp),
                                        C.c_float, C.c_float, C.c_float, _P(C.c_float),
                                        _P(C.c_float), C.c_float, _P(NavMlp), _P(NavMlp),
                                        _P(NavMlp), C.c_int32, C.c_float, _vp]),
    ("nav_adam", C.c_int, [_P(NavMlp), _vp, _vp, _vp, C.c_float, C.c_float, C.c_float,
                           C.c_float, C.c_float, _vp]),
    ("nav_polyak", C.c_int, [_P(NavMlp), _P(NavMlp), C.c_float, _vp]),
    ("nav_polyak_multi", C.c_int, [_P(NavMlp), _P(NavMlp), C.c_int32, C.c_float, _vp]),
    ("nav_mlp_pack", C.c_int, [_P(NavMlp), _vp]),
    ("nav_replay_sample", C.c_int, [_P(NavReplay), C.c_int64, C.c_int64, _vp, C.c_uint32,
                                    C.c_uint32, C.c_uint32, _vp, _vp]),
    ("nav_fill", C.c_int, [_vp, C.c_int64, C.c_float, _vp]),
    ("nav_strided_copy", C.c_int, [_vp, C.c_int32, C.c_int32, _vp, C.c_int32, C.c_int32,
                                   C.c_int64, C.c_int32, _vp]),
    ("nav_event_create", C.c_int, [_P(_vp)]),
    ("nav_event_destroy", C.c_int, [_vp]),
    ("nav_event_record", C.c_int, [_vp, _vp]),
    ("nav_event_elapsed_ms", C.c_int, [_vp, _vp, _P(C.c_float)]),
]

# Entry points that return int64 counts (negative = error) rather than a status code.
_COUNT_FNS = {"nav_mlp_param_count", "nav_mlp_packed_count", "nav_mlp_mask_count",
              "nav_mlp_row_blocks", "nav_mlp_edge_count", "nav_mlp_hidden_count",
              "nav_mlp_wgrad_splits", "nav_demo_index_res"}


class NavError(RuntimeError):
    pass


class _Checked:
    def __init__(self, name, fn):
        self.name, self.fn = name, fn

    def __call__(self, *args):
        r = self.fn(*args)
        if self.name in _COUNT_FNS:
            if r < 0:
                raise NavError(f"{self.name}: invalid argument")
        elif self.fn.restype is C.c_int and r != 0 and self.name != "nav_abi_version":
            what = "invalid argument" if r == NAV_EINVAL else f"HIP error {-r}"
            raise NavError(f"{self.name} failed: {what}")
        return r


class _Lib:
    def __init__(self, path):
        if not os.path.exists(path):
            raise NavError(f"{path} is missing: build it with `make -C "
                           f"residual-td3-robot-navigation_amd` (or __graft_entry__.build())")
        self.raw = C.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(self.raw, name)
            fn.restype = res
            fn.argtypes = args
            setattr(self, name, _Checked(name, fn))
        v = self.nav_abi_version()
        if v != ABI_VERSION:
            raise NavError(f"libnavenv ABI {v} != {ABI_VERSION}")


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _Lib(_lib_path)
    return _lib


def lib_path():
    """The library this process binds (libnavenv.so next to this file unless a tuning tool chose
    another build through use_library)."""
    return _lib_path


def use_library(path):
    """Bind another build of the same ABI instead of the in-tree libnavenv.so. For the A/B timing
    tools only (tools/withlib.py); must run before the first call into the library."""
    global _lib_path
    path = os.path.abspath(path)
    if _lib is not None and path != _lib_path:
        raise NavError(f"libnavenv is already loaded from {_lib_path}")
    _lib_path = path


def require_gpu():
    if not torch.cuda.is_available():
        raise NavError("nav needs a ROCm GPU (MI355X); no HIP device is visible")


def ptr(t):
    """Device pointer of a contiguous tensor (or None)."""
    if t is None:
        return None
    assert t.is_contiguous(), "nav tensors must be contiguous"
    return C.c_void_p(t.data_ptr())


def parr(*tensors):
    """C array of device pointers (None entries allowed) for the pointer-array parameters."""
    return (C.c_void_p * len(tensors))(*[None if t is None else t.data_ptr() for t in tensors])


def descs(*nets):
    """C array of nav_mlp descriptors."""
    return (NavMlp * len(nets))(*[n.desc() for n in nets])


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def params_struct(**kw):
    p = NavParams()
    lib().nav_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p
