"""nav — MI355X-native residual-TD3 robot navigation (benmcclusky/Residual-TD3-Robot-Navigation's
hot path): the vectorised Environment / Robot tick and the TD3 learner as gfx950 HIP kernels in
libnavenv.so (C-ABI: include/navenv.h), with the reference's Python API on top.

    from nav import Environment, Robot          # drop-ins for environment.py / robot.py
    from nav import VecEnv, VecTrainer, TD3     # the vectorised GPU path
"""
from . import config  # noqa: F401

__all__ = ["Environment", "Robot", "VecEnv", "VecTrainer", "TD3", "DeviceMLP", "ReplayRing"]


def __getattr__(name):
    # lazy: importing `nav` must not require a GPU (CPU tests import submodules)
    if name in ("VecEnv", "ReplayRing", "make_field"):
        from . import vec_env
        return getattr(vec_env, name)
    if name == "VecTrainer":
        from .trainer import VecTrainer
        return VecTrainer
    if name == "TD3":
        from .td3 import TD3
        return TD3
    if name == "DeviceMLP":
        from .mlp import DeviceMLP
        return DeviceMLP
    if name == "Environment":
        from .environment import Environment
        return Environment
    if name == "Robot":
        from .robot import Robot
        return Robot
    raise AttributeError(name)
