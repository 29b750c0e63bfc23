"""Batched CEM demonstrator (environment.py:140-179) for the vectorised trainer's group demo sets.

Every (group, demonstration) is one CEM problem: 4 iterations x 100 paths x 200 steps, the 10 best
paths' action mean / std feeding the next iteration. All problems advance together: one
nav_cem_rollout launch per iteration over every problem's paths, then one nav_cem_elite launch
(device top-10, float32 mean / std, argmax). The random draws are the reference's numpy draws, made
on the host from each group's own RandomState in the order robot-learning.py's demo ticks make
them (start state, CEM actions, then the demonstration's augmentation noise, demo after demo), so
each plan equals nav.Environment.get_demonstration's on the same stream (tests/test_gpu_cem.py).
Elite order: ascending reward, ties by path index; np.argsort orders exact ties
platform-dependently (x86-simd-sort), so plans with tied elite rewards are the one case not pinned.
"""
import ctypes as C

import numpy as np
import torch

from . import config as K
from ._lib import lib, ptr, stream_handle
from .demos import augment_draws, demo_set_from


def group_stream_draws(rng, T=K.DEMOS_CEM_PATH_LENGTH, P=K.DEMOS_CEM_NUM_PATHS,
                       I=K.DEMOS_CEM_NUM_ITERATIONS, n_demos=K.NUM_DEMO):
    """Consume one group's numpy stream as its robot-learning.py demo ticks would: per demo the
    start uniforms (environment.py:136), iteration 0's np.random.choice([-5, 5]) actions and the
    later iterations' standard normals (environment.py:157-159; a size-(P,T,2) draw is the same
    stream as the reference's per-step draws), then process_demonstration's augmentation normals
    (robot.py:802-815). Returns per demo (uniforms [2], a0 [P,T,2] f64, z [I-1,P,T,2] f64,
    augmentation draws)."""
    out = []
    for _ in range(n_demos):
        u = rng.random_sample(2)
        a0 = rng.choice([-K.ROBOT_MAX_ACTION, K.ROBOT_MAX_ACTION], (P, T, 2)).astype(np.float64)
        z = np.stack([rng.standard_normal((P, T, 2)) for _ in range(I - 1)])
        aug = augment_draws(rng, T)
        out.append((u, a0, z, aug))
    return out


def batched_demonstrations(field, regions, goals, uniforms, a0, z, device="cuda", stream=None,
                           T=K.DEMOS_CEM_PATH_LENGTH, P=K.DEMOS_CEM_NUM_PATHS,
                           I=K.DEMOS_CEM_NUM_ITERATIONS, E=K.DEMOS_CEM_NUM_ELITES):
    """get_demonstration for n problems at once. regions [n,4], goals [n,2], uniforms [n,2],
    a0 [n,P,T,2], z [n,I-1,P,T,2] (host or device). Returns (states [n,T,2], actions [n,T,2])
    float32 device tensors: the best final-iteration path without its last state and its
    actions (environment.py:173-179)."""
    dev = torch.device(device)
    f64 = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64).to(dev)  # noqa
    n = len(regions)
    reg, uni, gl = f64(regions), f64(uniforms), f64(goals)
    a0d = f64(a0)
    zd = f64(z)
    acts = torch.empty(n, P, T, 2, dtype=torch.float32, device=dev)
    paths = torch.empty(n, P, T + 1, 2, dtype=torch.float32, device=dev)
    rew = torch.empty(n, P, dtype=torch.float64, device=dev)
    mean = torch.zeros(n, T, 2, dtype=torch.float32, device=dev)
    std = torch.zeros(n, T, 2, dtype=torch.float32, device=dev)
    best = torch.zeros(n, dtype=torch.int32, device=dev)
    s = stream_handle(stream)
    L = lib()
    for it in range(I):
        zi = zd[:, it - 1].contiguous() if it > 0 else None
        L.nav_cem_rollout(ptr(field), n, P, T, it, ptr(reg), ptr(uni), ptr(gl), ptr(a0d),
                          ptr(zi), ptr(mean), ptr(std), ptr(acts), ptr(paths), ptr(rew), s)
        L.nav_cem_elite(n, P, T, E, ptr(rew), ptr(acts), ptr(mean), ptr(std), ptr(best), s)
    idx = best.long()
    ar = torch.arange(n, device=dev)
    return paths[ar, idx, :T].contiguous(), acts[ar, idx].contiguous()


def device_demo_sets(states, draws, n_demos=K.NUM_DEMO, stream=None,
                     interpolation_steps=K.AUG_INTERPOLATION):
    """Group demo sets on the device (nav_demo_augment): states [G*n_demos][T][2] float32 device
    tensor (CEM output, group-major), draws[g][d] = that demonstration's augmentation draws
    (augment_draws). Returns (points [sum m_g][2] f64 device tensor, offsets [G+1] int64 numpy);
    the same values as demo_set_from per group, bit for bit (tests/test_gpu_cem.py)."""
    n, T = states.shape[0], states.shape[1]
    G = n // n_demos
    n_aug = len(draws[0][0])
    noise = np.stack([np.stack(draws[g][d]) for g in range(G) for d in range(n_demos)])
    noise_d = torch.as_tensor(noise, dtype=torch.float64).to(states.device)
    per_demo = T + n_aug * ((T - 1) * (interpolation_steps + 1) + 1)
    out = torch.empty(n * per_demo, 2, dtype=torch.float64, device=states.device)
    lib().nav_demo_augment(n, T, interpolation_steps, n_aug, ptr(states.contiguous()),
                           ptr(noise_d), ptr(out), stream_handle(stream))
    off = np.arange(G + 1, dtype=np.int64) * n_demos * per_demo
    return out, off


def cem_group_demo_sets(field, regions, goals, seed, n_demos=K.NUM_DEMO, device="cuda",
                        on_device=True):
    """Per-group demonstration sets (CSR: points [sum m_g][2] f64, offsets [G+1] int64) built the
    way the reference builds one robot's: n_demos CEM demonstrations from the group's start region
    towards its goal, each with its 3 augmentations (robot.py:679-718, 771-824). Group g draws from
    numpy RandomState((seed + g) mod 2^32). on_device: the augmentation runs as nav_demo_augment
    and the points stay on the device; else the numpy restatement (demo_set_from) on the host."""
    G = len(regions)
    per_group = [group_stream_draws(np.random.RandomState((seed + g) & 0xFFFFFFFF), n_demos=n_demos)
                 for g in range(G)]
    rg = np.repeat(np.asarray(regions, np.float64), n_demos, 0)
    gl = np.repeat(np.asarray(goals, np.float64), n_demos, 0)
    uni = np.stack([d[0] for grp in per_group for d in grp])
    a0 = np.stack([d[1] for grp in per_group for d in grp])
    z = np.stack([d[2] for grp in per_group for d in grp])
    st, ac = batched_demonstrations(field, rg, gl, uni, a0, z, device)
    draws = [[per_group[g][d][3] for d in range(n_demos)] for g in range(G)]
    if on_device:
        return device_demo_sets(st, draws, n_demos)
    st, ac = st.cpu().numpy(), ac.cpu().numpy()
    pts, off = [], [0]
    for g in range(G):
        demos = [(st[g * n_demos + d], ac[g * n_demos + d]) for d in range(n_demos)]
        dset = demo_set_from(demos, draws=draws[g])
        pts.append(dset)
        off.append(off[-1] + len(dset))
    return np.concatenate(pts, 0), np.array(off, np.int64)
