"""Demonstration ingestion (robot.py:679-718) and augmentation (robot.py:771-824).

`augment` reproduces the reference's draw order and dtypes exactly (a single vectorised draw of
the same legacy-normal stream: the reference draws 2 gaussians per np.random.normal call, the cache
of the legacy polar method carries across calls, so one size-N call yields the same sequence), so
given the same demonstration states and numpy stream it yields the reference's demonstration set
bit for bit (nav_demo_augment on the device equals it bit for bit: tests/test_gpu_cem.py). The
drop-in's end-to-end trace test compares the set within 1e-4 because its demonstration states come
from the GPU CEM, whose dynamics differs from numpy's by < 1e-14 before the float32 cast of
environment.py:179, which can move a state by one float32 ulp.
"""
import numpy as np

from . import config as K


def augment_draw_size(T, interpolation_steps=K.AUG_INTERPOLATION):
    """Gaussians one augmentation of a T-state demonstration draws (robot.py:795-816)."""
    return (T - 1) * (interpolation_steps + 1) * 4 + 4


def augment_draws(rng, T, noise_level=K.AUG_NOISE, interpolation_steps=K.AUG_INTERPOLATION,
                  num_augmentations=K.NUM_AUGMENTS):
    """The normal draws of augment() for a T-state demonstration, from `rng`, in its order (for
    callers that consume a stream before the demonstration itself is known)."""
    n = augment_draw_size(T, interpolation_steps)
    return [rng.normal(0, noise_level, size=n) for _ in range(num_augmentations)]


def augment(states, actions, rng=np.random, noise_level=K.AUG_NOISE,
            interpolation_steps=K.AUG_INTERPOLATION, num_augmentations=K.NUM_AUGMENTS,
            draws=None):
    """robot.py:771-824. states/actions: [T][2] float32 (CEM output). Returns the list of
    augmented (states, actions) arrays, one [(T-1)*(steps+1)+1][2] float64 pair per augmentation.
    `draws` (augment_draws' output) replaces the draws from `rng`."""
    states = np.asarray(states)
    actions = np.asarray(actions)
    T = len(states)
    per = interpolation_steps + 1
    out = []
    # python floats (weak scalars under NEP 50): fraction * float32 array stays float32
    frac = [s / float(interpolation_steps + 1) for s in range(1, interpolation_steps + 1)]
    for k in range(num_augmentations):
        # draw order per i: steps x (state noise 2, action noise 2), then (state 2, action 2);
        # then the last state (2) and last action (2)
        g = draws[k] if draws is not None else rng.normal(0, noise_level,
                                                          size=(T - 1) * per * 4 + 4)
        body = g[:-4].reshape(T - 1, per, 2, 2)
        cur = states[:-1]
        nxt = states[1:]
        # synthetic_state = current + fraction * (next - current): float32 (NEP 50)
        diff = (nxt - cur)
        syn = np.stack([cur + f * diff for f in frac], 1)
        syn = syn.astype(states.dtype)
        aug_s = np.empty((T - 1, per, 2))
        aug_a = np.empty((T - 1, per, 2))
        aug_s[:, :interpolation_steps] = syn + body[:, :interpolation_steps, 0]
        aug_a[:, :interpolation_steps] = actions[:-1, None, :] + body[:, :interpolation_steps, 1]
        aug_s[:, interpolation_steps] = cur + body[:, interpolation_steps, 0]
        aug_a[:, interpolation_steps] = actions[:-1] + body[:, interpolation_steps, 1]
        s_all = np.concatenate([aug_s.reshape(-1, 2), (states[-1] + g[-4:-2])[None]], 0)
        a_all = np.concatenate([aug_a.reshape(-1, 2), (actions[-1] + g[-2:])[None]], 0)
        out.append((s_all, a_all))
    return out


def demo_set_from(demos, rng=np.random, draws=None):
    """Robot.demonstration_states after process_demonstration of each (states, actions) demo:
    originals then their 3 augmentations, demo after demo (robot.py:694-698). draws (nullable):
    per demo, augment_draws' output."""
    pts = []
    for k, (states, actions) in enumerate(demos):
        pts.append(np.asarray(states, np.float64))
        for s, _ in augment(states, actions, rng, draws=None if draws is None else draws[k]):
            pts.append(s)
    return np.concatenate(pts, 0) if pts else np.zeros((0, 2))
