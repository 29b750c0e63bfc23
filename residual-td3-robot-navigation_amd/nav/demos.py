"""Demonstration ingestion (robot.py:679-718) and augmentation (robot.py:771-824).

`augment` reproduces the reference's draw order and dtypes exactly (a single vectorised draw of
the same legacy-normal stream: the reference draws 2 gaussians per np.random.normal call, the cache
of the legacy polar method carries across calls, so one size-N call yields the same sequence), so
with the same numpy stream it yields the reference's demonstration set bit for bit.
"""
import numpy as np

from . import config as K


def augment(states, actions, rng=np.random, noise_level=K.AUG_NOISE,
            interpolation_steps=K.AUG_INTERPOLATION, num_augmentations=K.NUM_AUGMENTS):
    """robot.py:771-824. states/actions: [T][2] float32 (CEM output). Returns the list of
    augmented (states, actions) arrays, one [(T-1)*(steps+1)+1][2] float64 pair per augmentation."""
    states = np.asarray(states)
    actions = np.asarray(actions)
    T = len(states)
    per = interpolation_steps + 1
    out = []
    # python floats (weak scalars under NEP 50): fraction * float32 array stays float32
    frac = [s / float(interpolation_steps + 1) for s in range(1, interpolation_steps + 1)]
    for _ in range(num_augmentations):
        # draw order per i: steps x (state noise 2, action noise 2), then (state 2, action 2);
        # then the last state (2) and last action (2)
        g = rng.normal(0, noise_level, size=(T - 1) * per * 4 + 4)
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


def demo_set_from(demos, rng=np.random):
    """Robot.demonstration_states after process_demonstration of each (states, actions) demo:
    originals then their 3 augmentations, demo after demo (robot.py:694-698)."""
    pts = []
    for states, actions in demos:
        pts.append(np.asarray(states, np.float64))
        for s, _ in augment(states, actions, rng):
            pts.append(s)
    return np.concatenate(pts, 0) if pts else np.zeros((0, 2))


def synthetic_demo(region, goal, rng, T=K.DEMOS_CEM_PATH_LENGTH):
    """A straight-line stand-in for a CEM demonstration (used by the vectorised trainer's
    per-group demo sets until the batched CEM builds them): T float32 states from a uniform start
    in the init region towards the goal, with the matching constant actions."""
    l, r, b, t = region
    start = np.array([rng.uniform(l, r), rng.uniform(b, t)])
    a = np.clip((np.asarray(goal) - start) / T * 2.0, -K.ROBOT_MAX_ACTION, K.ROBOT_MAX_ACTION)
    s = start[None, :] + np.arange(T)[:, None] * a[None, :] * 0.5
    s = np.clip(s, 0, K.WORLD_SIZE - 1.0001)
    return s.astype(np.float32), np.repeat(a[None, :], T, 0).astype(np.float32)


def synthetic_group_demo_sets(regions, goals, seed, n_demos=K.NUM_DEMO):
    """Per-group demonstration sets (CSR: points [sum m_g][2] f64, offsets [G+1] int64), each of
    the reference's size: n_demos x (200 + 3 x 1195) = 11 355 points for 3 demos."""
    rng = np.random.RandomState(seed & 0xFFFFFFFF)
    pts, off = [], [0]
    for reg, goal in zip(regions, goals):
        demos = [synthetic_demo(reg, goal, rng) for _ in range(n_demos)]
        d = demo_set_from(demos, rng)
        pts.append(d)
        off.append(off[-1] + len(d))
    return np.concatenate(pts, 0), np.array(off, np.int64)
