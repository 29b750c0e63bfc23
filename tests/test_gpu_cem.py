"""Batched CEM demonstrator (environment.py:140-179) vs the N = 1 drop-in's get_demonstration on
the same numpy stream (that one is pinned to the reference's own outputs by
tests/test_gpu_dropin.py): every group's 3 demonstrations, bit for bit, and the group demo sets
built from them."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _groups(G, seed):
    from oracle import oracle as O
    p = O.default_params(seed)
    regions, goals = [], []
    for g in range(G):
        r, gl, _ = O.vec_init_one(p, g)
        regions.append(r)
        goals.append(gl)
    return np.array(regions), np.array(goals)


def test_batched_cem_equals_dropin_demonstrations():
    from nav import _lib
    from nav.cem import batched_demonstrations, group_stream_draws
    from nav.demos import augment, demo_set_from
    from nav.environment import Environment
    from nav.fields import make_fields
    from nav.vec_env import make_field
    _lib.require_gpu()
    speed, angle = make_fields(1707366464)
    field = make_field(speed, angle, DEV)
    G, nd, seed = 4, 3, 1234
    regions, goals = _groups(G, 77)
    draws = [group_stream_draws(np.random.RandomState(seed + g), n_demos=nd) for g in range(G)]
    uni = np.stack([d[0] for grp in draws for d in grp])
    a0 = np.stack([d[1] for grp in draws for d in grp])
    z = np.stack([d[2] for grp in draws for d in grp])
    st, ac = batched_demonstrations(field, np.repeat(regions, nd, 0), np.repeat(goals, nd, 0), uni,
                                    a0, z, DEV)
    st, ac = st.cpu().numpy(), ac.cpu().numpy()
    env = Environment(speed, angle)
    for g in range(G):
        # the drop-in on the group's stream: demo, its augmentation draws, next demo ...
        np.random.set_state(np.random.RandomState(seed + g).get_state())
        env.robot_init_region = regions[g].copy()
        env.goal_state = goals[g].copy()
        env._region.copy_(torch.tensor(regions[g][None]))
        env._goal.copy_(torch.tensor(goals[g][None]))
        demos = []
        for d in range(nd):
            s_ref, a_ref = env.get_demonstration()
            k = g * nd + d
            assert s_ref.dtype == st.dtype == np.float32
            assert np.array_equal(s_ref, st[k]), (g, d)
            assert np.array_equal(a_ref, ac[k]), (g, d)
            demos.append((s_ref, a_ref))
            augment(s_ref, a_ref, np.random)  # process_demonstration's draws
        # the group demo set from the batched plans and the pre-drawn augmentation noise
        got = demo_set_from([(st[g * nd + d], ac[g * nd + d]) for d in range(nd)],
                            draws=[draws[g][d][3] for d in range(nd)])
        # same demo set as augmenting the drop-in's demos with the draws in stream order
        want = []
        rs = np.random.RandomState(seed + g)
        for d in range(nd):
            rs.random_sample(2)
            rs.choice([-5, 5], (100, 200, 2))
            for _ in range(3):
                rs.standard_normal((100, 200, 2))
            want.append(np.asarray(demos[d][0], np.float64))
            for s_aug, _ in augment(demos[d][0], demos[d][1], rs):
                want.append(s_aug)
        assert np.array_equal(got, np.concatenate(want, 0)), g


def test_vec_trainer_uses_cem_demo_sets():
    from nav.trainer import VecTrainer
    tr = VecTrainer(n_envs=2048, hidden=64, n_hidden=2, batch=512, updates_per_step=2,
                    envs_per_group=512, device=DEV)
    off = tr.env.demo_off.cpu().numpy()
    assert len(off) == 5
    # 3 demonstrations x (200 + 3 x 1195) points per group, the reference's demo-set size
    assert np.all(np.diff(off) == 3 * (200 + 3 * 1195))
    pts = tr.env.demo_xy.cpu().numpy()
    assert np.isfinite(pts).all()
    # each group's first demonstration starts in that group's init region
    for g in range(4):
        r = tr.env.region[g * 512].cpu().numpy()
        s0 = pts[off[g]]
        assert r[0] - 1e-4 <= s0[0] <= r[1] + 1e-4 and r[2] - 1e-4 <= s0[1] <= r[3] + 1e-4


def test_device_demo_sets_equal_host_augmentation():
    """nav_demo_augment (the demo sets built on the device) equals the numpy restatement
    demo_set_from (pinned above against the drop-in's process_demonstration draws) bit for bit."""
    from nav.cem import cem_group_demo_sets
    from nav.fields import make_fields
    from nav.vec_env import make_field
    speed, angle = make_fields(1707366464)
    field = make_field(speed, angle, DEV)
    regions, goals = _groups(5, 31)
    dev_pts, dev_off = cem_group_demo_sets(field, regions, goals, 99, on_device=True)
    host_pts, host_off = cem_group_demo_sets(field, regions, goals, 99, on_device=False)
    assert np.array_equal(dev_off, host_off)
    got = dev_pts.cpu().numpy()
    assert got.dtype == host_pts.dtype == np.float64
    assert np.array_equal(got, host_pts)
