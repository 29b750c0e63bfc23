"""GPU parity of the environment / agent-tick kernels against the oracle and the reference goldens.

Tolerances (north_star): seeding and indexing bit-exact; float state within 1e-5 (observed: f64
state agrees to ~1e-13 — the kernels move by speed * R(rot) * a instead of the reference's
speed * |a| * (cos, sin)(atan2 + rot), the same displacement up to a few ulp, and numpy's SIMD
atan2 differs from libm by 1 ulp)."""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def nav():
    import nav as navpkg
    from nav import _lib
    _lib.require_gpu()
    _lib.lib()
    return navpkg


def field_of(speed, angle):
    from nav.vec_env import make_field
    return make_field(speed, angle, DEV)


def test_dynamics_vs_reference_golden(nav, orc):
    from nav.vec_env import VecEnv
    g = golden("dynamics.npz")
    f = field_of(g["speed"], g["angle"])
    s = torch.tensor(g["state"], device=DEV)
    a = torch.tensor(g["action"], device=DEV)
    env = VecEnv(1, f, init=False)
    out = env.dynamics(s, a).cpu().numpy()
    ref = g["dynamics"]
    nan = np.isnan(ref)
    assert (np.isnan(out) == nan).all()
    assert np.max(np.abs(out[~nan] - ref[~nan])) < 1e-11
    # against the oracle on the same inputs
    orc_out = np.array([orc.dynamics(g["speed"], g["angle"], g["state"][i], g["action"][i])
                        for i in range(len(ref))])
    assert np.max(np.abs(out[~nan] - orc_out[~nan])) < 1e-11


def test_env_step_commit_semantics(nav):
    from nav.vec_env import VecEnv
    g = golden("dynamics.npz")
    f = field_of(g["speed"], g["angle"])
    n = len(g["state"])
    env = VecEnv(n, f, init=False)
    env.state.copy_(torch.tensor(g["state"], device=DEV))
    ns = torch.zeros(n, 2, dtype=torch.float64, device=DEV)
    env.step(torch.tensor(g["action"], device=DEV), next_state=ns)
    out = env.state.cpu().numpy()
    assert np.max(np.abs(out - g["step"])) < 1e-11
    assert np.array_equal(ns.cpu().numpy(), out)
    nan_rows = np.isnan(g["action"]).any(1)
    assert np.array_equal(out[nan_rows], g["state"][nan_rows])  # NaN action: unchanged


def test_env_step_full_size_nontemporal_path(nav):
    """4 Mi + 37 envs (the non-temporal stream path, ragged last block): every env is a tiled copy
    of a golden case, so each must land on that case's reference result, and bit-identical to the
    small-n (default cache policy) launch of the same cases."""
    from nav.vec_env import VecEnv
    g = golden("dynamics.npz")
    f = field_of(g["speed"], g["angle"])
    k = len(g["state"])
    n = (1 << 22) + 37
    reps = (n + k - 1) // k
    st = torch.tensor(g["state"], device=DEV).repeat(reps, 1)[:n].contiguous()
    ac = torch.tensor(g["action"], device=DEV).repeat(reps, 1)[:n].contiguous()
    big = VecEnv(n, f, init=False)
    big.state.copy_(st)
    ns = torch.zeros(n, 2, dtype=torch.float64, device=DEV)
    big.step(ac, next_state=ns)
    small = VecEnv(k, f, init=False)
    small.state.copy_(st[:k])
    small.step(ac[:k])
    torch.cuda.synchronize()
    out = big.state.cpu().numpy()
    want = np.tile(g["step"], (reps, 1))[:n]
    assert np.max(np.abs(out - want)) < 1e-11
    assert np.array_equal(ns.cpu().numpy(), out)
    assert np.array_equal(out[:k], small.state.cpu().numpy())
    del big, st, ac, ns
    torch.cuda.empty_cache()


def test_env_step_k_equals_k_single_steps(nav):
    """nav_env_step_k (K steps, state in registers) == K nav_env_step launches, bit for bit,
    golden cases as starting states and random / NaN / out-of-range actions per step."""
    from nav.vec_env import VecEnv
    g = golden("dynamics.npz")
    f = field_of(g["speed"], g["angle"])
    n, K = len(g["state"]), 9
    rng = np.random.default_rng(4)
    acts = rng.uniform(-7, 7, (K, n, 2))
    acts[3, ::17] = np.nan
    a = torch.tensor(acts, device=DEV)
    one = VecEnv(n, f, init=False)
    many = VecEnv(n, f, init=False)
    for e in (one, many):
        e.state.copy_(torch.tensor(g["state"], device=DEV))
    nxt = torch.zeros(K, n, 2, dtype=torch.float64, device=DEV)
    many.step_k(a, next_states=nxt)
    for k in range(K):
        one.step(a[k].contiguous())
        assert torch.equal(nxt[k], one.state), k
    assert torch.equal(many.state, one.state)
    many.step_k(a)  # without the per-step output
    for k in range(K):
        one.step(a[k].contiguous())
    assert torch.equal(many.state, one.state)


def test_demo_flag_without_demo_set_keeps_stuck_penalty(nav, orc):
    """demo_flag set but no demonstration set — the reference's compute_reward returns
    the goal term (robot.py:749-751) and process_transition still subtracts the stuck penalty
    (robot.py:667-669). Motionless envs get stuck after 5 ticks; rows vs the oracle tick."""
    from nav.vec_env import ReplayRing, VecEnv
    from oracle.oracle import VecAgentState, default_params
    g = golden("trace.npz")
    n = 300
    env = VecEnv(n, field_of(g["speed"], g["angle"]), seed=17, envs_per_group=1,
                 demo_flag=True)
    assert (env.meta.cpu().numpy() & 4).all()
    rep = ReplayRing(n, DEV)
    p = default_params(17)
    ost = VecAgentState(n)
    rng = np.random.default_rng(2)
    stuck_seen = 0
    for t in range(8):
        a = rng.uniform(-1e-3, 1e-3, (n, 2))
        a[n // 2:] = rng.uniform(-5, 5, (n - n // 2, 2))
        _sync_oracle(env, ost)
        base = rep.position
        env.agent_step(torch.tensor(a, device=DEV), rep)
        torch.cuda.synchronize()
        rows = rep.rows.cpu().numpy()
        fl = env.flags.cpu().numpy()
        assert not (fl & 16).any()  # no demo term is pending without a demo set
        for e in range(n):
            flo, ns, row, r = ost.tick(p, g["speed"], g["angle"], np.zeros((0, 2)), e, a[e])
            assert (flo & 15) == (fl[e] & 15), (t, e)
            assert np.allclose(row, rows[(base + e) % rep.capacity], rtol=1e-6, atol=1e-5), (t, e)
        stuck_seen += int(((fl & 4) != 0).sum())
    assert stuck_seen > 0


def test_empty_launches_are_noops(nav):
    from nav import _lib
    from nav.vec_env import VecEnv
    g = golden("dynamics.npz")
    f = field_of(g["speed"], g["angle"])
    env = VecEnv(1, f, init=False)
    s = torch.zeros(0, 2, dtype=torch.float64, device=DEV)
    assert env.dynamics(s, s).shape == (0, 2)
    assert _lib.lib().nav_dynamics(None, None, None, None, 0, None) == 0


@pytest.mark.parametrize("n,epg", [(4096, 1), (5000, 7), (1, 1)])
def test_env_init_and_reset_bit_exact_vs_oracle(nav, orc, n, epg):
    from nav.vec_env import VecEnv
    from oracle.oracle import default_params, vec_init_one, vec_reset_one
    g = golden("dynamics.npz")
    env = VecEnv(n, field_of(g["speed"], g["angle"]), seed=1234567, envs_per_group=epg)
    torch.cuda.synchronize()
    p = default_params(1234567)
    region = env.region.cpu().numpy()
    goal = env.goal.cpu().numpy()
    state = env.state.cpu().numpy()
    draws = env.goal_draws.cpu().numpy()
    for e in list(range(min(n, 300))) + ([n - 1] if n > 300 else []):
        r, gl, k = vec_init_one(p, e // epg)
        assert np.array_equal(region[e], r) and np.array_equal(goal[e], gl) and draws[e] == k
        assert np.array_equal(state[e], vec_reset_one(p, e, 5, r))
    assert (draws > 0).all()
    d = np.linalg.norm(goal - 0.5 * np.stack([region[:, 0] + region[:, 1],
                                              region[:, 2] + region[:, 3]], 1), axis=1)
    assert (d >= 90).all()
    assert (env.plan_index.cpu() == 5).all() and (env.path_length.cpu() == 50).all()
    # Environment.reset with injected uniforms (numpy stream) and with Philox
    u = torch.rand(n, 2, dtype=torch.float64, device=DEV)
    env.reset(uniforms=u)
    uu = u.cpu().numpy()
    st = env.state.cpu().numpy()
    for e in range(min(n, 200)):
        assert np.array_equal(st[e], orc.reset_u(region[e], uu[e, 0], uu[e, 1]))
    mask = (torch.arange(n, device=DEV) % 2 == 0).to(torch.uint8)
    before = env.state.clone()
    env.reset(mask=mask)
    st = env.state.cpu().numpy()
    assert torch.equal(env.state[1::2], before[1::2])
    for e in range(0, min(n, 200), 2):
        assert np.array_equal(st[e], vec_reset_one(p, e, 5, region[e]))


def _sync_oracle(env, ost):
    ost.state[:] = env.state.cpu().numpy()
    ost.goal[:] = env.goal.cpu().numpy()
    ost.region[:] = env.region.cpu().numpy()
    ost.hist[:] = env.hist.cpu().numpy().transpose(1, 0, 2)
    ost.meta[:] = env.meta.cpu().numpy().astype(np.uint32)
    ost.plan_index[:] = env.plan_index.cpu().numpy()
    ost.path_length[:] = env.path_length.cpu().numpy()
    ost.episodes[:] = env.episodes.cpu().numpy()
    ost.noise_scale[:] = env.noise_scale.cpu().numpy()


def test_agent_step_vs_oracle_per_step(nav, orc):
    """Fused tick (nav_agent_step + nav_demo_reward) vs the oracle's restated tick, re-synced from
    the device state before every step so every step is compared on identical inputs."""
    from nav.vec_env import ReplayRing, VecEnv
    from oracle.oracle import VecAgentState, default_params
    g = golden("trace.npz")
    n, epg = 512, 256
    env = VecEnv(n, field_of(g["speed"], g["angle"]), seed=99, envs_per_group=epg)
    demo = g["demo_set"]
    G = n // epg
    # group g uses a shifted copy of the reference demo set
    pts = np.concatenate([demo + 0.5 * k for k in range(G)])
    off = np.arange(G + 1, dtype=np.int64) * len(demo)
    env.set_demo(pts, off)
    rep = ReplayRing(n * 3, DEV)
    p = default_params(99)
    ost = VecAgentState(n)
    rng = np.random.default_rng(0)
    rows_o = np.zeros((rep.capacity, 8), np.float32)
    checked_demo = 0
    for t in range(40):
        # push some envs towards their goals so goal hits happen, freeze others to get stuck
        s = env.state.cpu().numpy(); gl = env.goal.cpu().numpy()
        a = rng.uniform(-6, 6, (n, 2))
        a[: n // 4] = np.clip(gl[: n // 4] - s[: n // 4], -5, 5)
        a[n // 4: n // 2] = rng.uniform(-0.05, 0.05, (n // 4, 2))
        _sync_oracle(env, ost)
        base = rep.position
        reward = torch.zeros(n, dtype=torch.float64, device=DEV)
        env.agent_step(torch.tensor(a, device=DEV), rep, reward_out=reward)
        torch.cuda.synchronize()
        # oracle: per-group demo set
        ns_o = np.zeros((n, 2))
        flags_o = np.zeros(n, np.int64)
        r_o = np.zeros(n)
        for grp in range(G):
            sl = slice(grp * epg, (grp + 1) * epg)
            sub = VecAgentState(epg)
            for k in ("state", "goal", "region", "hist", "meta", "plan_index", "path_length",
                      "episodes", "noise_scale"):
                getattr(sub, k)[:] = getattr(ost, k)[sl]
            dset = pts[off[grp]:off[grp + 1]]
            for j in range(epg):
                e = grp * epg + j
                fl, ns, row, r = sub.tick(p, g["speed"], g["angle"], dset, j, a[e])
                # the oracle tick was called with env index j: redo its reset draw for env e
                ns_o[e] = ns
                flags_o[e] = fl
                r_o[e] = r
                rows_o[(base + e) % rep.capacity] = row
            for k in ("state", "goal", "region", "hist", "meta", "plan_index", "path_length",
                      "episodes", "noise_scale"):
                getattr(ost, k)[sl] = getattr(sub, k)
        ended = (flags_o & 8) != 0
        # reset draws use the env index: recompute them for the ended envs in the oracle copy
        from oracle.oracle import vec_reset_one
        for e in np.nonzero(ended)[0]:
            ost.state[e] = vec_reset_one(p, int(e), int(ost.episodes[e]), ost.region[e])
        assert np.max(np.abs(env.next_state.cpu().numpy() - ns_o)) < 1e-11
        fl_dev = env.flags.cpu().numpy().astype(np.int64)
        assert np.array_equal(fl_dev & 15, flags_o & 15), t
        assert np.array_equal(env.plan_index.cpu().numpy(), ost.plan_index)
        assert np.array_equal(env.path_length.cpu().numpy(), ost.path_length)
        assert np.array_equal(env.episodes.cpu().numpy(), ost.episodes)
        assert np.array_equal(env.noise_scale.cpu().numpy(), ost.noise_scale)
        assert np.array_equal(env.meta.cpu().numpy().astype(np.uint32), ost.meta)
        assert np.max(np.abs(env.state.cpu().numpy() - ost.state)) < 1e-11
        got = rep.rows.cpu().numpy()
        idx = (base + np.arange(n)) % rep.capacity
        close = np.abs(got[idx] - rows_o[idx]) <= 1e-5 * np.maximum(1, np.abs(rows_o[idx]))
        assert close.all(), t
        # the launch's reward / done reduction (north_star: reduced by wavefront shuffles), every
        # column of every 64-env row: the pushed reward (demo term included: the fused launch)
        # within 1e-5 relative, the done / goal / stuck / ended counts exact
        bs = env.block_stats.cpu().numpy().astype(np.float64)
        rows64 = lambda v: v.reshape(-1, 64).sum(1)  # noqa: E731
        cols = (r_o, flags_o & 1, (flags_o >> 1) & 1, (flags_o >> 2) & 1, (flags_o >> 3) & 1)
        ref = np.stack([rows64(np.asarray(c, np.float64)) for c in cols], 1)
        mag = rows64(np.abs(r_o))
        assert np.all(np.abs(bs[:, 0] - ref[:, 0]) <= 1e-5 * np.maximum(1.0, mag)), t
        assert np.array_equal(bs[:, 1:5], ref[:, 1:5]), t
        assert (bs[:, 5:] == 0).all()
        checked_demo += int(((fl_dev & 16) != 0).sum())
    assert checked_demo > 0  # the demo term was part of the checked sums


def test_agent_step_replays_reference_trace(nav):
    """The reference's own headless tick loop (golden trace) replayed through nav_agent_step with
    N = 1: same actions, same demo set, reset states injected at the reference's reset ticks."""
    from nav.vec_env import ReplayRing, VecEnv
    t = golden("trace.npz")
    env = VecEnv(1, field_of(t["speed"], t["angle"]), init=False)
    types = t["tick_type"]
    first = int(np.nonzero(types == 0)[0][0])
    c = t["counters"]
    env.state[0] = torch.tensor(t["tick_state"][first])
    env.goal[0] = torch.tensor(t["goal"])
    env.region[0] = torch.tensor(t["region"])
    env.plan_index[0] = int(c[first][0])
    env.path_length[0] = int(c[first][1])
    env.episodes[0] = int(c[first][2])
    env.noise_scale[0] = float(c[first][6])
    env.meta[0] = 4
    env.set_demo(t["demo_set"])
    rep = ReplayRing(2048, DEV)
    reward = torch.zeros(1, dtype=torch.float64, device=DEV)
    n_checked = 0
    for i in range(first, len(types)):
        if types[i] != 0:
            continue
        lo = t["push_idx"][i][0]
        reward.fill_(np.nan)
        base = env.agent_step(torch.tensor(t["tick_action"][i][None], device=DEV), rep,
                              reward_out=reward)
        fl = int(env.flags[0].item())
        r = reward.item() if fl & 16 else float(rep.rows[base, 4].item())
        ref_r = t["push_r"][lo]
        if fl & 16:
            assert abs(r - ref_r) <= 1e-9 * max(1.0, abs(ref_r)), i
        else:
            assert np.float32(r) == np.float32(ref_r), i
        assert abs(float(rep.rows[base, 4].item()) - ref_r) <= 1e-5 * max(1.0, abs(ref_r))
        assert bool(fl & 1) == bool(t["push_d"][lo])
        assert np.max(np.abs(env.next_state[0].cpu().numpy() - t["push_s2"][lo])) < 1e-11
        if i + 1 < len(types) and types[i + 1] == 2:
            assert fl & 8
            assert env.episodes[0].item() == int(c[i + 1][2])
            assert env.path_length[0].item() == int(c[i + 1][1])
            assert env.noise_scale[0].item() == c[i + 1][6]
            env.state[0] = torch.tensor(t["tick_next"][i + 1])  # the reference's reset draw
        else:
            assert not fl & 8
        n_checked += 1
    assert n_checked > 300


def test_demo_index_bit_exact_vs_brute_force(nav, orc):
    """The two-level demo index returns the brute-force minimum bit for bit (same f64 values),
    through the tick's block-cooperative demo pass (nav_agent_step_indexed) and the per-env
    indexed pass (nav_demo_reward_indexed), on states at dynamics-cell and index-cell corners, on
    demo points, and packed around the demo path (the longest candidate lists). The block_stats
    reward column is the pushed (final) reward's sum in all three launch forms, bit for bit."""
    from nav.vec_env import ReplayRing, VecEnv
    t = golden("trace.npz")
    demo = t["demo_set"]
    n, epg = 4096, 1024
    G = n // epg
    pts = np.concatenate([demo + 3.0 * k for k in range(G)])
    off = np.arange(G + 1, dtype=np.int64) * len(demo)
    rng = np.random.default_rng(9)
    s = rng.uniform(0, 99, (n, 2))
    s[:512] = np.floor(s[:512])  # exactly on dynamics-cell corners
    s[512:1024] = demo[rng.integers(0, len(demo), 512)].clip(0, 98.99)  # on demo points
    s[1024:1536] = np.floor(s[1024:1536] * 4) / 4  # on index-cell corners
    near = demo[rng.integers(0, len(demo), 1536)] + rng.uniform(-0.4, 0.4, (1536, 2))
    s[1536:3072] = near.clip(0, 98.99)  # packed around the demo path
    # envs of group g query demo set g = the trace's demo shifted by 3 g
    shift = 3.0 * (np.arange(n) // epg)
    for lo, hi in ((512, 1024), (1536, 3072)):
        s[lo:hi] += shift[lo:hi, None]
    s = s.clip(0, 99.99)
    rewards = []
    for mode in ("fused", "per_env", "brute"):
        env = VecEnv(n, field_of(t["speed"], t["angle"]), seed=5, envs_per_group=epg)
        env.set_demo(pts, off, index=mode != "brute")
        env.fuse_demo = mode == "fused"
        env.state.copy_(torch.tensor(s))
        rep = ReplayRing(n, DEV)
        r = torch.zeros(n, dtype=torch.float64, device=DEV)
        env.agent_step(torch.zeros(n, 2, dtype=torch.float64, device=DEV), rep, reward_out=r)
        rewards.append((r.cpu().numpy(), env.flags.cpu().numpy(), rep.rows.cpu().numpy(),
                        env.block_stats.cpu().numpy()))
        if mode != "brute":
            assert env.demo_index.mean_candidates < 200
    (ri, fi, wi, si), (rp, fp, wp, sp), (rb, fb, wb, sb) = rewards
    assert np.array_equal(si, sb) and np.array_equal(sp, sb)
    pushed = wb[:, 4].astype(np.float64).reshape(-1, 64).sum(1)
    assert np.allclose(sb[:, 0], pushed, rtol=1e-5, atol=1e-3)
    assert np.array_equal(fi, fb) and np.array_equal(fp, fb)
    m = (fi & 16) != 0
    assert m.sum() > n // 2
    assert np.array_equal(ri[m], rb[m]) and np.array_equal(rp[m], rb[m])
    assert np.array_equal(wi, wb) and np.array_equal(wp, wb)


def test_compute_reward_kernel_vs_oracle(nav, orc):
    from nav._lib import lib, params_struct, ptr, stream_handle
    t = golden("trace.npz")
    demo = torch.tensor(t["demo_set"], device=DEV)
    rng = np.random.default_rng(3)
    ns = rng.uniform(0, 100, (777, 2))
    goal = rng.uniform(5, 95, (777, 2))
    ns[:20] = goal[:20] + rng.uniform(-3, 3, (20, 2))
    out = torch.zeros(777, dtype=torch.float64, device=DEV)
    hit = torch.zeros(777, dtype=torch.uint8, device=DEV)
    p = params_struct()
    nst, gt = torch.tensor(ns, device=DEV), torch.tensor(goal, device=DEV)
    lib().nav_compute_reward(C.byref(p), 777, ptr(nst), ptr(gt), ptr(demo), len(demo), 1,
                             ptr(out), ptr(hit), stream_handle())
    o = out.cpu().numpy()
    for i in range(777):
        r, gr = orc.compute_reward(ns[i], goal[i], t["demo_set"], True)
        assert r == o[i] and gr == bool(hit[i].item())


def test_device_field_generator_vs_host(nav):
    """nav_fields_generate (set_dynamics as nav.fields restates it) vs make_fields on the host:
    the angle table bit for bit, the speed table within 4 ulp (numpy's SIMD float32 exp is not
    correctly rounded; the device rounds the f64 exp), over several seeds. Parity against the reference itself is unpinned
    (perlin_noise is absent)."""
    from nav.fields import make_field_device, make_fields
    for seed in (1707366464, 0, 12345):
        speed, angle = make_fields(seed)
        f = make_field_device(seed, DEV).cpu().numpy()
        assert np.array_equal(f[..., 1], angle), seed
        ulp = np.abs(f[..., 0].view(np.int32).astype(np.int64) - speed.view(np.int32))
        assert ulp.max() <= 4, (seed, ulp.max())
        assert (ulp == 0).mean() > 0.5


@pytest.mark.parametrize("groups", [1, 7, 64])
def test_demo_index_scans_vs_cumsum(nav, groups):
    """nav_demo_index_scan / _subscan (the multi-workgroup exclusive scans of the demo index
    build: tile totals, their scan, the tiles from their offsets) equal numpy's exclusive cumsum
    with the total in the last entry, on ragged sizes (10 000 and 160 000 cells per group are not
    multiples of the 4 096-count tile)."""
    from nav._lib import lib, ptr
    L = lib()
    res = L.nav_demo_index_res()
    for n_per, fn in ((10000, L.nav_demo_index_scan), (10000 * res * res, L.nav_demo_index_subscan)):
        n = groups * n_per
        g = np.random.default_rng(n)
        cnt = g.integers(0, 60, n).astype(np.int32)
        cnt[g.integers(0, n, max(1, n // 50))] = 0
        c = torch.tensor(cnt, device="cuda")
        start = torch.full((n + 1,), -7, dtype=torch.int64, device="cuda")
        fn(ptr(c), groups, ptr(start), None)
        torch.cuda.synchronize()
        ref = np.zeros(n + 1, dtype=np.int64)
        ref[1:] = np.cumsum(cnt, dtype=np.int64)
        assert np.array_equal(start.cpu().numpy(), ref), (groups, n_per)
