"""Pin the CPU oracle (oracle/nav_oracle.c, oracle/td3_oracle.py) against vectors produced by the
reference itself (tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest

from conftest import golden


def test_legacy_rng_stream_matches_numpy(orc):
    # numpy legacy RandomState is the reference's RNG (environment.py:29-53, robot.py:111, 640)
    for seed in (1707366464, 0, 1, 987654321):
        rs = np.random.RandomState(seed)
        o = orc.LegacyRandomState(seed)
        assert [rs.random_sample() for _ in range(7)] == [o.random_sample() for _ in range(7)]
        assert [rs.randint(0, 4) for _ in range(9)] == [o.randint(0, 4) for _ in range(9)]
        assert [rs.normal(0, 1) for _ in range(9)] == [o.gauss() for _ in range(9)]
        assert (rs.permutation(1500) == o.permutation(1500)).all()
        assert (rs.choice(999, 100, replace=False) == o.permutation(999)[:100]).all()


def test_dynamics_and_step_vs_reference(orc):
    g = golden("dynamics.npz")
    sp, an = g["speed"], g["angle"]
    n = len(g["state"])
    out = np.array([orc.dynamics(sp, an, g["state"][i], g["action"][i]) for i in range(n)])
    ref = g["dynamics"]
    nan = np.isnan(ref)
    assert (np.isnan(out) == nan).all()
    # atan2 may differ by 1 ulp (numpy's SIMD atan2 vs libm); the 1e-5 bar of north_star is far off
    assert np.max(np.abs(out[~nan] - ref[~nan])) < 1e-12
    assert np.mean(out[~nan] == ref[~nan]) > 0.9
    for i in range(n):
        s, ok = orc.step(sp, an, g["state"][i], g["action"][i])
        assert ok == g["committed"][i]
        assert np.max(np.abs(s - g["step"][i])) < 1e-12


def test_init_goal_reset_stream_bit_exact(orc):
    g = golden("rng_init.npz")
    for k, seed in enumerate(g["seeds"]):
        o = orc.LegacyRandomState(int(seed))
        region, goal, side, draws = o.init_and_goal()
        assert (region == g["region"][k]).all(), seed
        assert (goal == g["goal"][k]).all(), seed
        for j in range(3):
            assert (o.reset(region) == g["resets"][k][j]).all()
        assert [o.random_sample() for _ in range(4)] == list(g["tail"][k])


def test_agent_trace_vs_reference(orc):
    """Replay the reference's headless tick loop through the oracle's fused tick (same actions,
    same reset states, same demo set): rewards, dones, flags and counters must match."""
    t = golden("trace.npz")
    p = orc.default_params()
    types = t["tick_type"]
    first = int(np.nonzero(types == 0)[0][0])
    st = orc.VecAgentState(1)
    c = t["counters"]
    st.state[0] = t["tick_state"][first]
    st.goal[0] = t["goal"]
    st.region[0] = t["region"]
    st.plan_index[0] = int(c[first][0])
    st.path_length[0] = int(c[first][1])
    st.episodes[0] = int(c[first][2])
    st.noise_scale[0] = c[first][6]
    st.meta[0] = 4  # demo_flag
    demo = t["demo_set"]
    n_checked = 0
    for i in range(first, len(types)):
        if types[i] != 0:
            continue
        a = t["tick_action"][i]
        lo, hi = t["push_idx"][i]
        assert hi - lo == 1
        reset_state = None
        if i + 1 < len(types) and types[i + 1] == 2:
            reset_state = t["tick_next"][i + 1]
        flags, ns, row, r = st.tick(p, t["speed"], t["angle"], demo, 0, a, reset_state)
        assert np.max(np.abs(ns - t["push_s2"][lo])) < 1e-12
        assert abs(r - t["push_r"][lo]) <= 1e-9 * max(1.0, abs(t["push_r"][lo]))
        assert bool(flags & 1) == bool(t["push_d"][lo])
        assert row[4] == np.float32(t["push_r"][lo])
        # counters after the reference's NEXT tick (which is where its reset/increment lands)
        if reset_state is not None:
            cc = c[i + 1]
            assert st.episodes[0] == int(cc[2]) and st.path_length[0] == int(cc[1])
            assert st.noise_scale[0] == cc[6]
            assert st.plan_index[0] == 1 and int(cc[0]) == 0
            assert np.array_equal(st.state[0], t["tick_next"][i + 1])
        else:
            assert (st.meta[0] & 2) == 0
        n_checked += 1
    assert n_checked > 300


def test_action_epilogue_and_actor_vs_reference(orc):
    import torch
    from oracle.td3_oracle import MLP, make_mlp_params
    g = golden("actions.npz")
    actor = MLP(make_mlp_params(int(g["actor_seed"]), [2, 200, 200, 200, 2]))
    b = (g["states"] - g["goals"]).astype(np.float32)
    with torch.no_grad():
        res = actor.forward(torch.tensor(b)).numpy()
    # batch-64 vs the reference's batch-1 GEMM: summation order differs (fp32)
    assert np.allclose(res, g["residual"], rtol=2e-5, atol=1e-4)
    for i in range(len(b)):
        a = orc.act_epilogue(g["states"][i], g["goals"][i], g["residual"][i], g["sigmas"][i],
                             g["z"][i])
        assert (a == g["action_train"][i]).all()
        a = orc.act_epilogue(g["states"][i], g["goals"][i], g["residual"][i], 0.0, None)
        assert (a == g["action_test"][i]).all()


def test_td3_oracle_vs_reference():
    from oracle.td3_oracle import TD3Oracle, make_mlp_params, param_digest
    g = golden("td3.npz")
    ora = TD3Oracle(make_mlp_params(21, [2, 200, 200, 200, 2]),
                    make_mlp_params(22, [4, 200, 200, 200, 1]),
                    make_mlp_params(23, [4, 200, 200, 200, 1]))
    it = {"s": 0, "n": 0}
    S, A, R, S2, D, idx, noise = (g[k] for k in ("S", "A", "R", "S2", "D", "idx", "noise"))

    def sample():
        i = idx[it["s"]]; it["s"] += 1
        return S[i], A[i], R[i], S2[i], D[i]

    def nz():
        x = noise[it["n"]]; it["n"] += 1
        return x

    closs, aloss = ora.td3_update(sample, nz, int(g["epochs"]))
    # fp32 losses are means over the batch: torch-CPU's reduction order follows the host's vector
    # ISA, and the fixture was written on another host (1.9e-5 relative seen on the actor loss)
    np.testing.assert_allclose(np.array(closs), g["critic_loss"], rtol=1e-4)
    np.testing.assert_allclose(np.array(aloss), g["actor_loss"], rtol=1e-4)
    for name, net in ora.networks().items():
        dig = param_digest(net)
        for k, (s, q, ix, v) in enumerate(dig):
            assert (ix == g[name + "_idx"][k]).all()
            np.testing.assert_allclose(v, g[name + "_val"][k], rtol=0, atol=1e-7)
            np.testing.assert_allclose(s, g[name + "_sum"][k], rtol=1e-6, atol=1e-5)


def test_cpu_demo_index_equals_brute_force(orc):
    """The CPU port's exact demo index (cpu_baseline leg) returns the brute-force minimum bit for
    bit: the reference's demo set (incl. augmented points off the world), shifted copies, queries
    on cell corners, on demo points, off the world."""
    from conftest import golden
    demo = golden("trace.npz")["demo_set"]
    rng = np.random.default_rng(21)
    for shift in (0.0, 7.3, -3.1):
        d = np.ascontiguousarray(demo + shift)
        ix = orc.DemoIndexCPU(d)
        assert ix.total < 60 * 10000  # sublinear: tens of candidates per cell, not 11 355
        q = rng.uniform(-2, 101, (3000, 2))
        q[:300] = np.floor(q[:300])
        q[300:600] = d[rng.integers(0, len(d), 300)]
        for x, y in q:
            want = orc.lib().orc_demo_min(orc.ptr(d, orc._dp), len(d), float(x), float(y))
            assert ix.min(float(x), float(y)) == want


def test_td3_oracle_gradients_vs_reference():
    """The oracle's autograd gradients (TD3Oracle.last_grads) of the first train_critic and
    train_actor equal the reference's own param.grad (td3_grads.npz, robot.py:355-363, 393-395)
    on the same weights, batches and noise: the oracle is pinned at the gradient level, where
    Adam's sign-like first step hides a gradient scale."""
    from conftest import golden_grad_check
    from oracle.td3_oracle import TD3Oracle, make_mlp_params
    g, gg = golden("td3.npz"), golden("td3_grads.npz")
    ora = TD3Oracle(make_mlp_params(21, [2, 200, 200, 200, 2]),
                    make_mlp_params(22, [4, 200, 200, 200, 1]),
                    make_mlp_params(23, [4, 200, 200, 200, 1]))
    S, A, R, S2, D = (g[k] for k in ("S", "A", "R", "S2", "D"))
    i = gg["critic_idx"]
    assert np.array_equal(i, g["idx"][0]) and np.array_equal(gg["noise"], g["noise"][0])
    ora.train_critic((S[i], A[i], R[i], S2[i], D[i]), gg["noise"])
    for name, key in (("critic1", "c1"), ("critic2", "c2")):
        sc = golden_grad_check(gg, name, [t.numpy() for t in ora.last_grads[key]], 1e-6, 1e-7)
        assert abs(sc - 1) <= 1e-6, (name, sc)
    ora.train_actor(S[gg["actor_idx"]])
    sc = golden_grad_check(gg, "actor", [t.numpy() for t in ora.last_grads["actor"]], 1e-6, 1e-7)
    assert abs(sc - 1) <= 1e-6, sc
