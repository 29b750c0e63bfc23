"""GPU checks at the bench configuration (BASELINE config 3: 65 536 envs in 64 groups of 1 024,
2x256 actor/critic, TD3 batch 32 768): the fused tick of a random subset of envs spread over every
group against the oracle's restated tick (robot.py:645-675, 727-762, environment.py:98-137) on the
same inputs, and size-independent invariants of the whole state and of the learner after it."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def trainer():
    from nav import _lib
    from nav.trainer import VecTrainer
    _lib.require_gpu()
    torch.cuda.set_device(0)
    tr = VecTrainer(n_envs=65536, hidden=256, n_hidden=2, batch=32768, updates_per_step=2,
                    envs_per_group=1024, device=DEV)
    for _ in range(3):  # the replay ring holds a batch after the first step: learner active
        tr.step()
    torch.cuda.synchronize()
    return tr


def test_bench_config_tick_subset_vs_oracle(trainer, orc):
    from oracle import oracle as O
    tr, env = trainer, trainer.env
    n = tr.n
    fields = env.field.cpu().numpy()
    speed, angle = np.ascontiguousarray(fields[..., 0]), np.ascontiguousarray(fields[..., 1])
    ost = O.VecAgentState(n)
    ost.state[:] = env.state.cpu().numpy()
    ost.goal[:] = env.goal.cpu().numpy()
    ost.region[:] = env.region.cpu().numpy()
    ost.hist[:] = env.hist.cpu().numpy().transpose(1, 0, 2)
    ost.meta[:] = env.meta.cpu().numpy().astype(np.uint32)
    ost.plan_index[:] = env.plan_index.cpu().numpy()
    ost.path_length[:] = env.path_length.cpu().numpy()
    ost.episodes[:] = env.episodes.cpu().numpy()
    ost.noise_scale[:] = env.noise_scale.cpu().numpy()
    pts = env.demo_xy.cpu().numpy()
    off = env.demo_off.cpu().numpy()
    epg = n // (len(off) - 1)
    p = O.default_params(tr.seed)
    tr.act()
    a = tr.action.cpu().numpy()
    assert np.isfinite(a).all() and np.abs(a).max() <= 5.0
    base = tr.replay.position
    env.agent_step(tr.action, tr.replay)
    torch.cuda.synchronize()
    rows = tr.replay.rows.cpu().numpy()
    nxt = env.next_state.cpu().numpy()
    st = env.state.cpu().numpy()
    rng = np.random.default_rng(5)
    idx = np.concatenate([g * epg + rng.choice(epg, 2, replace=False)
                          for g in range(len(off) - 1)])
    for e in idx:
        grp = e // epg
        fl, ns, row, r = ost.tick(p, speed, angle, pts[off[grp]:off[grp + 1]], int(e), a[e])
        assert np.max(np.abs(ns - nxt[e])) < 1e-11, e
        assert np.allclose(row, rows[(base + e) % tr.replay.capacity], rtol=1e-5, atol=1e-5), e
        assert np.max(np.abs(ost.state[e] - st[e])) < 1e-11, e
    for k in ("plan_index", "path_length", "episodes"):
        assert np.array_equal(getattr(env, k)[idx].cpu().numpy(), getattr(ost, k)[idx]), k


def test_bench_config_invariants(trainer):
    tr, env = trainer, trainer.env
    tr.step()
    torch.cuda.synchronize()
    s = env.state.cpu().numpy()
    assert np.isfinite(s).all() and s.min() >= 0.0 and s.max() <= 100.0 - 1.0001
    plan, path = env.plan_index.cpu().numpy(), env.path_length.cpu().numpy()
    assert (plan >= 1).all() and (plan < path).all()  # an episode ends at plan == path - 1
    assert (env.episodes.cpu().numpy() >= 0).all()
    ns = env.noise_scale.cpu().numpy()
    assert np.isfinite(ns).all() and (ns > 0).all()
    filled = min(len(tr.replay), tr.replay.capacity)
    rows = tr.replay.rows[:filled].cpu().numpy()
    assert np.isfinite(rows).all()
    assert np.isin(rows[:, 7], (0.0, 1.0)).all()       # done flag
    assert (np.abs(rows[:, 2:4]) <= 5.0).all()          # stored actions are clipped
    for net in tr.td3.networks().values():
        assert torch.isfinite(net.params).all()


def test_fused_demo_reward_is_bit_identical():
    """nav_agent_step_indexed (tick + demo reward in one launch) vs nav_agent_step followed by
    nav_demo_reward_indexed: same replay rows, env state, rewards and learner, bit for bit."""
    from nav.trainer import VecTrainer
    runs = []
    for fused in (True, False):
        tr = VecTrainer(n_envs=8192, hidden=256, n_hidden=2, batch=4096, updates_per_step=2,
                        envs_per_group=1024, device=DEV)
        tr.env.fuse_demo = fused
        rewards = []
        for _ in range(5):
            tr.act()
            r = torch.full((tr.n,), float("nan"), dtype=torch.float64, device=DEV)
            tr.env.agent_step(tr.action, tr.replay, reward_out=r)
            tr.steps += 1
            tr.learn()
            rewards.append(r)
        torch.cuda.synchronize()
        runs.append((tr, torch.stack(rewards)))
    (a, ra), (b, rb) = runs
    assert torch.equal(a.replay.rows, b.replay.rows)
    assert torch.equal(a.env.state, b.env.state)
    assert torch.equal(a.env.flags, b.env.flags)
    assert torch.equal(ra.isnan(), rb.isnan()) and torch.equal(ra.nan_to_num(), rb.nan_to_num())
    assert (~ra.isnan()).any()  # some envs took the demo term
    for k, net in a.td3.networks().items():
        assert torch.equal(net.params, b.td3.networks()[k].params), k


# 40 000 envs: 625 row blocks, more than two workgroups per CU (512 on a 256-CU MI355X): a second
# wave of workgroups, and the GEMM priority of the grid's upper half (gemm_cols) on both
@pytest.mark.parametrize("n,demos", [(8192, True), (5000, True), (1000, False), (40000, True)])
def test_fused_act_tick_is_bit_identical(n, demos):
    """nav_act_tick (actor forward + the env tick in one launch) vs nav_act followed by
    nav_agent_step_indexed: same actions, replay rows, env state, flags, next states, rewards,
    block stats and learner, bit for bit, over ragged env counts and with / without demo sets."""
    from nav.trainer import VecTrainer
    runs = []
    for fused in (True, False):
        tr = VecTrainer(n_envs=n, hidden=256, n_hidden=2, batch=2048, updates_per_step=2,
                        envs_per_group=1024, demos=demos, device=DEV)
        got = []
        for _ in range(6):
            r = torch.full((tr.n,), float("nan"), dtype=torch.float64, device=DEV)
            if fused:
                tr.env.act_tick(tr.td3.actor_network, tr.steps, tr.replay, action_out=tr.action,
                                reward_out=r)
            else:
                tr.act()
                tr.env.agent_step(tr.action, tr.replay, reward_out=r)
            tr.steps += 1
            tr.learn()
            got.append((tr.action.clone(), r, tr.env.next_state.clone(), tr.env.goal_term.clone(),
                        tr.env.block_stats.clone()))
        torch.cuda.synchronize()
        runs.append((tr, got))
    (a, ga), (b, gb) = runs
    assert torch.equal(a.replay.rows, b.replay.rows)
    assert torch.equal(a.env.state, b.env.state)
    assert torch.equal(a.env.flags, b.env.flags)
    for t, (x, y) in enumerate(zip(ga, gb)):
        for i, (u, v) in enumerate(zip(x, y)):
            assert torch.equal(u.isnan(), v.isnan()), (t, i)
            assert torch.equal(u.nan_to_num(), v.nan_to_num()), (t, i)
    if demos:
        assert any((~g[1].isnan()).any() for g in ga)  # some envs took the demo term
    for k, net in a.td3.networks().items():
        assert torch.equal(net.params, b.td3.networks()[k].params), k


def test_td3_update_at_bench_config_vs_oracle():
    """The learner pinned at the bench configuration (2x256 actor/critics, batch 32 768, the
    bench's 2 epochs per step: critic, actor + Polyak, critic): TD3.td3_update with injected batch
    indices and smoothing noise vs the oracle's restatement of robot.py:258-398 on the CPU."""
    from test_gpu_shared_policy import make_learner, replay_rows, ring_of
    from oracle.td3_oracle import TD3Oracle, make_mlp_params
    B, hidden, nh, epochs = 32768, 256, 2, 2
    sizes = lambda di, do: [di] + [hidden] * nh + [do]  # noqa: E731
    params = (make_mlp_params(81, sizes(2, 2)), make_mlp_params(82, sizes(4, 1)),
              make_mlp_params(83, sizes(4, 1)))
    td3 = make_learner(B, hidden, nh, params)
    rows = replay_rows(4 * B, 9)
    rep = ring_of(rows)
    rng = np.random.default_rng(13)
    idx = [rng.integers(0, len(rows), B) for _ in range(epochs + (epochs + 1) // 2)]
    noise = [rng.standard_normal((B, 2)).astype(np.float32) for _ in range(epochs)]
    it = {"s": 0, "n": 0}

    def idx_fn():
        x = idx[it["s"]]; it["s"] += 1
        return torch.tensor(x, dtype=torch.int64, device=DEV)

    def eps_fn():
        x = noise[it["n"]]; it["n"] += 1
        return torch.tensor(x, device=DEV)

    td3.td3_update(rep, num_epochs=epochs, idx_fn=idx_fn, eps_fn=eps_fn, track_losses=True)
    torch.cuda.synchronize()
    ora = TD3Oracle(*params)
    it2 = {"s": 0, "n": 0}

    def sample():
        r = rows[idx[it2["s"]]]; it2["s"] += 1
        return r[:, 0:2], r[:, 2:4], r[:, 4], r[:, 5:7], r[:, 7] > 0.5

    def nz():
        x = noise[it2["n"]]; it2["n"] += 1
        return x

    closs, aloss = ora.td3_update(sample, nz, epochs)
    np.testing.assert_allclose(td3.critic_losses, np.mean(closs, 1), rtol=1e-4)
    np.testing.assert_allclose(td3.actor_losses, aloss, rtol=1e-4)
    mine = td3.networks()
    for name, onet in ora.networks().items():
        got = torch.cat([t.reshape(-1) for wb in mine[name].export() for t in wb])
        ref = torch.cat([t.reshape(-1) for wb in onet.params for t in wb])
        d = (got - ref).abs()
        # one Adam step moves a weight by ~lr = 1e-5: every entry within 2e-7 (measured on
        # MI355X: <= 3e-8; the two paths only differ in the order the batch rows are summed)
        print(f"{name}: max |diff| {float(d.max()):.3e}")
        assert float(d.max()) <= 2e-7, name


def _flat_vs_tensors(net, flat, ref_tensors, tag):
    """Compare a device-layout flat gradient with per-tensor reference gradients ([W0, b0, W1,
    ...] at logical sizes): every entry within rtol 1e-4 + 1e-6 of the tensor's max, padding
    exactly zero; returns (<g, g_ref>, |g_ref|^2) over the whole net."""
    from nav.mlp import layer_offsets
    offs, _ = layer_offsets(net.d_in, net.d_out, net.hp, net.n_hidden)
    dot, nrm = 0.0, 0.0
    for l, (w_off, b_off, fo, fi) in enumerate(offs):
        for ref, got in ((ref_tensors[2 * l], flat[w_off:w_off + fo * fi].view(fo, fi)),
                         (ref_tensors[2 * l + 1], flat[b_off:b_off + fo].view(fo))):
            ref = ref.detach().double()
            sl = tuple(slice(0, n) for n in ref.shape)
            g = got[sl].double()
            bad = (g - ref).abs() > 1e-4 * ref.abs() + 1e-6 * ref.abs().max()
            print(f"{tag} layer {l} {tuple(ref.shape)}: max rel {float(((g - ref).abs() / (ref.abs() + 1e-30)).max()):.2e}, "
                  f"outside tol {int(bad.sum())}")
            assert not bad.any(), (tag, l, tuple(ref.shape))
            pad = got.clone()
            pad[sl] = 0
            assert (pad == 0).all(), (tag, l)
            dot += float((g * ref).sum())
            nrm += float((ref * ref).sum())
    return dot, nrm


def test_learner_gradients_at_bench_config_vs_oracle():
    """The learner's gradients themselves at the bench configuration (2x256, B = 32 768: the
    64-row row-kernel form, 8 / 16 weight-gradient splits) against the oracle's autograd of
    robot.py:341-363 / 382-395 on the same batch and noise, BEFORE any Adam step — Adam's first
    step is lr * sign(g) and later ones are scale-invariant, so a parameter comparison cannot see
    a uniform gradient-scale error (a wrong 2/B, -1/B or split count); this does. The oracle uses
    the kernels' own ReLU decisions (pre-activations within rounding of 0 may branch either way).
    Every entry within rtol 1e-4; scale <g, g_ref> / |g_ref|^2 within 1e-5 of 1 per net."""
    from test_gpu_mlp import relu_bits
    from test_gpu_shared_policy import make_learner, replay_rows, ring_of
    from oracle.td3_oracle import TD3Oracle, make_mlp_params
    B, hidden, nh = 32768, 256, 2
    sizes = lambda di, do: [di] + [hidden] * nh + [do]  # noqa: E731
    params = (make_mlp_params(91, sizes(2, 2)), make_mlp_params(92, sizes(4, 1)),
              make_mlp_params(93, sizes(4, 1)))
    td3 = make_learner(B, hidden, nh, params)
    rows = replay_rows(4 * B, 19)
    rep = ring_of(rows)
    rng = np.random.default_rng(23)
    ic, ia = rng.integers(0, len(rows), B), rng.integers(0, len(rows), B)
    noise = rng.standard_normal((B, 2)).astype(np.float32)
    T = lambda x, dt=None: torch.tensor(x, dtype=dt, device=DEV)  # noqa: E731
    gc = td3.critic_gradients(rep, idx=T(ic, torch.int64), eps=T(noise)).cpu()
    hp = td3.critic_network_1.hp
    bits = {"c1": relu_bits(td3.mask1, nh, hp, hidden, B), "c2": relu_bits(td3.mask2, nh, hp, hidden, B)}
    ora = TD3Oracle(*params)
    r = rows[ic]
    ora.train_critic((r[:, 0:2], r[:, 2:4], r[:, 4], r[:, 5:7], r[:, 7] > 0.5), noise, bits=bits)
    cc = td3.critic_network_1.count
    for k, (key, net) in enumerate((("c1", td3.critic_network_1), ("c2", td3.critic_network_2))):
        dot, nrm = _flat_vs_tensors(net, gc[k * cc:(k + 1) * cc], ora.last_grads[key], key)
        print(f"{key}: scale {dot / nrm:.8f}")
        assert abs(dot / nrm - 1.0) <= 1e-5, key
    # the critics' Adam step from that bucket (train_critic's), then train_actor's gradient
    td3.critic_step()
    ga = td3.actor_gradients(rep, idx=T(ia, torch.int64)).cpu()
    bits = {"actor": relu_bits(td3.mask_a, nh, hp, hidden, B),
            "c1": relu_bits(td3.mask1, nh, hp, hidden, B)}
    ora.train_actor(rows[ia][:, 0:2], bits=bits)
    dot, nrm = _flat_vs_tensors(td3.actor_network, ga, ora.last_grads["actor"], "actor")
    print(f"actor: scale {dot / nrm:.8f}")
    assert abs(dot / nrm - 1.0) <= 1e-5
