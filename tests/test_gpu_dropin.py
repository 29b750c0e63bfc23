"""The N = 1 drop-ins (nav.Environment, nav.Robot) against the reference's own outputs: same numpy
seed -> same goal, region, start states, demonstrations, rewards and Robot counters."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def navmods():
    from nav import _lib
    _lib.require_gpu()
    from nav import environment, robot
    return environment, robot


def test_environment_seeding_bit_exact(navmods):
    environment, _ = navmods
    g = golden("rng_init.npz")
    d = golden("dynamics.npz")
    for k, seed in enumerate(g["seeds"]):
        np.random.seed(int(seed))
        env = environment.Environment(d["speed"], d["angle"])
        assert np.array_equal(np.asarray(env.robot_init_region, np.float64), g["region"][k])
        assert np.array_equal(np.asarray(env.goal_state, np.float64), g["goal"][k])
        for j in range(3):
            assert np.array_equal(env.reset(), g["resets"][k][j])
        assert np.array_equal(np.random.random_sample(4), g["tail"][k])


def test_environment_dynamics_and_step_api(navmods):
    environment, _ = navmods
    d = golden("dynamics.npz")
    np.random.seed(0)
    env = environment.Environment(d["speed"], d["angle"])
    for i in range(0, 300, 7):
        out = env.dynamics(list(d["state"][i]), list(d["action"][i]))  # graphics.py:224 form
        ref = d["dynamics"][i]
        if np.isnan(ref).any():
            assert np.isnan(out).any()
        else:
            assert np.max(np.abs(out - ref)) < 1e-11
        env.robot_state = d["state"][i].copy()
        before = env.robot_state
        after = env.step(d["action"][i])
        assert (after is before) == (not d["committed"][i])
        assert np.max(np.abs(after - d["step"][i])) < 1e-11


def ulps_f32(a, b):
    """|a - b| in float32 ulps (both finite float32 of one sign: positions in the world)."""
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def _trace_setup(environment, robot):
    t = golden("trace.npz")
    torch.manual_seed(0)
    np.random.seed(1707366464)
    env = environment.Environment(t["speed"], t["angle"])
    state = env.reset()
    rb = robot.Robot(env.goal_state)
    rb.td3_agent.td3_update = lambda memory: None  # as the trace generator did
    return t, env, state, rb


def test_demonstration_matches_reference(navmods):
    environment, robot = navmods
    t, env, state, rb = _trace_setup(environment, robot)
    assert np.array_equal(np.asarray(env.goal_state, np.float64), t["goal"])
    ds, da = env.get_demonstration()
    assert ds.dtype == np.float32 and ds.shape == (200, 2) and da.shape == (200, 2)
    assert np.array_equal(da, t["demo_actions"][0])
    # nav/demos.py's claim, checked: the GPU CEM's dynamics differs from numpy's by < 1e-14
    # before environment.py:179's float32 cast, which can move a state by at most one float32
    # ulp (<= 7.6e-6 in [64, 128): inside north_star's 1e-5)
    ref = t["demo_states"][0].astype(np.float32)
    assert np.all(ulps_f32(ds, ref) <= 1), int(ulps_f32(ds, ref).max())
    assert np.max(np.abs(ds.astype(np.float64) - ref)) <= 1e-5


def test_robot_replays_reference_trace(navmods):
    """robot-learning.py's loop with nav.Environment + nav.Robot, teacher-forced with the
    reference's actions (the actor weights differ): every numpy draw, reset, demonstration,
    reward, done flag and Robot counter must follow the reference's trace."""
    environment, robot = navmods
    t, env, state, rb = _trace_setup(environment, robot)
    types = t["tick_type"]
    pushes = []
    orig = rb.memory.advance

    def advance(n):
        pushes.append((rb.memory.position, n))
        return orig(n)

    rb.memory.advance = advance
    c = t["counters"]
    for i in range(len(types)):
        at = rb.get_next_action_type(state, 100.0)
        assert {"step": 0, "demo": 1, "reset": 2}[at] == types[i], i
        if at == "reset":
            state = env.reset()
            assert np.array_equal(state, t["tick_next"][i]), i
        elif at == "demo":
            ds, da = env.get_demonstration()
            rb.process_demonstration(ds, da, 100.0)
        else:
            rb.get_next_action_training(state, 100.0)  # consumes the same noise draws
            a = t["tick_action"][i]
            ns = env.step(a)
            assert np.max(np.abs(ns - t["tick_next"][i])) < 1e-9, i
            rb.process_transition(state, a, ns, 100.0)
            state = ns
            lo = t["push_idx"][i][0]
            slot, n = pushes[-1]
            row = rb.memory.rows[slot].cpu().numpy()
            ref_r = t["push_r"][lo]
            assert abs(row[4] - ref_r) <= 1e-4 * max(1.0, abs(ref_r)), i
            assert row[7] == float(t["push_d"][lo])
        cc = c[i]
        assert (rb.plan_index, rb.path_length, rb.num_episodes) == (cc[0], cc[1], cc[2]), i
        assert (int(rb.goal_reached), int(rb.stuck_flag), int(rb.demo_flag)) == \
            (cc[3], cc[4], cc[5]), i
        assert rb.current_noise_scale == cc[6]
    assert len(rb.demonstration_states) == len(t["demo_set"])
    got = np.asarray([np.asarray(x, np.float64) for x in rb.demonstration_states])
    # the originals are the CEM's float32 states (<= 1 ulp, above); an augmented point is a
    # float32 interpolation of two of them plus float64 noise (robot.py:795-816), so it moves
    # by at most what one ulp of its endpoints moves the interpolation: north_star's 1e-5
    err = np.abs(got - t["demo_set"])
    print(f"demo set: max |diff| {err.max():.3e}, exact {np.mean(err == 0):.4f}")
    assert err.max() <= 1e-5
    assert len(rb.memory) == len(t["push_r"])


def test_td3_update_dropin_runs(navmods):
    """robot.py's TD3.td3_update(memory) end to end: 100 epochs, batch 100, numpy-drawn
    permutations, finite weights afterwards."""
    environment, robot = navmods
    rb = robot.Robot(np.array([60.0, 40.0]))
    rng = np.random.default_rng(0)
    for _ in range(300):
        s = rng.uniform(0, 100, 2)
        rb.memory.push(s, rng.uniform(-5, 5, 2), rng.uniform(-100, 0), s + 1, False)
    np.random.seed(3)
    rb.td3_agent.td3_update(rb.memory)
    torch.cuda.synchronize()
    for net in rb.td3_agent.networks().values():
        assert torch.isfinite(net.params).all()
    assert rb.td3_agent.actor_optimizer.step_count == 50
    assert rb.td3_agent.critic_optimizer_1.step_count == 100
    st = rb.memory.sample(100)
    assert st[0].shape == (100, 2) and st[4].dtype == bool


def test_td3_update_predrawn_equals_per_epoch_draws(navmods):
    """The drop-in's td3_update takes every epoch's np.random.choice / torch.randn draws up
    front; the parameters equal an update that draws them lazily at each train_critic /
    train_actor call, as robot.py:300-333 / 386-390 do, bit for bit."""
    from nav.td3 import TD3 as GpuTD3
    environment, robot = navmods
    rng = np.random.default_rng(0)
    rows = [(s, rng.uniform(-5, 5, 2), rng.uniform(-100, 0), s + 1, False)
            for s in rng.uniform(0, 100, (400, 2))]
    robots = []
    for _ in range(2):
        rb = robot.Robot(np.array([60.0, 40.0]))
        for r in rows:
            rb.memory.push(*r)
        robots.append(rb)
    a, b = robots
    for k, net in a.td3_agent.networks().items():  # same initial networks
        b.td3_agent.networks()[k].params.copy_(net.params)
        b.td3_agent.networks()[k].pack()
    np.random.seed(11)
    torch.manual_seed(12)
    a.td3_agent.td3_update(a.memory)
    np.random.seed(11)
    torch.manual_seed(12)
    B, mem = 100, b.memory

    def idx_fn():
        return torch.as_tensor(np.random.choice(len(mem), B, replace=False), dtype=torch.int64,
                               device="cuda")
    GpuTD3.td3_update(b.td3_agent, mem, 100, idx_fn=idx_fn,
                      eps_fn=lambda: torch.randn(B, 2).to("cuda"))
    torch.cuda.synchronize()
    for k, net in a.td3_agent.networks().items():
        assert torch.equal(net.params, b.td3_agent.networks()[k].params), k


def test_headless_driver_short_run(navmods):
    from nav import driver
    d = golden("dynamics.npz")
    r = driver.run(seed=5, max_ticks=40, budget=False, verbose=False,
                   env_kwargs={"speed": d["speed"], "angle": d["angle"]})
    assert r["demos"] == 3 and r["steps"] > 0 and r["ticks"] == 40


def test_headless_driver_with_learner(navmods):
    """config 1 in small: the loop through the demos into training episodes, td3_update (100
    epochs of batch 100, robot.py:258-285) running at every episode end, budget off."""
    import torch
    from nav import driver
    from nav.robot import Robot
    d = golden("dynamics.npz")
    updates = []

    class CountingRobot(Robot):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.init_actor = self.td3_agent.actor_network.params.clone()
            inner = self.td3_agent.td3_update

            def counted(buf):
                inner(buf)
                updates.append(len(buf))
            self.td3_agent.td3_update = counted

    r = driver.run(robot_cls=CountingRobot, seed=5, budget=False, verbose=False,
                   max_episodes=8, env_kwargs={"speed": d["speed"], "angle": d["angle"]})
    robot = r["robot"]
    assert r["demos"] == 3 and robot.num_episodes == 8 and r["mode"] == "training"
    assert len(updates) >= 3  # an update at every training episode end
    # the replay holds the demos' transitions and every training step
    assert len(robot.memory) == 3 * 199 + r["steps"]
    assert updates == sorted(updates) and updates[0] >= 3 * 199
    nets = robot.td3_agent.networks()
    assert all(torch.isfinite(n.params).all() for n in nets.values())
    # the actor moved away from its initial parameters
    assert not torch.equal(robot.init_actor, nets["actor"].params)


def test_td3_update_live_hyperparams_vs_oracle(navmods):
    """robot.py's td3_update reads self.gamma / tau / policy_noise / noise_clip / max_action /
    batch_size / num_epochs at every call (robot.py:258-339): the drop-in copies the agent's live
    attributes into its learner config before each update. Two updates with every one of them
    changed in between (including the batch size, which rebuilds the workspace and the cached
    launch arguments) against the oracle run on the same numpy / torch draws: all six networks
    within 5e-7 (Adam moves a weight by ~lr = 1e-5 per step)."""
    from oracle.td3_oracle import TD3Oracle
    environment, robot = navmods
    rng = np.random.default_rng(5)
    rb = robot.Robot(np.array([60.0, 40.0]))
    for s in rng.uniform(0, 100, (400, 2)):
        rb.memory.push(s, rng.uniform(-5, 5, 2), rng.uniform(-100, 0), s + rng.normal(0, 1, 2),
                       bool(rng.uniform() < 0.1))
    ag = rb.td3_agent
    nets = ag.networks()
    init = {k: [(W.numpy(), b.numpy()) for W, b in nets[k].export()]
            for k in ("actor", "critic1", "critic2")}
    ora = TD3Oracle(init["actor"], init["critic1"], init["critic2"], actor_lr=ag.cfg.actor_lr,
                    critic_lr=ag.cfg.critic_lr, gamma=ag.gamma, tau=ag.tau,
                    policy_noise=ag.policy_noise, noise_clip=ag.noise_clip,
                    policy_update_delay=ag.policy_update_delay, max_action=ag.max_action)
    rows = rb.memory.rows[:len(rb.memory)].cpu().numpy().astype(np.float64)
    L = len(rows)
    plans = [dict(seed=(11, 12), num_epochs=4),
             dict(seed=(13, 14), num_epochs=3, gamma=0.9, tau=0.01, policy_noise=0.3,
                  noise_clip=0.4, max_action=2.0, batch_size=64)]
    for plan in plans:
        for k in ("gamma", "tau", "policy_noise", "noise_clip", "max_action", "batch_size",
                  "num_epochs"):
            if k in plan:
                setattr(ag, k, plan[k])
        np.random.seed(plan["seed"][0])
        torch.manual_seed(plan["seed"][1])
        ag.td3_update(rb.memory)
        torch.cuda.synchronize()
        # the oracle on the same draws: np.random.choice per critic / actor sample in epoch
        # order, torch.randn(B, 2) per critic epoch
        ora.gamma, ora.tau, ora.max_action = ag.gamma, ag.tau, ag.max_action
        ora.policy_noise, ora.noise_clip = ag.policy_noise, ag.noise_clip
        B = ag.batch_size
        np.random.seed(plan["seed"][0])
        torch.manual_seed(plan["seed"][1])

        def sample():
            r = rows[np.random.choice(L, B, replace=False)]
            return r[:, 0:2], r[:, 2:4], r[:, 4], r[:, 5:7], r[:, 7] > 0.5

        ora.td3_update(sample, lambda: torch.randn(B, 2).numpy(), ag.num_epochs)
    worst = 0.0
    for name, onet in ora.networks().items():
        for (W, b), (Wr, br) in zip(nets[name].export(), onet.params):
            d = max(float((W - Wr).abs().max()), float((b - br).abs().max()))
            worst = max(worst, d)
            assert d <= 5e-7, (name, d)
    print(f"max |diff| vs oracle after both updates: {worst:.2e}")
    assert ag.cfg.max_action == 2.0 and ag.cfg.batch_size == 64 and ag.cfg.gamma == 0.9
