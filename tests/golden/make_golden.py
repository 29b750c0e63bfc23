"""Generate the committed golden fixtures by running the REFERENCE itself (container-only).

Imports /root/reference/environment.py and robot.py with two stub modules for dependencies that are
absent from the image: `pyglet` (graphics only; reached through robot.py:19 -> graphics.PathToDraw)
and `perlin_noise` (environment.py:7, used only by set_dynamics). The dynamics fields are injected
instead of generated, so every vector below is exercised through the reference's own code.

Writes small .npz files next to this script:
  dynamics.npz  Environment.dynamics/step on 4096 (state, action) cases incl. NaN/inf/clip/edges
  rng_init.npz  np.random.seed(s) -> set_init_and_goal + 3 resets, 32 seeds, + stream position
  trace.npz     headless robot-learning.py tick loop (3 CEM demos + 400 training ticks): the demo
                set, per-step (s, a, r, s', done), tick types, Robot counters and flags
  actions.npz   Robot.get_next_action_training/testing with generator-defined actor weights
  td3.npz       TD3.td3_update(4 epochs) with generator weights, injected batches and randn noise
  td3_grads.npz the same run's first param.grad of each optimizer (train_critic's two
                loss.backward(), robot.py:355-363; train_actor's, robot.py:393-395): the small
                tensors whole, the hidden x hidden weights as 4096 sampled entries + digests

Usage: python tests/golden/make_golden.py   (skips cleanly when /root/reference is absent)
"""
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))


def import_reference():
    sys.path.insert(0, REF)
    sys.modules.setdefault("pyglet", types.ModuleType("pyglet"))
    pn = types.ModuleType("perlin_noise")

    class PerlinNoise:  # never called: fields are injected
        def __init__(self, octaves=1, seed=None):
            raise RuntimeError("perlin_noise is not available; inject dynamics fields")

    pn.PerlinNoise = PerlinNoise
    sys.modules["perlin_noise"] = pn
    import environment  # noqa: E402
    import robot  # noqa: E402
    return environment, robot


def make_fields(seed):
    """Synthetic fields with the value ranges set_dynamics produces (speed = sigmoid-stretched in
    (0,1), angle in [0,1]); float32 [100,100], x-major like environment.py:67-95."""
    rng = np.random.default_rng(seed)
    x = np.linspace(0, 1, 100)
    base = np.zeros((100, 100))
    for k in range(1, 6):
        ph = rng.uniform(0, 2 * np.pi, 2)
        base += rng.uniform(0.2, 1.0) * np.outer(np.sin(2 * np.pi * k * x + ph[0]),
                                                  np.cos(2 * np.pi * k * x + ph[1]))
    base += 0.3 * rng.standard_normal((100, 100))
    n = (base - base.min()) / (base.max() - base.min())
    speed = (1 / (1 + np.exp(-10 * (n - 0.5)))).astype(np.float32)
    ang = rng.standard_normal((100, 100)).cumsum(0).cumsum(1)
    angle = ((ang - ang.min()) / (ang.max() - ang.min())).astype(np.float32)
    return speed, angle


def new_env(environment, speed, angle):
    e = environment.Environment.__new__(environment.Environment)
    e.robot_state = np.array([0.0, 0.0], dtype=np.float32)
    e.robot_init_region = np.array([0.0, 0.0, 0.0, 0.0], dtype=np.float32)
    e.goal_state = np.array([0.0, 0.0], dtype=np.float32)
    e.dynamics_speed = speed
    e.dynamics_angle = angle
    return e


def gen_dynamics(environment):
    speed, angle = make_fields(1)
    env = new_env(environment, speed, angle)
    rng = np.random.default_rng(2)
    K = 4096
    s = rng.uniform(0, 100, (K, 2))
    a = rng.uniform(-7, 7, (K, 2))
    # edge cases: integer cell boundaries, world edges, the clip value, [99,100) reachable by reset
    s[:64] = np.floor(s[:64])
    s[64:128] = np.floor(s[64:128]) + 1 - 1e-9
    s[128:136] = [[0, 0], [98.9999, 98.9999], [0, 98.9999], [98.9999, 0], [99.5, 99.9], [99.99, 3],
                  [50, 50], [1e-300, 5]]
    a[136:144] = [[np.nan, 1], [1, np.nan], [np.inf, 0], [-np.inf, -np.inf], [0, 0], [5, 5],
                  [-5, 5], [1e9, -1e9]]
    a[144:208] = rng.uniform(-0.01, 0.01, (64, 2))  # tiny moves
    a[208:272] = rng.uniform(-300, 300, (64, 2))  # heavy clipping
    dyn = np.zeros((K, 2))
    stepped = np.zeros((K, 2))
    committed = np.zeros(K, np.int8)
    for i in range(K):
        dyn[i] = env.dynamics(s[i].copy(), a[i].copy())
        env.robot_state = s[i].copy()
        before = env.robot_state
        out = env.step(a[i].copy())
        stepped[i] = out
        committed[i] = 0 if out is before else 1
    np.savez_compressed(os.path.join(OUT, "dynamics.npz"), speed=speed, angle=angle, state=s,
                        action=a, dynamics=dyn, step=stepped, committed=committed)


def gen_rng_init(environment):
    seeds = np.array([1707366464, 0, 1, 2, 3, 42, 7, 99, 123, 1000, 2024, 31337] +
                     list(range(10, 30)), np.uint32)
    regions, goals, resets, tails = [], [], [], []
    speed, angle = make_fields(1)
    for sd in seeds:
        np.random.seed(int(sd))
        env = new_env(environment, speed, angle)
        env.set_init_and_goal()
        regions.append(np.asarray(env.robot_init_region, np.float64))
        goals.append(np.asarray(env.goal_state, np.float64))
        resets.append([env.reset().copy() for _ in range(3)])
        tails.append(np.random.random_sample(4))
    np.savez_compressed(os.path.join(OUT, "rng_init.npz"), seeds=seeds, region=np.array(regions),
                        goal=np.array(goals), resets=np.array(resets), tail=np.array(tails))


def gen_trace(environment, robot, n_ticks=400):
    """Headless copy of robot-learning.py:54-101 with the money budget removed; torch seeded only to
    make this generator reproducible; td3_update stubbed (it consumes no numpy draws, and the trace
    records the actions, so the learner does not influence what is checked)."""
    import torch
    torch.manual_seed(0)
    np.random.seed(1707366464)
    speed, angle = make_fields(3)
    env = new_env(environment, speed, angle)
    env.set_init_and_goal()
    state = env.reset()
    rb = robot.Robot(env.goal_state)
    rb.td3_agent.td3_update = lambda memory: None
    pushes = []
    orig_push = rb.memory.push

    def push(s, a, r, s2, d):
        pushes.append((np.array(s, np.float64), np.array(a, np.float64), float(r),
                       np.array(s2, np.float64), bool(d)))
        orig_push(s, a, r, s2, d)

    rb.memory.push = push
    types_, tick_state, tick_action, tick_next, push_idx = [], [], [], [], []
    ctr = []  # after each tick: plan_index, path_length, num_episodes, goal, stuck, demo, noise
    demos = []
    for _ in range(n_ticks):
        t = rb.get_next_action_type(state, 100.0)
        types_.append({"step": 0, "demo": 1, "reset": 2}[t])
        a = np.full(2, np.nan)
        ns = np.full(2, np.nan)
        s_in = np.array(state, np.float64)
        k_before = len(pushes)
        if t == "reset":
            state = env.reset()
            ns = np.array(state, np.float64)
        elif t == "demo":
            ds, da = env.get_demonstration()
            demos.append((ds.copy(), da.copy()))
            rb.process_demonstration(ds, da, 100.0)
        else:
            a = rb.get_next_action_training(state, 100.0)
            ns_ = env.step(a)
            rb.process_transition(state, a, ns_, 100.0)
            state = ns_
            ns = np.array(ns_, np.float64)
        tick_state.append(s_in)
        tick_action.append(np.array(a, np.float64))
        tick_next.append(ns)
        push_idx.append((k_before, len(pushes)))
        ctr.append((rb.plan_index, rb.path_length, rb.num_episodes, int(rb.goal_reached),
                    int(rb.stuck_flag), int(rb.demo_flag), rb.current_noise_scale))
    demo_set = np.array([np.asarray(x, np.float64) for x in rb.demonstration_states])
    P = pushes
    np.savez_compressed(
        os.path.join(OUT, "trace.npz"), speed=speed, angle=angle,
        goal=np.asarray(env.goal_state, np.float64),
        region=np.asarray(env.robot_init_region, np.float64), demo_set=demo_set,
        demo_states=np.array([d[0] for d in demos]), demo_actions=np.array([d[1] for d in demos]),
        tick_type=np.array(types_, np.int8), tick_state=np.array(tick_state),
        tick_action=np.array(tick_action), tick_next=np.array(tick_next),
        push_idx=np.array(push_idx, np.int32),
        push_s=np.array([p[0] for p in P]), push_a=np.array([p[1] for p in P]),
        push_r=np.array([p[2] for p in P]), push_s2=np.array([p[3] for p in P]),
        push_d=np.array([p[4] for p in P]), counters=np.array(ctr, np.float64))


def load_net(net, params):
    import torch
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    assert len(layers) == len(params)
    with torch.no_grad():
        for lin, (W, b) in zip(layers, params):
            lin.weight.copy_(torch.tensor(W))
            lin.bias.copy_(torch.tensor(b))


def gen_actions(environment, robot):
    sys.path.insert(0, ROOT)
    from oracle.td3_oracle import make_mlp_params
    import torch
    torch.manual_seed(0)
    actor_p = make_mlp_params(11, [2, 200, 200, 200, 2])
    rb = robot.Robot(np.array([60.0, 40.0]))
    load_net(rb.td3_agent.actor_network, actor_p)
    rng = np.random.default_rng(5)
    K = 64
    states = rng.uniform(0, 100, (K, 2))
    goals = rng.uniform(5, 95, (K, 2))
    sigmas = 0.75 ** rng.integers(0, 12, K)
    seeds = rng.integers(0, 2**31, K)
    a_tr, a_te, res, z = [], [], [], []
    for i in range(K):
        rb.goal_state = goals[i]
        rb.current_noise_scale = float(sigmas[i])
        np.random.seed(int(seeds[i]))
        a_tr.append(rb.get_next_action_training(states[i].copy(), 0.0))
        np.random.seed(int(seeds[i]))
        z.append(np.random.normal(0, 1, 2))
        a_te.append(rb.get_next_action_testing(states[i].copy()))
        res.append(rb.residual_action(states[i] - goals[i]))
    np.savez_compressed(os.path.join(OUT, "actions.npz"), actor_seed=11, states=states, goals=goals,
                        sigmas=sigmas, action_train=np.array(a_tr), action_test=np.array(a_te),
                        residual=np.array(res, np.float32), z=np.array(z))


def gen_td3(robot, epochs=4, B=100, n_trans=300):
    sys.path.insert(0, ROOT)
    from oracle.td3_oracle import make_mlp_params, param_digest
    import torch
    torch.manual_seed(0)
    pa = make_mlp_params(21, [2, 200, 200, 200, 2])
    p1 = make_mlp_params(22, [4, 200, 200, 200, 1])
    p2 = make_mlp_params(23, [4, 200, 200, 200, 1])
    actor, c1, c2 = robot.Residual_Actor_Network(), robot.Residual_Critic_Network(), \
        robot.Residual_Critic_Network()
    load_net(actor, pa)
    load_net(c1, p1)
    load_net(c2, p2)
    agent = robot.TD3(actor, c1, c2)
    rng = np.random.default_rng(31)
    S = rng.uniform(0, 100, (n_trans, 2))
    A = rng.uniform(-5, 5, (n_trans, 2))
    R = rng.uniform(-500, 50, n_trans)
    S2 = np.clip(S + rng.uniform(-4, 4, (n_trans, 2)), 0, 98.9999)
    D = rng.random(n_trans) < 0.1
    n_samples = epochs + (epochs + 1) // 2
    idx = np.stack([rng.permutation(n_trans)[:B] for _ in range(n_samples)]).astype(np.int32)
    noise = rng.standard_normal((epochs, B, 2)).astype(np.float32)
    it = {"s": 0, "n": 0}

    class Buf:
        def sample(self, bs):
            i = idx[it["s"]]
            it["s"] += 1
            return S[i], A[i], R[i], S2[i], D[i]

    orig = torch.randn_like

    def fake_randn_like(x):
        t = torch.tensor(noise[it["n"]])
        it["n"] += 1
        return t

    closs, aloss = [], []
    agent_train_critic, agent_train_actor = agent.train_critic, agent.train_actor
    # the gradients the reference forms in loss.backward(), read at each optimizer's first step
    first_grads = {}

    def record(name, opt):
        step = opt.step

        def wrapped(*a, **k):
            if name not in first_grads:
                first_grads[name] = [p.grad.detach().clone() for g in opt.param_groups
                                     for p in g["params"]]
            return step(*a, **k)
        opt.step = wrapped

    record("critic1", agent.critic_optimizer_1)
    record("critic2", agent.critic_optimizer_2)
    record("actor", agent.actor_optimizer)

    def tc(rb):
        r = agent_train_critic(rb)
        closs.append(r)
        return r

    def ta(rb):
        r = agent_train_actor(rb)
        aloss.append(r)
        return r

    agent.train_critic, agent.train_actor = tc, ta
    agent.num_epochs = epochs
    torch.randn_like = fake_randn_like
    try:
        agent.td3_update(Buf())
    finally:
        torch.randn_like = orig
    nets = {"actor": agent.actor_network, "critic1": agent.critic_network_1,
            "critic2": agent.critic_network_2, "target_actor": agent.target_actor,
            "target_critic1": agent.target_critic_network_1,
            "target_critic2": agent.target_critic_network_2}
    out = dict(epochs=epochs, B=B, S=S, A=A, R=R, S2=S2, D=D, idx=idx, noise=noise,
               critic_loss=np.array(closs), actor_loss=np.array(aloss))
    for name, net in nets.items():
        dig = param_digest(list(net.parameters()))
        out[name + "_sum"] = np.array([d[0] for d in dig])
        out[name + "_sq"] = np.array([d[1] for d in dig])
        out[name + "_idx"] = np.array([d[2] for d in dig])
        out[name + "_val"] = np.array([d[3] for d in dig])
    probe = rng.uniform(0, 100, (16, 2)).astype(np.float32)
    probe_a = rng.uniform(-5, 5, (16, 2)).astype(np.float32)
    with torch.no_grad():
        out["probe_s"] = probe
        out["probe_a"] = probe_a
        out["probe_actor"] = agent.actor_network(torch.tensor(probe)).numpy()
        out["probe_q1"] = agent.critic_network_1(torch.tensor(probe), torch.tensor(probe_a)).numpy()
    np.savez_compressed(os.path.join(OUT, "td3.npz"), **out)
    gout = dict(critic_idx=idx[0], actor_idx=idx[1], noise=noise[0])
    grng = np.random.default_rng(99)
    for name, grads in first_grads.items():
        for t, g in enumerate(grads):
            a = g.numpy().astype(np.float32)
            key = f"{name}_{t}"
            if a.size <= 1024:
                gout[key] = a
            else:  # a hidden x hidden weight: sampled entries + whole-tensor digests
                ix = grng.integers(0, a.size, 4096)
                proj = np.random.default_rng(1000 + t).standard_normal(a.size)
                gout[key + "_idx"] = ix
                gout[key + "_val"] = a.ravel()[ix]
                gout[key + "_shape"] = np.array(a.shape)
                gout[key + "_dig"] = np.array([a.astype(np.float64).sum(),
                                               (a.astype(np.float64) ** 2).sum(),
                                               (a.astype(np.float64).ravel() * proj).sum()])
    np.savez_compressed(os.path.join(OUT, "td3_grads.npz"), **gout)


def main():
    if not os.path.isdir(REF):
        print("reference absent; fixtures are committed, nothing to do")
        return
    environment, robot = import_reference()
    gen_dynamics(environment)
    gen_rng_init(environment)
    gen_actions(environment, robot)
    gen_td3(robot)
    gen_trace(environment, robot)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
