"""TEST INFRASTRUCTURE ONLY — torch-CPU fp32 restatement of the reference's residual-TD3 learner.

Restates robot.py:128-206 (networks), :209-398 (TD3: train_critic, train_actor, soft_update, Adam,
MSE) with every random input injectable (batch indices, target-smoothing noise) so that the HIP
path can be compared on identical inputs. Pinned against tests/golden/td3.npz, which was produced by
running the reference's own TD3 class on the same injected inputs (tests/golden/make_golden.py).

Only tests/ and bench.py's cpu_baseline leg use this module.
"""
import math

import numpy as np
import torch


def make_mlp_params(seed, sizes, bias_scale=0.1):
    """Documented counter-free generator for test weights: numpy default_rng(seed), layer by layer,
    W ~ U(-sqrt(6/fan_in), +sqrt(6/fan_in)) [out, in] (the Kaiming-uniform bound of robot.py:164),
    b ~ U(-bias_scale, bias_scale). Returns a list of (W, b) float32 numpy arrays."""
    rng = np.random.default_rng(seed)
    params = []
    for fan_in, fan_out in zip(sizes[:-1], sizes[1:]):
        bound = math.sqrt(6.0 / fan_in)
        W = rng.uniform(-bound, bound, (fan_out, fan_in)).astype(np.float32)
        b = rng.uniform(-bias_scale, bias_scale, fan_out).astype(np.float32)
        params.append((W, b))
    return params


class MLP:
    """ReLU MLP, linear output (robot.py:153-159 / 193-200)."""

    def __init__(self, params):
        self.params = [(torch.tensor(W).clone(), torch.tensor(b).clone()) for W, b in params]

    def clone(self):
        m = MLP.__new__(MLP)
        m.params = [(W.clone(), b.clone()) for W, b in self.params]
        return m

    def tensors(self):
        out = []
        for W, b in self.params:
            out += [W, b]
        return out

    def forward(self, x, bits=None):
        """bits (optional, test injection): per hidden layer a bool [rows][width] ReLU decision
        to use instead of (z > 0) — h = z * bits — so a gradient comparison is not moved by a
        pre-activation within rounding of 0 taking the other branch (the values differ from
        relu(z) only inside that band)."""
        h = x
        n = len(self.params)
        for i, (W, b) in enumerate(self.params):
            h = torch.nn.functional.linear(h, W, b)
            if i < n - 1:
                h = torch.relu(h) if bits is None else h * bits[i].to(h.dtype)
        return h


class Adam:
    """torch.optim.Adam defaults restated (lr given, betas .9/.999, eps 1e-8, no weight decay)."""

    def __init__(self, tensors, lr, betas=(0.9, 0.999), eps=1e-8):
        self.t = tensors
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = [torch.zeros_like(x) for x in tensors]
        self.v = [torch.zeros_like(x) for x in tensors]
        self.step_count = 0

    def step(self, grads):
        self.step_count += 1
        bc1 = 1 - self.b1 ** self.step_count
        bc2 = 1 - self.b2 ** self.step_count
        step_size = self.lr / bc1
        bc2_sqrt = math.sqrt(bc2)
        with torch.no_grad():
            for p, g, m, v in zip(self.t, grads, self.m, self.v):
                m.lerp_(g, 1 - self.b1)
                v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                denom = (v.sqrt() / bc2_sqrt).add_(self.eps)
                p.addcdiv_(m, denom, value=-step_size)


class TD3Oracle:
    def __init__(self, actor_params, critic1_params, critic2_params, actor_lr=1e-5, critic_lr=1e-5,
                 gamma=0.99, tau=0.001, policy_noise=0.2, noise_clip=0.5, policy_update_delay=2,
                 max_action=5.0):
        self.actor = MLP(actor_params)
        self.critic1 = MLP(critic1_params)
        self.critic2 = MLP(critic2_params)
        self.target_actor = self.actor.clone()
        self.target_critic1 = self.critic1.clone()
        self.target_critic2 = self.critic2.clone()
        self.opt_actor = Adam(self.actor.tensors(), actor_lr)
        self.opt_c1 = Adam(self.critic1.tensors(), critic_lr)
        self.opt_c2 = Adam(self.critic2.tensors(), critic_lr)
        self.gamma, self.tau = gamma, tau
        self.policy_noise, self.noise_clip = policy_noise, noise_clip
        self.delay, self.max_action = policy_update_delay, max_action
        self.last_grads = {}

    @staticmethod
    def _q(net, s, a, bits=None):
        return net.forward(torch.cat([s, a], dim=1), bits)

    def train_critic(self, batch, noise, bits=None):
        """robot.py:312-366. batch = (s, a, r, s2, d) numpy; noise = standard normal [B,2] f32;
        bits (optional): {"c1": [...], "c2": [...]} injected ReLU decisions of the online critics
        (MLP.forward)."""
        s, a, r, s2, d = batch
        s = torch.tensor(np.asarray(s), dtype=torch.float32)
        a = torch.tensor(np.asarray(a), dtype=torch.float32)
        r = torch.tensor(np.asarray(r), dtype=torch.float32).unsqueeze(1)
        s2 = torch.tensor(np.asarray(s2), dtype=torch.float32)
        nd = torch.tensor(1 - np.asarray(d).astype(np.int64), dtype=torch.float32).unsqueeze(1)
        with torch.no_grad():
            eps = (torch.tensor(noise) * self.policy_noise).clamp(-self.noise_clip, self.noise_clip)
            a2 = (self.target_actor.forward(s2) + eps).clamp(-self.max_action, self.max_action)
            q1t = self._q(self.target_critic1, s2, a2)
            q2t = self._q(self.target_critic2, s2, a2)
            y = r + self.gamma * torch.min(q1t, q2t) * nd
        losses = []
        for net, opt, key in ((self.critic1, self.opt_c1, "c1"), (self.critic2, self.opt_c2, "c2")):
            ts = net.tensors()
            for t in ts:
                t.requires_grad_(True)
            q = self._q(net, s, a, None if bits is None else bits[key])
            loss = torch.nn.functional.mse_loss(q, y)
            grads = torch.autograd.grad(loss, ts)
            for t in ts:
                t.requires_grad_(False)
            self.last_grads[key] = [g.clone() for g in grads]
            opt.step(grads)
            losses.append(loss.item())
        self.last_y = y.squeeze(1).clone()
        return losses

    def train_actor(self, states, bits=None):
        """robot.py:369-398 (critic-1 grads are discarded, as zero_grad does in the reference);
        bits (optional): {"actor": [...], "c1": [...]} injected ReLU decisions (MLP.forward)."""
        s = torch.tensor(np.asarray(states), dtype=torch.float32)
        ts = self.actor.tensors()
        for t in ts:
            t.requires_grad_(True)
        a = self.actor.forward(s, None if bits is None else bits["actor"])
        loss = -self._q(self.critic1, s, a, None if bits is None else bits["c1"]).mean()
        grads = torch.autograd.grad(loss, ts)
        for t in ts:
            t.requires_grad_(False)
        self.last_grads["actor"] = [g.clone() for g in grads]
        self.opt_actor.step(grads)
        return loss.item()

    def soft_update(self):
        """robot.py:293-310: theta' = theta' * (1 - tau) + theta * tau per tensor."""
        with torch.no_grad():
            for tgt, src in ((self.target_actor, self.actor), (self.target_critic1, self.critic1),
                             (self.target_critic2, self.critic2)):
                for tp, sp in zip(tgt.tensors(), src.tensors()):
                    tp.copy_(tp * (1.0 - self.tau) + sp * self.tau)

    def td3_update(self, sample_fn, noise_fn, num_epochs):
        """robot.py:258-285 with the sampler and the randn source injected."""
        closs, aloss = [], []
        for epoch in range(num_epochs):
            closs.append(self.train_critic(sample_fn(), noise_fn()))
            if epoch % self.delay == 0:
                aloss.append(self.train_actor(sample_fn()[0]))
                self.soft_update()
        return closs, aloss

    def networks(self):
        return {"actor": self.actor, "critic1": self.critic1, "critic2": self.critic2,
                "target_actor": self.target_actor, "target_critic1": self.target_critic1,
                "target_critic2": self.target_critic2}


def param_digest(net, n_samples=64, seed=99):
    """Per-tensor (sum, sum of squares, sampled entries) in float64: the compact fixture form."""
    rng = np.random.default_rng(seed)
    out = []
    for t in net.tensors() if hasattr(net, "tensors") else net:
        a = t.detach().double().numpy().ravel() if torch.is_tensor(t) else np.asarray(t).ravel()
        idx = rng.integers(0, a.size, n_samples)
        out.append((a.sum(), (a * a).sum(), idx, a[idx]))
    return out
