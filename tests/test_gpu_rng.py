"""Distribution checks of the vector path's counter-based randomness (Philox4x32-10 keyed by the
run seed): the learner's with-replacement replay sampling (robot.py:98-115 draws a permutation
prefix; the vector path draws uniform indices), the target-policy smoothing noise
(robot.py:338-339: clamp(0.2 z, +-0.5)) and the exploration noise (robot.py:614-620:
noise_scale * max_action * z). The N = 1 drop-in consumes numpy's stream instead and is pinned bit
for bit elsewhere; here the statistics are the contract. Each test reads the kernels' outputs with
the networks zeroed so the outputs expose the draws directly. Thresholds: p > 1e-4 for the
chi-square / KS tests (fixed seeds, so the outcome is deterministic), moments within 5 standard
errors."""
import ctypes as C

import numpy as np
import pytest
import torch
from scipy import stats

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def nav():
    from nav import _lib
    _lib.require_gpu()
    _lib.lib()
    torch.cuda.set_device(0)


def _zero_net(d_in, d_out, hidden=64, nh=2):
    from nav.mlp import DeviceMLP
    net = DeviceMLP(d_in, d_out, hidden, nh, DEV)
    net.params.zero_()
    net.pack()
    return net


def test_replay_sampling_uniform_with_replacement(nav):
    """train_critic's and train_actor's Philox batches: every index of the ring equally likely,
    the two batches of one epoch and of consecutive epochs different streams."""
    from nav import config as K
    from nav._lib import stream_handle
    from nav.td3 import TD3
    from nav.vec_env import ReplayRing
    size, B = 1000, 32768
    cfg = K.TD3Config(batch_size=B, num_epochs=1, net=K.NetConfig(hidden=64, n_hidden=2))
    td3 = TD3(cfg, device=DEV, seed=12345)
    ring = ReplayRing(4096, DEV)
    ring.rows[:size, 0] = torch.arange(size, dtype=torch.float32, device=DEV)  # s0 = own index
    ring.size = size
    s = stream_handle()
    draws = []
    for counter in range(2):
        td3.update_counter = counter
        td3._critic_rows(ring, None, None, s)
        torch.cuda.synchronize()
        draws.append(td3.batch[:, 0].long().cpu())
        td3._actor_rows(ring, None, s)
        torch.cuda.synchronize()
        draws.append(td3.batch2[:, 0].long().cpu())
    for d in draws:
        assert d.min() >= 0 and d.max() < size
        counts = torch.bincount(d, minlength=size).numpy()
        assert stats.chisquare(counts).pvalue > 1e-4
        # with replacement: duplicates at the birthday rate of B draws over `size` indices
        assert len(np.unique(d.numpy())) == (counts > 0).sum()
    for i in range(len(draws)):
        for j in range(i + 1, len(draws)):
            assert (draws[i] == draws[j]).float().mean() < 0.01  # independent streams
    # the same (seed, counter) reproduces its batch exactly
    td3.update_counter = 0
    td3._critic_rows(ring, None, None, s)
    torch.cuda.synchronize()
    assert torch.equal(td3.batch[:, 0].long().cpu(), draws[0])


def test_target_smoothing_noise_distribution(nav):
    """Target policy smoothing (robot.py:338-339) through nav_mlp_forward's OUT_TARGET with a zero
    target actor: out = clamp(clamp(0.2 z, +-0.5), +-5) with z ~ N(0, 1) per (row, output)."""
    from nav.mlp import forward
    net = _zero_net(2, 2)
    M = 65536
    x = torch.randn(M, 2, device=DEV)
    out = torch.zeros(M, 2, device=DEV)
    forward([net], x, 2, 0, [out], 2, 0, M, out_mode=1, eps=None, policy_noise=0.2,
            noise_clip=0.5, max_action=5.0, seed=(7, 0), counter=3)
    v = out.cpu().double().numpy()
    assert np.abs(v).max() <= 0.5
    z = v / 0.2
    clipped = np.abs(z) >= 2.5 - 1e-6
    p_clip = 2 * stats.norm.sf(2.5)
    n = z.size
    assert abs(clipped.mean() - p_clip) < 5 * np.sqrt(p_clip * (1 - p_clip) / n)
    # the unclipped part against N(0, 1) truncated to |z| < 2.5
    core = z[~clipped]
    tn = stats.truncnorm(-2.5, 2.5)
    assert stats.kstest(core, tn.cdf).pvalue > 1e-4
    assert abs(np.corrcoef(z[:, 0], z[:, 1])[0, 1]) < 5 / np.sqrt(M)
    # another counter gives another draw
    out2 = torch.zeros_like(out)
    forward([net], x, 2, 0, [out2], 2, 0, M, out_mode=1, eps=None, seed=(7, 0), counter=4)
    assert (out2 == out).float().mean() < 0.05


def test_exploration_noise_distribution(nav):
    """Exploration noise of get_next_action_training (robot.py:614-620) through nav_act with a
    zero actor and state = goal: action = clip(noise_scale * max_action * z, +-5), z ~ N(0, 1)
    per (env, coordinate), a fresh draw per step."""
    from nav._lib import lib, params_struct, ptr, stream_handle
    net = _zero_net(2, 2)
    n = 65536
    p = params_struct(seed_lo=99, seed_hi=0)
    state = (torch.rand(n, 2, dtype=torch.float64, device=DEV) * 90 + 5).contiguous()
    goal = state.clone()
    scale = torch.full((n,), 0.1, dtype=torch.float64, device=DEV)  # sigma = 0.1 * 5 = 0.5
    acts = []
    for step in (0, 1):
        a = torch.zeros(n, 2, dtype=torch.float64, device=DEV)
        rc = lib().nav_act(C.byref(p), C.byref(net.desc()), n, ptr(state), ptr(goal), ptr(scale),
                           None, step, 0, ptr(a), None, stream_handle())
        assert rc == 0
        torch.cuda.synchronize()
        acts.append(a.cpu().numpy() / 0.5)
    for z in acts:
        assert stats.kstest(z.ravel(), "norm").pvalue > 1e-4
        assert abs(z.mean()) < 5 / np.sqrt(z.size)
        assert abs(z.std() - 1) < 5 * np.sqrt(0.5 / z.size)
        assert abs(np.corrcoef(z[:, 0], z[:, 1])[0, 1]) < 5 / np.sqrt(n)
    assert abs(np.corrcoef(acts[0].ravel(), acts[1].ravel())[0, 1]) < 5 / np.sqrt(2 * n)
    # testing mode (robot.py:572-595): no noise at all
    a = torch.zeros(n, 2, dtype=torch.float64, device=DEV)
    lib().nav_act(C.byref(p), C.byref(net.desc()), n, ptr(state), ptr(goal), ptr(scale), None, 0,
                  1, ptr(a), None, stream_handle())
    torch.cuda.synchronize()
    assert torch.count_nonzero(a).item() == 0
