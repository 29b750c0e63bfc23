"""Shared-policy learner (BASELINE config 5) on the GPU: two learners, each on its half of a
B-row batch, exchanging one SUM bucket per update (the all-reduce nav.dist.GradAllReduce issues
over RCCL), must equal one learner on the whole batch — the update of robot.py:258-398 with the
batch split across ranks. The collective itself is simulated in-process (one process, one GPU):
the sum of the two buckets is written into both, exactly what a 2-rank SUM all-reduce returns.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def replay_rows(n, seed):
    """Replay rows shaped like the tick's (robot.py:79-96): s in the world, clipped actions,
    goal + demo-shaped rewards, s' = a step away, ~2 % dones."""
    rng = np.random.default_rng(seed)
    s = rng.uniform(0, 98.9999, (n, 2))
    a = rng.uniform(-5, 5, (n, 2))
    s2 = np.clip(s + 0.8 * a, 0, 98.9999)
    goal = rng.uniform(5, 95, (n, 2))
    r = -np.linalg.norm(s2 - goal, axis=1) - 10 * rng.uniform(0, 5, n)
    d = (rng.uniform(size=n) < 0.02).astype(np.float64)
    return np.concatenate([s, a, r[:, None], s2, d[:, None]], 1).astype(np.float32)


def make_learner(B, hidden, nh, params):
    from nav import config as K
    from nav.mlp import DeviceMLP
    from nav.td3 import TD3
    pa, p1, p2 = params
    mk = lambda di, do, p: DeviceMLP(di, do, hidden, nh, DEV).load(p)  # noqa: E731
    cfg = K.TD3Config(batch_size=B, num_epochs=2, net=K.NetConfig(hidden=hidden, n_hidden=nh))
    return TD3(cfg, DEV, actor=mk(2, 2, pa), critic1=mk(4, 1, p1), critic2=mk(4, 1, p2))


def ring_of(rows):
    from nav.vec_env import ReplayRing
    rep = ReplayRing(len(rows), DEV)
    rep.rows.copy_(torch.tensor(rows))
    rep.size = len(rows)
    return rep


@pytest.mark.parametrize("hidden,nh,B,epochs", [(256, 2, 8192, 4), (200, 3, 1000, 4)])
def test_two_half_batch_learners_equal_full_batch(hidden, nh, B, epochs):
    from nav import _lib
    from oracle.td3_oracle import make_mlp_params
    _lib.require_gpu()
    sizes = lambda di, do: [di] + [hidden] * nh + [do]  # noqa: E731
    params = (make_mlp_params(71, sizes(2, 2)), make_mlp_params(72, sizes(4, 1)),
              make_mlp_params(73, sizes(4, 1)))
    full = make_learner(B, hidden, nh, params)
    h = B // 2
    ranks = [make_learner(h, hidden, nh, params) for _ in range(2)]
    rep = ring_of(replay_rows(3 * B, 5))
    g = torch.Generator(device="cpu").manual_seed(11)
    for epoch in range(epochs):
        idx = torch.randint(0, len(rep), (B,), generator=g).to(DEV)
        eps = torch.randn(B, 2, generator=g).to(DEV)
        full.train_critic(rep, idx=idx, eps=eps)
        buckets = [r.critic_gradients(rep, idx=idx[k * h:(k + 1) * h].contiguous(),
                                      eps=eps[k * h:(k + 1) * h].contiguous())
                   for k, r in enumerate(ranks)]
        tot = buckets[0] + buckets[1]          # the SUM all-reduce of the one critic bucket
        for b, r in zip(buckets, ranks):
            b.copy_(tot)
            r.critic_step(grad_div=2.0)
        if epoch % 2 == 0:
            idx = torch.randint(0, len(rep), (B,), generator=g).to(DEV)
            full.train_actor(rep, idx=idx)
            buckets = [r.actor_gradients(rep, idx=idx[k * h:(k + 1) * h].contiguous())
                       for k, r in enumerate(ranks)]
            tot = buckets[0] + buckets[1]
            for b, r in zip(buckets, ranks):
                b.copy_(tot)
                r.actor_step(grad_div=2.0)
            for r in [full] + ranks:
                r.soft_update_all()
        for r in [full] + ranks:
            r.update_counter += 1
    torch.cuda.synchronize()
    mine = [r.networks() for r in ranks]
    ref = full.networks()
    for name in ref:
        a, b, f = mine[0][name].params, mine[1][name].params, ref[name].params
        assert torch.equal(a, b), name  # the ranks stay bit-identical
        d = (a - f).abs()
        # one Adam step moves a weight by ~lr = 1e-5: every entry within 2e-7 (measured on
        # MI355X: <= 3e-8; the two paths only differ in the order the batch rows are summed)
        print(f"{name}: max |diff| {float(d.max()):.3e}")
        assert float(d.max()) <= 2e-7, name


class _PairHook:
    """An in-process stand-in for GradAllReduce between two learners that run in two threads:
    both deposit their bucket, rank 0 writes the SUM into both (what a 2-rank SUM all-reduce
    returns) and keeps a copy of it before any Adam step sees it. world_size = 2, so TD3 divides
    by 2 inside nav_adam_multi, exactly as with nav.dist.GradAllReduce."""

    world_size = 2

    def __init__(self, shared, rank):
        self.shared, self.rank = shared, rank
        self.calls = 0

    def __call__(self, bucket):
        sh = self.shared
        sh["slots"][self.rank] = bucket
        sh["barrier"].wait()
        if self.rank == 0:  # every launch before this point is on the one (null) stream
            a, b = sh["slots"]
            tot = a + b
            sh["sums"].append(tot.clone())
            a.copy_(tot)
            b.copy_(tot)
        sh["barrier"].wait()
        self.calls += 1


def _call_plan(B, epochs, seed):
    """The td3_update call sequence's draws: per epoch (critic idx, eps[, actor idx])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    plan = []
    for epoch in range(epochs):
        c = torch.randint(0, 3 * B, (B,), generator=g).to(DEV)
        e = torch.randn(B, 2, generator=g).to(DEV)
        a = torch.randint(0, 3 * B, (B,), generator=g).to(DEV) if epoch % 2 == 0 else None
        plan.append((c, e, a))
    return plan


@pytest.mark.parametrize("hidden,nh,B,epochs", [(256, 2, 8192, 4), (200, 3, 1000, 3)])
def test_grad_hook_branch_gradient_level(hidden, nh, B, epochs):
    """The product shared-policy branch (TD3._grads_and_step with a grad_hook: reduce ->
    hook -> nav_adam_multi(grad_div), robot.py:355-363, 393-395), driven through td3_update /
    train_critic / train_actor by two half-batch learners in two threads, against one full-batch
    learner. Checked BEFORE Adam: the summed bucket / 2 equals the full learner's flat gradient
    (rtol 1e-4; the scale, <g, g_full> / |g_full|^2, within 1e-5 of 1 — a missing or doubled
    / world or / B fails here, which Adam's scale invariance would hide in the parameters); and
    after: the parameters equal the full learner's."""
    import threading
    from nav import _lib
    from oracle.td3_oracle import make_mlp_params
    _lib.require_gpu()
    sizes = lambda di, do: [di] + [hidden] * nh + [do]  # noqa: E731
    params = (make_mlp_params(81, sizes(2, 2)), make_mlp_params(82, sizes(4, 1)),
              make_mlp_params(83, sizes(4, 1)))
    full = make_learner(B, hidden, nh, params)
    h = B // 2
    shared = {"slots": [None, None], "barrier": threading.Barrier(2, timeout=60), "sums": []}
    hooks = [_PairHook(shared, k) for k in range(2)]
    from nav import config as K
    from nav.mlp import DeviceMLP
    from nav.td3 import TD3
    cfg = K.TD3Config(batch_size=h, num_epochs=epochs, net=K.NetConfig(hidden=hidden, n_hidden=nh))
    mk = lambda di, do, p: DeviceMLP(di, do, hidden, nh, DEV).load(p)  # noqa: E731
    ranks = [TD3(cfg, DEV, actor=mk(2, 2, params[0]), critic1=mk(4, 1, params[1]),
                 critic2=mk(4, 1, params[2]), grad_hook=hooks[k]) for k in range(2)]
    assert all(r.grad_div == 2.0 for r in ranks)
    rep = ring_of(replay_rows(3 * B, 6))
    plan = _call_plan(B, epochs, 12)
    # the full-batch learner, gradient and step split so its pre-Adam gradients are visible
    want = []
    for epoch, (c, e, a) in enumerate(plan):
        want.append(full.critic_gradients(rep, idx=c, eps=e).clone())
        full.critic_step()
        if a is not None:
            want.append(full.actor_gradients(rep, idx=a).clone())
            full.actor_step()
            full.soft_update_all()
        full.update_counter += 1

    def run(k):
        torch.cuda.set_device(0)
        it = iter([x for c, e, a in plan for x in ((c, e), (a, None)) if x[0] is not None])
        sl = slice(k * h, (k + 1) * h)
        cur = {}

        def idx_fn():
            i, e = next(it)
            cur["eps"] = None if e is None else e[sl].contiguous()
            return i[sl].contiguous()
        ranks[k].td3_update(rep, idx_fn=idx_fn, eps_fn=lambda: cur["eps"])

    errs = []

    def guarded(k):
        try:
            run(k)
        except BaseException as ex:  # surface a thread's failure in the test
            errs.append(ex)
            shared["barrier"].abort()
    th = [threading.Thread(target=guarded, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    torch.cuda.synchronize()
    n_actor = sum(a is not None for _, _, a in plan)
    assert [hk.calls for hk in hooks] == [epochs + n_actor] * 2
    assert len(shared["sums"]) == len(want)
    for k, (got, ref) in enumerate(zip(shared["sums"], want)):
        g = got / 2  # the mean over ranks = the full batch's mean-loss gradient
        scale = float((g * ref).sum() / (ref * ref).sum())
        err = float((g - ref).abs().max())
        print(f"bucket {k}: scale {scale:.8f} max|diff| {err:.3e} max|g| "
              f"{float(ref.abs().max()):.3e}")
        assert abs(scale - 1.0) <= 1e-5, (k, scale)
        torch.testing.assert_close(g, ref, rtol=1e-4, atol=1e-5 * float(ref.abs().max()))
    mine = [r.networks() for r in ranks]
    for name, f in full.networks().items():
        a, b = mine[0][name].params, mine[1][name].params
        assert torch.equal(a, b), name
        assert float((a - f.params).abs().max()) <= 2e-7, name
        assert torch.equal(mine[0][name].packed, mine[1][name].packed), name


def test_grad_hook_requires_world_size():
    """A plain SUM callable has no world_size: refused instead of training on world x grads."""
    from nav import _lib
    from nav.td3 import TD3
    from nav import config as K
    _lib.require_gpu()
    with pytest.raises(ValueError):
        TD3(K.TD3Config(batch_size=64), DEV, grad_hook=lambda bucket: None)


@pytest.mark.parametrize("grad_div", [1.0, 2.0, 8.0])
def test_adam_multi_grad_div_vs_oracle(grad_div):
    """nav_adam_multi (the shared-policy Adam, two nets in one launch) with non-zero m / v state
    and grad_div in {1, 2, 8} against torch-semantics Adam (oracle) applied to g / grad_div,
    3 steps, atol 2e-7 — pins the / world the all-reduce path relies on."""
    from nav import _lib
    from nav._lib import descs, lib, parr, stream_handle
    from nav.mlp import DeviceMLP, layer_offsets
    from nav.td3 import _Adam
    from oracle.td3_oracle import Adam, make_mlp_params
    import ctypes as C
    _lib.require_gpu()
    nets, refs, opts, ropts, flats = [], [], [], [], []
    for k in range(2):
        p = make_mlp_params(90 + k, [4, 200, 200, 200, 1])
        net = DeviceMLP(4, 1, 200, 3, DEV).load(p)
        opt = _Adam(net, 1e-3)
        g = torch.Generator().manual_seed(100 + k)
        opt.m.copy_((torch.randn(net.count, generator=g) * 1e-2).to(DEV))
        opt.v.copy_((torch.rand(net.count, generator=g) * 1e-3).to(DEV))
        opt.step_count = 5
        ref_t = [torch.tensor(t) for wb in p for t in wb]
        ro = Adam(ref_t, 1e-3)
        offs, _ = layer_offsets(4, 1, net.hp, 3)
        ms, vs = [], []
        for (w_off, b_off, fo, fi), (W, b) in zip(offs, p):
            for off, shp in ((w_off, W.shape), (b_off, b.shape)):
                if len(shp) == 2:
                    ms.append(opt.m[off:off + fo * fi].view(fo, fi)[:shp[0], :shp[1]].cpu())
                    vs.append(opt.v[off:off + fo * fi].view(fo, fi)[:shp[0], :shp[1]].cpu())
                else:
                    ms.append(opt.m[off:off + shp[0]].cpu())
                    vs.append(opt.v[off:off + shp[0]].cpu())
        ro.m, ro.v, ro.step_count = ms, vs, 5
        nets.append(net); refs.append(ref_t); opts.append(opt); ropts.append(ro)
        flats.append((offs, p))
    # padded entries of m / v must stay what the kernel leaves them (zeros propagate): zero them
    for net, opt in zip(nets, opts):
        mask = torch.zeros(net.count, dtype=torch.bool, device=DEV)
        offs, _ = layer_offsets(4, 1, net.hp, 3)
        sizes = [4, 200, 200, 200, 1]
        for l, (w_off, b_off, fo, fi) in enumerate(offs):
            mask[w_off:w_off + fo * fi].view(fo, fi)[:sizes[l + 1], :sizes[l]] = True
            mask[b_off:b_off + sizes[l + 1]] = True
        opt.m[~mask] = 0
        opt.v[~mask] = 0
    for step in range(3):
        grads = []
        for k, net in enumerate(nets):
            gt = [torch.randn_like(t) for t in refs[k]]
            flat = torch.zeros(net.count)
            offs, _ = flats[k]
            for l, (w_off, b_off, fo, fi) in enumerate(offs):
                gW, gb = gt[2 * l], gt[2 * l + 1]
                flat[w_off:w_off + fo * fi].view(fo, fi)[:gW.shape[0], :gW.shape[1]] = gW
                flat[b_off:b_off + gb.shape[0]] = gb
            grads.append(flat.to(DEV))
            ropts[k].step([x / grad_div for x in gt])
        coeffs = [o.advance() for o in opts]
        lib().nav_adam_multi(descs(*nets), 2, parr(*grads), parr(*[o.m for o in opts]),
                             parr(*[o.v for o in opts]), 0.9, 0.999, 1e-8,
                             (C.c_float * 2)(*[c[0] for c in coeffs]),
                             (C.c_float * 2)(*[c[1] for c in coeffs]), grad_div,
                             stream_handle())
    torch.cuda.synchronize()
    for k, net in enumerate(nets):
        got = net.export()
        for l, (W, b) in enumerate(got):
            d = max(float((W - refs[k][2 * l]).abs().max()), float((b - refs[k][2 * l + 1]).abs().max()))
            assert d <= 2e-7, (k, l, d)


def _rank_worker(rank, ws, port, hidden, nh, B, epochs, q):
    """One rank of the 2-process shared-policy run: the product hook (nav.dist.GradAllReduce:
    one SUM all_reduce per bucket, here over gloo since RCCL refuses two ranks on one device)
    inside TD3._grads_and_step, driven by td3_update on this rank's half of each batch."""
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        from nav import config as K
        from nav.dist import GradAllReduce, make_grad_hook
        from nav.mlp import DeviceMLP
        from nav.td3 import TD3
        from oracle.td3_oracle import make_mlp_params
        hook = make_grad_hook(ws)
        assert isinstance(hook, GradAllReduce)
        sizes = lambda di, do: [di] + [hidden] * nh + [do]  # noqa: E731
        params = (make_mlp_params(81, sizes(2, 2)), make_mlp_params(82, sizes(4, 1)),
                  make_mlp_params(83, sizes(4, 1)))
        h = B // ws
        cfg = K.TD3Config(batch_size=h, num_epochs=epochs,
                          net=K.NetConfig(hidden=hidden, n_hidden=nh))
        mk = lambda di, do, p: DeviceMLP(di, do, hidden, nh, DEV).load(p)  # noqa: E731
        td3 = TD3(cfg, DEV, actor=mk(2, 2, params[0]), critic1=mk(4, 1, params[1]),
                  critic2=mk(4, 1, params[2]), grad_hook=hook)
        rep = ring_of(replay_rows(3 * B, 6))
        plan = _call_plan(B, epochs, 12)
        it = iter([x for c, e, a in plan for x in ((c, e), (a, None)) if x[0] is not None])
        sl = slice(rank * h, (rank + 1) * h)
        cur = {}

        def idx_fn():
            i, e = next(it)
            cur["eps"] = None if e is None else e[sl].contiguous()
            return i[sl].contiguous()
        td3.td3_update(rep, idx_fn=idx_fn, eps_fn=lambda: cur["eps"])
        torch.cuda.synchronize()
        out = {k: n.params.cpu().numpy() for k, n in td3.networks().items()}
        q.put((rank, out, hook.calls, hook.bytes))
        dist.destroy_process_group()
    except BaseException as ex:
        q.put((rank, repr(ex), 0, 0))
        raise


def test_adam_polyak_multi_bitwise_vs_adam_then_polyak():
    """nav_adam_polyak_multi (the hook path's policy epoch: the actor's Adam step from the reduced
    bucket and the three soft updates in one launch) equals nav_adam_multi followed by
    nav_polyak_multi bit for bit: parameters, moments, every target and every packed image."""
    import ctypes as C
    from nav import _lib
    from nav._lib import descs, lib, parr, stream_handle
    from nav.mlp import DeviceMLP
    from oracle.td3_oracle import make_mlp_params
    _lib.require_gpu()
    L = lib()
    s = stream_handle()
    res = []
    for fused in (True, False):
        mk = lambda di, do, seed: DeviceMLP(di, do, 256, 2, DEV).load(  # noqa: E731
            make_mlp_params(seed, [di, 256, 256, do]))
        a, ta = mk(2, 2, 11), mk(2, 2, 12)
        c1, c2, t1, t2 = mk(4, 1, 13), mk(4, 1, 14), mk(4, 1, 15), mk(4, 1, 16)
        g = torch.Generator().manual_seed(17)
        grad = (torch.randn(a.count, generator=g) * 1e-2).to(DEV)
        m = (torch.randn(a.count, generator=g) * 1e-3).to(DEV)
        v = (torch.rand(a.count, generator=g) * 1e-4).to(DEV)
        ss, bc = (C.c_float * 1)(1e-3), (C.c_float * 1)(0.7)
        if fused:
            assert L.nav_adam_polyak_multi(descs(a), 1, parr(grad), parr(m), parr(v), 0.9, 0.999,
                                           1e-8, ss, bc, 8.0, descs(ta), descs(t1, t2),
                                           descs(c1, c2), 2, 0.005, s) == 0
        else:
            assert L.nav_adam_multi(descs(a), 1, parr(grad), parr(m), parr(v), 0.9, 0.999, 1e-8,
                                    ss, bc, 8.0, s) == 0
            assert L.nav_polyak_multi(descs(ta, t1, t2), descs(a, c1, c2), 3, 0.005, s) == 0
        torch.cuda.synchronize()
        res.append([x.cpu() for x in (a.params, a.packed, m, v, ta.params, ta.packed, t1.params,
                                       t1.packed, t2.params, t2.packed)])
    for x, y in zip(*res):
        assert torch.equal(x, y)


def test_shared_policy_through_real_collective_two_processes():
    """BASELINE config 5's product path end to end with a real collective: two processes, each a
    TD3(grad_hook=nav.dist.GradAllReduce) on its half batch, all-reducing through
    torch.distributed (gloo: RCCL needs one device per rank, this box has one GPU), against the
    full-batch learner in this process. Same code path as bench.py --shared-policy but the
    backend."""
    import socket
    import torch.multiprocessing as mp
    from nav import _lib
    _lib.require_gpu()
    hidden, nh, B, epochs = 256, 2, 4096, 4
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, hidden, nh, B, epochs, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, out, calls, nbytes = q.get(timeout=240)
            assert not isinstance(out, str), out
            res[r] = (out, calls, nbytes)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    from oracle.td3_oracle import make_mlp_params
    sizes = lambda di, do: [di] + [hidden] * nh + [do]  # noqa: E731
    params = (make_mlp_params(81, sizes(2, 2)), make_mlp_params(82, sizes(4, 1)),
              make_mlp_params(83, sizes(4, 1)))
    full = make_learner(B, hidden, nh, params)
    full.cfg.num_epochs = epochs
    rep = ring_of(replay_rows(3 * B, 6))
    plan = _call_plan(B, epochs, 12)
    it = iter([x for c, e, a in plan for x in ((c, e), (a, None)) if x[0] is not None])
    cur = {}

    def idx_fn():
        i, e = next(it)
        cur["eps"] = e
        return i
    full.td3_update(rep, idx_fn=idx_fn, eps_fn=lambda: cur["eps"])
    torch.cuda.synchronize()
    n_actor = (epochs + 1) // 2
    cc, ca = full.critic_network_1.count, full.actor_network.count
    for r in range(2):
        _, calls, nbytes = res[r]
        assert calls == epochs + n_actor  # one message per bucket: critics (twins) + actor
        assert nbytes == 4 * (epochs * 2 * cc + n_actor * ca)
    for name, f in full.networks().items():
        a, b = res[0][0][name], res[1][0][name]
        assert np.array_equal(a, b), name  # ranks bit-identical
        d = float(np.abs(a - f.params.cpu().numpy()).max())
        print(f"{name}: max |diff| vs full batch {d:.3e}")
        assert d <= 2e-7, name


def _overlap_worker(rank, ws, port, steps, q):
    """One rank of the overlapped-collect check: the same shared-policy VecTrainer run twice in
    this process, with and without the next collect beside the last epoch's critic all-reduce
    (gloo), returning every parameter, the replay ring and the env state of both runs."""
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        from nav.dist import broadcast_params, make_grad_hook, shard_seed
        from nav.trainer import VecTrainer
        out = {}
        for overlap in (True, False):
            hook = make_grad_hook(ws)
            tr = VecTrainer(n_envs=2048, hidden=256, n_hidden=2, batch=1024, updates_per_step=2,
                            seed=shard_seed(2024, rank), envs_per_group=1024, device=DEV,
                            grad_hook=hook, overlap_collect=overlap)
            assert tr.overlap_collect is overlap
            nets = list(tr.td3.networks().values())
            broadcast_params([n.params for n in nets])
            for n in nets:
                n.pack()
            for _ in range(steps):
                tr.step()
            torch.cuda.synchronize()
            res = {k: n.params.cpu().numpy() for k, n in tr.td3.networks().items()}
            res["replay"] = tr.replay.rows.cpu().numpy()
            for k in tr.ENV_STATE:
                res["env_" + k] = getattr(tr.env, k).cpu().numpy()
            out[overlap] = (res, hook.calls)
        q.put((rank, out))
        dist.destroy_process_group()
    except BaseException as ex:
        q.put((rank, repr(ex)))
        raise


def test_overlapped_collect_bit_identical_two_processes():
    """VecTrainer's overlapped step (shared policy: step k+1's collect on a second stream from
    td3_update's collect_ready event, beside step k's final critic all-reduce and Adam step)
    against the serial step, two processes over gloo on this GPU: every parameter, the replay ring
    and the env state bit-identical per rank, and the ranks' parameters identical to each other
    (robot.py:272-285 schedule: critic every epoch, actor on even epochs)."""
    import socket
    import torch.multiprocessing as mp
    from nav import _lib
    _lib.require_gpu()
    steps = 8
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, out = q.get(timeout=240)
            assert not isinstance(out, str), out
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    for r in range(2):
        on, calls_on = res[r][True]
        off, calls_off = res[r][False]
        assert calls_on == calls_off > 0
        for k in off:
            assert np.array_equal(on[k], off[k]), (r, k)
    for k in ("actor", "critic1", "critic2", "target_actor", "target_critic1", "target_critic2"):
        assert np.array_equal(res[0][True][0][k], res[1][True][0][k]), k
    # the ranks' env blocks are independent (seed + rank)
    assert not np.array_equal(res[0][True][0]["replay"], res[1][True][0]["replay"])
