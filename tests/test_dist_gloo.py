"""world_size-2 gloo tests (CPU) of the N > 1 path: independent env-block sharding, the timed
region's max over ranks, and shared-policy gradient averaging (BASELINE configs 4 and 5)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, ws, port):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=ws)


def _worker_shard(rank, ws, port, q):
    _init(rank, ws, port)
    from nav.dist import max_over_ranks, shard_seed
    from oracle import oracle as O
    p = O.default_params(shard_seed(1707366464, rank))
    goals = np.array([O.vec_init_one(p, e)[1] for e in range(8)])
    t = torch.tensor(goals)
    out = [torch.zeros_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    m = max_over_ranks(1.5 + rank, "cpu")
    if rank == 0:
        q.put((np.stack([o.numpy() for o in out]), m))
    dist.destroy_process_group()


def _bucket_step(net, opt, X, Y, hook):
    """One shared-policy step the way nav.td3 takes it: every gradient of the net into ONE flat
    bucket, the hook's SUM all-reduce, then Adam on bucket / world_size (nav_adam_multi's
    grad_div)."""
    ts = net.tensors()
    for t in ts:
        t.requires_grad_(True)
    loss = torch.nn.functional.mse_loss(net.forward(X), Y)
    grads = torch.autograd.grad(loss, ts)
    for t in ts:
        t.requires_grad_(False)
    bucket = torch.cat([g.reshape(-1) for g in grads])
    div = 1.0
    if hook is not None:
        hook(bucket)
        div = float(hook.world_size)
    parts, o = [], 0
    for g in grads:
        parts.append((bucket[o:o + g.numel()] / div).view_as(g))
        o += g.numel()
    opt.step(parts)


def _worker_shared_policy(rank, ws, port, q):
    _init(rank, ws, port)
    from nav.dist import GradAllReduce, broadcast_params, make_grad_hook
    from oracle.td3_oracle import MLP, Adam, make_mlp_params
    torch.manual_seed(100 + rank)  # ranks start different: broadcast must fix that
    net = MLP(make_mlp_params(5 + rank, [4, 64, 64, 1]))
    broadcast_params(net.tensors())
    rng = np.random.default_rng(7)
    X = torch.tensor(rng.standard_normal((64, 4)), dtype=torch.float32)
    Y = torch.tensor(rng.standard_normal((64, 1)), dtype=torch.float32)
    half = slice(rank * 32, (rank + 1) * 32)  # per-rank batch B / world: each rank its half
    hook = make_grad_hook(ws)
    assert isinstance(hook, GradAllReduce) and hook.world_size == ws
    opt = Adam(net.tensors(), 1e-3)
    for _ in range(3):
        _bucket_step(net, opt, X[half], Y[half], hook)
    flat = torch.cat([t.reshape(-1) for t in net.tensors()])
    out = [torch.zeros_like(flat) for _ in range(ws)]
    dist.all_gather(out, flat)
    if rank == 0:
        q.put(([o.numpy() for o in out], hook.calls, hook.bytes))
    dist.destroy_process_group()


def _spawn(fn):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_independent_env_blocks_world2():
    from oracle import oracle as O
    goals, m = _spawn(_worker_shard)
    assert m == 2.5  # max over ranks of the timed region
    for r in range(2):
        p = O.default_params(1707366464 + r)
        ref = np.array([O.vec_init_one(p, e)[1] for e in range(8)])
        assert np.array_equal(goals[r], ref)
    assert not np.array_equal(goals[0], goals[1])  # distinct blocks, no overlap


def test_shared_policy_allreduce_equals_full_batch_world2():
    from oracle.td3_oracle import MLP, Adam, make_mlp_params
    flats, calls, nbytes = _spawn(_worker_shared_policy)
    np.testing.assert_array_equal(flats[0], flats[1])  # ranks stay bit-identical
    n_params = flats[0].size
    assert calls == 3 and nbytes == 3 * 4 * n_params  # one bucket message per step
    # single process, full batch of 64 = mean of the two 32-row halves' gradients
    net = MLP(make_mlp_params(5, [4, 64, 64, 1]))
    rng = np.random.default_rng(7)
    X = torch.tensor(rng.standard_normal((64, 4)), dtype=torch.float32)
    Y = torch.tensor(rng.standard_normal((64, 1)), dtype=torch.float32)
    opt = Adam(net.tensors(), 1e-3)
    for _ in range(3):
        _bucket_step(net, opt, X, Y, None)
    flat = torch.cat([t.reshape(-1) for t in net.tensors()]).numpy()
    np.testing.assert_allclose(flats[0], flat, rtol=0, atol=1e-6)


def _bench(args, env_extra=None):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=240)


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` with no outer torch.distributed.run starts the ranks itself (a child
    launcher): two ranks join one group and rank 0's line says n_gpus 2 (the rank ids sum to 1)."""
    import json
    r = _bench(["--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line: rank 0's
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rank_sum"] == 1
    r1 = _bench(["--launch-check"])  # N = 1: no launcher, one process
    assert r1.returncode == 0 and json.loads(r1.stdout.strip())["n_gpus"] == 1


def test_bench_world_size_mismatch_fails():
    r = _bench(["--gpus", "4", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
