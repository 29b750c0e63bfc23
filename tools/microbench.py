"""Per-kernel microbenchmarks at the bench shapes (HIP events, same stream), for tuning.

python tools/microbench.py [--hidden 256 --layers 2 --batch 32768 --envs 65536]
Prints one JSON object: avg µs and achieved TFLOP/s or GB/s per kernel.
"""
import argparse
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "residual-td3-robot-navigation_amd"))

import torch  # noqa: E402


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps  # µs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--quick", action="store_true", help="MLP kernels only (for counter runs)")
    args = ap.parse_args()
    from nav import prof
    from nav._lib import NavMlp, descs, lib, parr, ptr, stream_handle
    from nav.mlp import DeviceMLP, forward
    from nav.trainer import VecTrainer
    dev = "cuda"
    H, L, B = args.hidden, args.layers, args.batch
    g = torch.Generator().manual_seed(0)
    crit = [DeviceMLP(4, 1, H, L, dev).init_kaiming(g) for _ in range(2)]
    DeviceMLP(2, 2, H, L, dev).init_kaiming(g)
    bt = torch.randn(B, 8, device=dev) * 10
    bt[:, 7] = 0
    x = bt[:, :4].contiguous()
    q = [torch.zeros(B, 1, device=dev) for _ in range(2)]
    acts = [torch.zeros(L, B, crit[0].hp, device=dev) for _ in range(2)]
    masks = [crit[0].mask_buffer(B) for _ in range(2)]
    res = {}
    f1 = prof.mlp_fwd_flops(4, 1, H, L, B)
    us = timeit(lambda: forward(crit, x, 4, 0, q, 1, 0, B))
    res["fwd_twin_critic"] = {"us": us, "TFs": 2 * f1 / us / 1e6}
    nblk = lib().nav_mlp_row_blocks(B)
    ec = lib().nav_mlp_edge_count(4, 1, crit[0].hp, L)
    es = [torch.zeros(nblk, ec, device=dev) for _ in range(2)]
    dq = [torch.zeros(B, device=dev) for _ in range(2)]
    lp = torch.zeros(2, nblk, device=dev)
    arr = lambda t: (C.c_void_p * 2)(*[v.data_ptr() for v in t])  # noqa: E731
    cdescs = (NavMlp * 2)(*[c.desc() for c in crit])
    s = stream_handle()
    mid = crit[0].middle_layers()
    us = timeit(lambda: lib().nav_td3_critic_forward(cdescs, B, ptr(bt), 8, 0, ptr(bt), ptr(q[0]),
                                                     ptr(q[1]), 0.99, arr(dq), arr([lp[0], lp[1]]),
                                                     arr(es), arr(acts), mid, arr(masks), s))
    res["fwd_twin_critic_loss"] = {"us": us, "TFs": 2 * f1 / us / 1e6}
    dz = torch.zeros_like(acts[0])
    dz2 = torch.zeros_like(acts[0])
    us = timeit(lambda: lib().nav_mlp_backward(descs(*crit), 2, B, parr(*dq), 1, parr(*masks),
                                               ptr(bt), 8, 0, None, parr(dz, dz2), mid, None,
                                               parr(*es), s))
    fb = prof.mlp_bwd_flops(4, 1, H, L, B, False, True)
    res["bwd_twin_critic_edges"] = {"us": us, "TFs": 2 * fb / us / 1e6}
    dxb = torch.zeros(B, 4, device=dev)
    us = timeit(lambda: lib().nav_mlp_backward(descs(crit[0]), 1, B, parr(dq[0]), 1,
                                               parr(masks[0]), None, 0, 0, None, None, 0,
                                               parr(dxb), None, s))
    res["bwd_critic_dx"] = {"us": us, "TFs": prof.mlp_bwd_flops(4, 1, H, L, B, True) / us / 1e6}
    hc = max(4, lib().nav_mlp_hidden_count(crit[0].hp, L))
    grad = torch.zeros(crit[0].count, device=dev)
    fw = prof.mlp_wgrad_flops(H, L, B)
    for splits in (32, 64, 128):
        sl = torch.zeros(splits, hc, device=dev)
        sl2 = torch.zeros(splits, hc, device=dev)
        us_w = timeit(lambda: lib().nav_mlp_wgrad(descs(*crit), 2, B, ptr(bt), 8, 0, parr(*acts),
                                                  parr(dz, dz2), parr(*dq), 1, parr(*masks),
                                                  parr(sl, sl2), splits, s)) / 2
        us_r = timeit(lambda: lib().nav_grad_reduce(C.byref(crit[0].desc()), ptr(sl), splits,
                                                    ptr(es[0]), nblk, ptr(grad), s))
        res[f"wgrad_splits{splits}"] = {"wgrad_us": us_w, "TFs": fw / us_w / 1e6,
                                         "reduce_us": us_r}
    if args.quick:
        print(json.dumps(res), flush=True)
        return
    # act + env tick + demo at the env count
    tr = VecTrainer(n_envs=args.envs, hidden=H, n_hidden=L, batch=B, updates_per_step=0,
                    device=dev)
    us = timeit(lambda: tr.act())
    res["act"] = {"us": us, "TFs": prof.mlp_fwd_flops(2, 2, H, L, args.envs) / us / 1e6}
    t = prof.KernelTimer()
    with prof.timing(t):
        for _ in range(10):
            tr.collect()
    sm = t.summary()
    m_per = tr.env.demo_xy.shape[0] / (tr.env.demo_off.shape[0] - 1)
    res["agent_step"] = {"us": sm["agent_step"]["avg_us"],
                         "GBs": prof.AGENT_STEP_BYTES * args.envs / sm["agent_step"]["avg_us"] / 1e3}
    ix = tr.env.demo_index
    res["demo_reward_indexed"] = {"us": sm["demo_reward"]["avg_us"],
                                  "mean_candidates": ix.mean_candidates if ix else None}
    ix_saved, tr.env.demo_index = tr.env.demo_index, None
    t = prof.KernelTimer()
    with prof.timing(t):
        for _ in range(10):
            tr.collect()
    sm = t.summary()
    res["demo_reward_brute"] = {"us": sm["demo_reward"]["avg_us"],
                                "f64_TFs": prof.demo_flops(args.envs, m_per) /
                                sm["demo_reward"]["avg_us"] / 1e6}
    from nav.vec_env import DemoIndex
    us = timeit(lambda: DemoIndex(tr.env.demo_xy, tr.env.demo_off))
    res["demo_index_build"] = {"us": us}
    tr.env.demo_index = ix_saved
    # host cost of issuing one full training step vs its GPU time
    import time
    tr2 = VecTrainer(n_envs=args.envs, hidden=H, n_hidden=L, batch=B, updates_per_step=2,
                     device=dev)
    for _ in range(3):
        tr2.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        tr2.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res["train_step"] = {"host_issue_us": (t1 - t0) * 1e5, "wall_us": (t2 - t0) * 1e5}
    print(json.dumps({k: {kk: round(vv, 3) if isinstance(vv, float) else vv
                          for kk, vv in v.items()} for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
