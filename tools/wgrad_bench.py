"""Weight-gradient kernel microbenchmark at the bench shapes (tuning only, not a test).

python tools/wgrad_bench.py [--batch 32768 --hidden 256 --layers 2 --reps 50 --splits c,a]
Times nav_mlp_wgrad for the twin critics (one launch, 2 nets) and the actor (1 net) with HIP
events on the launch stream, plus the gradient reduce that consumes the slabs. Inputs: random
rows, ReLU bits from a real forward. Prints one JSON line.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "residual-td3-robot-navigation_amd"))

import torch  # noqa: E402


def timeit(fn, reps, warm=3):
    for _ in range(warm):
        fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--splits", default="")
    args = ap.parse_args()
    from nav import prof
    from nav._lib import descs, lib, parr, ptr, stream_handle
    from nav.mlp import DeviceMLP, forward
    dev, H, L, B = "cuda", args.hidden, args.layers, args.batch
    g = torch.Generator().manual_seed(0)
    crit = [DeviceMLP(4, 1, H, L, dev).init_kaiming(g) for _ in range(2)]
    actor = DeviceMLP(2, 2, H, L, dev).init_kaiming(g)
    hp = crit[0].hp
    bt = (torch.rand(B, 8, device=dev) * 99).contiguous()
    s = stream_handle()
    lb = lib()
    res = {}
    sc, sa = (lb.nav_mlp_wgrad_splits(2, 1, hp, L, B), lb.nav_mlp_wgrad_splits(1, 2, hp, L, B))
    if args.splits:
        sc, sa = (int(v) for v in args.splits.split(","))
    hc = max(4, lb.nav_mlp_hidden_count(hp, L))
    flops = prof.mlp_wgrad_flops(H, L, B)
    for name, nets, d_out, splits in (("critic", crit, 1, sc), ("actor", [actor], 2, sa)):
        n = len(nets)
        masks = [x.mask_buffer(B) for x in nets]
        acts = [torch.zeros(L, B, hp, device=dev) for _ in nets]
        outs = [torch.zeros(B, d_out, device=dev) for _ in nets]
        for k, x in enumerate(nets):
            forward([x], bt, 8, 0, [outs[k]], d_out, 0, B, acts=[acts[k]], masks=[masks[k]])
        dz = [torch.zeros(L, B, hp, device=dev) for _ in nets]
        dy = [torch.randn(B, d_out, device=dev) / B for _ in nets]
        slabs = [torch.zeros(splits, hc, device=dev) for _ in nets]
        d_in = nets[0].d_in

        def run():
            lb.nav_mlp_wgrad(descs(*nets), n, B, ptr(bt), 8, 0, parr(*acts), parr(*dz),
                             parr(*dy), d_out, parr(*masks), parr(*slabs), splits, s)
        us = timeit(run, args.reps)
        nblk = lb.nav_mlp_row_blocks(B)
        es = [torch.zeros(nblk, lb.nav_mlp_edge_count(d_in, d_out, hp, L), device=dev)
              for _ in nets]
        grads = [torch.zeros(x.count, device=dev) for x in nets]

        def red():
            lb.nav_grad_reduce_multi(descs(*nets), n, parr(*slabs), splits, parr(*es), nblk,
                                     parr(*grads), s)
        us_r = timeit(red, args.reps)
        ms = [torch.zeros(x.count, device=dev) for x in nets]
        vs = [torch.zeros(x.count, device=dev) for x in nets]
        import ctypes as C
        ssz = (C.c_float * n)(*([1e-9] * n))
        bc2 = (C.c_float * n)(*([1.0] * n))

        def red_adam():  # the product's reduce fused with Adam (tiny steps: the weights barely move)
            lb.nav_grad_reduce_adam(descs(*nets), n, parr(*slabs), splits, parr(*es), nblk,
                                    parr(*grads), parr(*ms), parr(*vs), 0.9, 0.999, 1e-8, ssz,
                                    bc2, s)
        us_ra = timeit(red_adam, args.reps)
        res[name] = {"splits": splits, "wgrad_us": round(us, 2),
                     "TFs": round(n * flops / us / 1e6, 1),
                     "frac_157": round(n * flops / us / 1e6 / 157.3, 3),
                     "reduce_us": round(us_r, 2), "reduce_adam_us": round(us_ra, 2),
                     "slab_MB": round(n * splits * hc * 4 / 1e6, 2)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
