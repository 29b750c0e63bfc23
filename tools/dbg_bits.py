"""Debug helper (not a test): the critic row backward's edge partials (W0 | b0 | b1 per row block)
from the fused nav_td3_critic_rows against the unfused nav_td3_critic_forward +
nav_mlp_backward on the same batch, and both against an fp64 recomputation. Prints per segment
the max |diff| between the two paths, the row blocks where they differ, and each path's error
against fp64 relative to the segment's scale.

python tools/dbg_bits.py [--batch 16421]
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

DEV = "cuda"


def make_net(d_in, d_out, hidden, nh, seed):
    from nav.mlp import DeviceMLP
    from oracle.td3_oracle import make_mlp_params
    p = make_mlp_params(seed, [d_in] + [hidden] * nh + [d_out])
    return DeviceMLP(d_in, d_out, hidden, nh, DEV).load(p), p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16421)
    args = ap.parse_args()
    from nav._lib import NavReplay, descs, lib, parr, ptr, stream_handle
    from nav.mlp import forward
    L = lib()
    s = stream_handle()
    hidden, nh, B = 256, 2, args.batch
    ta, _ = make_net(2, 2, hidden, nh, 61)
    tc = [make_net(4, 1, hidden, nh, 62 + k)[0] for k in range(2)]
    crp = [make_net(4, 1, hidden, nh, 64 + k) for k in range(2)]
    cr = [c for c, _ in crp]
    hp = ta.hp
    cap = 5000
    g = torch.Generator().manual_seed(9)
    rows = torch.randn(cap, 8, generator=g) * 10
    rows[:, 7] = (torch.rand(cap, generator=g) < 0.1).float()
    rows = rows.to(DEV)
    rd = NavReplay(rows.data_ptr(), cap)
    seed, counter = 1707366464, 3
    slo, shi = seed & 0xFFFFFFFF, seed >> 32
    nblk = L.nav_mlp_row_blocks(B)
    f = lambda *sh: torch.zeros(*sh, device=DEV)  # noqa: E731
    ec = L.nav_mlp_edge_count(4, 1, hp, nh)

    def bufs():
        return dict(batch=f(B, 8), dq=[f(B), f(B)], lp=f(2, nblk), es=[f(nblk, ec), f(nblk, ec)],
                    acts=[f(nh, B, hp), f(nh, B, hp)],
                    masks=[cr[0].mask_buffer(B) for _ in range(2)])
    u = bufs()
    L.nav_replay_sample(C.byref(rd), cap, B, None, slo, shi, 2 * counter, ptr(u["batch"]), s)
    tgt_in, q1t, q2t = f(B, 4), f(B), f(B)
    L.nav_strided_copy(ptr(u["batch"]), 8, 5, ptr(tgt_in), 4, 0, B, 2, s)
    forward([ta], u["batch"], 8, 5, [tgt_in], 4, 2, B, out_mode=1, seed=(slo, shi),
            counter=counter)
    forward(tc, tgt_in, 4, 0, [q1t, q2t], 1, 0, B)
    L.nav_td3_critic_forward(descs(*cr), B, ptr(u["batch"]), 8, 0, ptr(u["batch"]), ptr(q1t),
                             ptr(q2t), 0.99, parr(*u["dq"]), parr(u["lp"][0], u["lp"][1]),
                             parr(*u["es"]), parr(*u["acts"]), 0, parr(*u["masks"]), s)
    w = bufs()
    wdz = [f(nh, B, hp), f(nh, B, hp)]
    L.nav_td3_critic_rows(C.byref(ta.desc()), descs(*tc), descs(*cr), C.byref(rd), cap, B, None,
                          slo, shi, counter, None, 0.2, 0.5, 5.0, 0.99, ptr(w["batch"]),
                          parr(*w["dq"]), parr(w["lp"][0], w["lp"][1]), parr(*w["es"]),
                          parr(*w["acts"]), 0, parr(*w["masks"]), 1, parr(*wdz), 0, -1, s)
    udz = [f(nh, B, hp), f(nh, B, hp)]
    ues = [u["es"][0].clone(), u["es"][1].clone()]
    dx = [f(B, 4), f(B, 4)]
    L.nav_mlp_backward(descs(*cr), 2, B, parr(*u["dq"]), 1, parr(*u["masks"]), ptr(u["batch"]),
                       8, 0, None, parr(*udz), 0, parr(*dx), parr(*ues), s)
    torch.cuda.synchronize()
    out = {"B": B, "nblk": nblk, "batch_equal": bool(torch.equal(u["batch"], w["batch"])),
           "dq_equal": [bool(torch.equal(u["dq"][k], w["dq"][k])) for k in range(2)],
           "masks_equal": [bool(torch.equal(u["masks"][k], w["masks"][k])) for k in range(2)]}
    x = u["batch"][:, :4].double().cpu()
    segs = {"W0": (0, 4 * hp), "b0": (4 * hp, 5 * hp), "b1": (5 * hp, 6 * hp)}
    for k in range(2):
        p = crp[k][1]
        W0, b0 = (torch.tensor(t, dtype=torch.float64) for t in p[0])
        W1, b1 = (torch.tensor(t, dtype=torch.float64) for t in p[1])
        Wo = torch.tensor(p[2][0], dtype=torch.float64)
        z0 = x @ W0.t() + b0
        h0 = torch.relu(z0)
        z1 = h0 @ W1.t() + b1
        dq = u["dq"][k].double().cpu()
        dz1 = (dq[:, None] * Wo) * (z1 > 0)
        dz0 = (dz1 @ W1) * (z0 > 0)
        blk = torch.arange(B) // 64
        ref = torch.zeros(nblk, 6 * hp, dtype=torch.float64)
        ref[:, 0:4 * hp].index_add_(0, blk, (dz0[:, :, None] * x[:, None, :]).reshape(B, -1))
        ref[:, 4 * hp:5 * hp].index_add_(0, blk, dz0)
        ref[:, 5 * hp:6 * hp].index_add_(0, blk, dz1)
        a, b = ues[k].double().cpu(), w["es"][k].double().cpu()
        res = {}
        for name, (lo, hi) in segs.items():
            d = (a[:, lo:hi] - b[:, lo:hi]).abs()
            bad = torch.nonzero(d.amax(1) > 0).flatten().tolist()
            sc = ref[:, lo:hi].abs().max().item()
            res[name] = {"max_diff": d.max().item(), "blocks_differ": bad[:20],
                         "n_blocks_differ": len(bad),
                         "unfused_err": (a[:, lo:hi] - ref[:, lo:hi]).abs().max().item() / sc,
                         "fused_err": (b[:, lo:hi] - ref[:, lo:hi]).abs().max().item() / sc}
        dxr = dz0 @ W0
        res["dx_unfused_err"] = (dx[k].double().cpu() - dxr).abs().max().item() / \
            dxr.abs().max().item()
        # repeatability of the unfused launch and a single-net launch, per-row dx errors
        reps = []
        for n_nets, nets in ((2, cr), (1, [cr[k]])):
            for _ in range(2):
                dxx = [f(B, 4) for _ in nets]
                L.nav_mlp_backward(descs(*nets), n_nets, B, parr(*[u["dq"][i if n_nets == 2 else k] for i in range(n_nets)]),
                                   1, parr(*[u["masks"][i if n_nets == 2 else k] for i in range(n_nets)]),
                                   ptr(u["batch"]), 8, 0, None, None, 0, parr(*dxx), None, s)
                torch.cuda.synchronize()
                reps.append(dxx[k if n_nets == 2 else 0].double().cpu())
        res["dx_runs_equal"] = [bool(torch.equal(reps[0], r)) for r in reps[1:]]
        res["dx_run_errs"] = [(r - dxr).abs().max().item() / dxr.abs().max().item() for r in reps]
        rerr = ((dx[k].double().cpu() - dxr).abs().amax(1) / dxr.abs().max().item())
        bad = torch.nonzero(rerr > 1e-4).flatten()
        res["bad_rows"] = bad[:30].tolist()
        res["n_bad_rows"] = int(bad.numel())
        if bad.numel():
            r0 = int(bad[0])
            res["bad_row0"] = {"dq": float(dq[r0]), "top_bits": int((z1[r0] > 0).sum()),
                               "l0_bits": int((z0[r0] > 0).sum()), "err": float(rerr[r0])}
        # stress: 2-net launches in both net orders, bad rows per run (row, block, row in block)
        st = []
        for order in ((0, 1), (1, 0)):
            for _ in range(3):
                nets = [cr[i] for i in order]
                dxx = [f(B, 4) for _ in nets]
                L.nav_mlp_backward(descs(*nets), 2, B, parr(*[u["dq"][i] for i in order]), 1,
                                   parr(*[u["masks"][i] for i in order]), ptr(u["batch"]), 8, 0,
                                   None, None, 0, parr(*dxx), None, s)
                torch.cuda.synchronize()
                got = dxx[order.index(k)].double().cpu()
                e = (got - dxr).abs().amax(1) / dxr.abs().max().item()
                bad = torch.nonzero(e > 1e-2).flatten().tolist()
                st.append({"order": order, "bad": [(r, r // 64, r % 64) for r in bad[:12]],
                           "n": len(bad)})
        res["stress"] = st
        # which columns of dz0 are wrong in the bad rows (dz0 rows saved: save_mask bit 0)
        cols = []
        for _ in range(3):
            dzz = [f(nh, B, hp), f(nh, B, hp)]
            L.nav_mlp_backward(descs(*cr), 2, B, parr(*u["dq"]), 1, parr(*u["masks"]),
                               ptr(u["batch"]), 8, 0, None, parr(*dzz), 1, None, None, s)
            torch.cuda.synchronize()
            got = dzz[k][0].double().cpu()[:, :hidden]
            ref0 = dz0
            e = (got - ref0).abs() / ref0.abs().max().item()
            badr = torch.nonzero(e.amax(1) > 1e-3).flatten().tolist()
            for r in badr[:4]:
                bc = torch.nonzero(e[r] > 1e-3).flatten().tolist()
                cols.append({"row": r, "rib": r % 64, "n_cols": len(bc), "cols": bc[:16],
                             "got": [round(float(got[r, c]), 7) for c in bc[:4]],
                             "ref": [round(float(ref0[r, c]), 7) for c in bc[:4]],
                             "ref_row_prev": [round(float(ref0[r - 1, c]), 7) for c in bc[:4]]})
        res["cols"] = cols
        out["critic%d" % k] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
