"""Diagnostic (tuning aid, not a test): nav_mlp_backward's dx vs torch autograd at one shape,
the worst rows and whether they sit inside the ReLU-kink rounding bound.
python tools/dx_diag.py d_in d_out hidden nh M"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "residual-td3-robot-navigation_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

import torch  # noqa: E402


def main():
    d_in, d_out, hidden, nh, M = map(int, sys.argv[1:6])
    from test_gpu_mlp import make_net, torch_mlp
    from nav._lib import descs, lib, parr, ptr, stream_handle
    from nav.mlp import forward
    DEV = "cuda"
    net, layers = make_net(d_in, d_out, hidden, nh, 11)
    g = torch.Generator().manual_seed(1000 + M)
    x = (torch.randn(M, d_in, generator=g) * 10).contiguous()
    dy = torch.randn(M, d_out, generator=g) / M
    out = torch.zeros(M, d_out, device=DEV)
    acts = torch.zeros(nh, M, net.hp, device=DEV)
    masks = net.mask_buffer(M)
    xd, dyd = x.to(DEV), dy.to(DEV)
    forward([net], xd, d_in, 0, [out], d_out, 0, M, acts=[acts],
            save_mask=net.middle_layers() | net.top_layer(), masks=[masks])
    dz = torch.zeros(nh, M, net.hp, device=DEV)
    dx = torch.zeros(M, d_in, device=DEV)
    L = lib()
    L.nav_mlp_backward(descs(net), 1, M, parr(dyd), d_out, parr(masks), ptr(xd), d_in, 0,
                       parr(acts[nh - 1]), parr(dz), net.middle_layers(), parr(dx), None,
                       stream_handle())
    tl = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in layers]
    xr = x.clone().requires_grad_(True)
    (torch_mlp(tl, xr) * dy).sum().backward()
    with torch.no_grad():
        h, near = x, torch.zeros(M, dtype=torch.bool)
        for W, b in layers[:-1]:
            z = torch.nn.functional.linear(h, W, b)
            near |= (z.abs() <= W.shape[1] * 1.2e-7 * (h.abs() @ W.abs().t() + b.abs())).any(1)
            h = torch.relu(z)
    err = (dx.cpu() - xr.grad).abs().max(1).values
    tol = 1e-3 * xr.grad.abs().max(1).values + 1e-6 * (xr.grad.abs().max() + 1e-3)
    bad = (err > tol).nonzero().flatten()
    print("M", M, "near rows", int(near.sum()), "bad rows", bad.tolist()[:20],
          "bad & near", [bool(near[i]) for i in bad.tolist()[:20]],
          "max err", float(err.max()), "max |dx|", float(xr.grad.abs().max()))


if __name__ == "__main__":
    main()
