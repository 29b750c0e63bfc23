"""GPU parity of the MFMA MLP kernels and the TD3 learner.

Numerics: every hidden x hidden GEMM (the row kernels and both weight-gradient kernels) runs on
the fp16 matrix cores with its fp32 operands scaled by powers of two and split into two fp16
planes (x 2^e = hi + lo to 22 significant bits): the three products lo.hi + hi.lo + hi.hi
accumulate in fp32 (k_wgrad_fact: two, its A operand — the ReLU bit — is exact in fp16). The
result is f32-class, not bit-fp32: pinned here against an fp64 reference at max |err| / scale
<= 2e-6 (measured 2.4-5.7e-7; fp32 itself ~1e-7; a two-plane bf16 split, a 16-bit-mantissa
GEMM, measures 6-8e-6 and fails it). The thin layers are fp32 fma chains. Against a
torch fp32 reference of the same op the outputs and gradients agree to rtol 1e-4 / 1e-3 with an atol
scaled by the operand magnitudes (stated per test)."""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def nav():
    from nav import _lib
    _lib.require_gpu()
    _lib.lib()
    import nav as navpkg
    return navpkg


def torch_mlp(layers, x):
    h = x
    for i, (W, b) in enumerate(layers):
        h = torch.nn.functional.linear(h, W, b)
        if i < len(layers) - 1:
            h = torch.relu(h)
    return h


def make_net(d_in, d_out, hidden, nh, seed):
    from nav.mlp import DeviceMLP
    from oracle.td3_oracle import make_mlp_params
    p = make_mlp_params(seed, [d_in] + [hidden] * nh + [d_out])
    net = DeviceMLP(d_in, d_out, hidden, nh, DEV).load(p)
    return net, [(torch.tensor(W), torch.tensor(b)) for W, b in p]


@pytest.mark.parametrize("d_in,d_out,hidden,nh", [(2, 2, 200, 3), (4, 1, 200, 3), (2, 2, 256, 2),
                                                  (4, 1, 256, 2), (4, 1, 64, 1), (2, 2, 96, 4)])
@pytest.mark.parametrize("M", [1, 100, 1000, 4097])
def test_forward_vs_torch(nav, d_in, d_out, hidden, nh, M):
    from nav.mlp import forward
    net, layers = make_net(d_in, d_out, hidden, nh, 5)
    x = torch.randn(M, d_in) * 20
    out = torch.zeros(M, d_out, device=DEV)
    acts = torch.zeros(nh, M, net.hp, device=DEV)
    forward([net], x.to(DEV).contiguous(), d_in, 0, [out], d_out, 0, M, acts=[acts])
    ref = torch_mlp(layers, x)
    scale = ref.abs().max().item() + 1
    assert torch.allclose(out.cpu(), ref, rtol=1e-4, atol=1e-5 * scale)
    # saved activations = post-ReLU hidden outputs, zero in the padded columns
    h = x
    for l in range(nh):
        h = torch.relu(torch.nn.functional.linear(h, *layers[l]))
        a = acts[l].cpu()
        assert torch.allclose(a[:, :hidden], h, rtol=1e-4, atol=1e-5 * (h.abs().max() + 1))
        assert (a[:, hidden:] == 0).all()


@pytest.mark.parametrize("d_in,d_out,hidden,nh", [(4, 1, 256, 2), (2, 2, 200, 3), (4, 1, 64, 1)])
def test_forward_row_block_heights_bitwise(nav, d_in, d_out, hidden, nh):
    """Batches <= 16 384 rows run 32-row blocks (RT = 1), larger ones 64-row blocks (RT = 2). The
    forward is the same K-ordered chain and the same output-layer lane tree either way: the first
    16 384 rows of a 16 421-row forward equal a 16 384-row forward bit for bit (outputs, saved
    activations and ReLU bits), and both match torch."""
    from nav.mlp import forward
    net, layers = make_net(d_in, d_out, hidden, nh, 9)
    M1, M2 = 16384, 16421
    x = (torch.randn(M2, d_in) * 20).to(DEV).contiguous()
    res = []
    for M in (M1, M2):
        out = torch.zeros(M, d_out, device=DEV)
        acts = torch.zeros(nh, M, net.hp, device=DEV)
        masks = net.mask_buffer(M)
        forward([net], x[:M].contiguous(), d_in, 0, [out], d_out, 0, M, acts=[acts],
                masks=[masks])
        res.append((out, acts, masks))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0][:M1])
    assert torch.equal(res[0][1], res[1][1][:, :M1])
    ref = torch_mlp(layers, x.cpu())
    scale = ref.abs().max().item() + 1
    assert torch.allclose(res[1][0].cpu(), ref, rtol=1e-4, atol=1e-5 * scale)
    # ReLU bit images: row tile = row / 32 in both; compare every tile of the first 16 384 rows
    from nav._lib import lib
    nt = net.hp // 32
    m1 = res[0][2].view(nh, -1, nt, 64)[:, :M1 // 32]
    m2 = res[1][2].view(nh, -1, nt, 64)[:, :M1 // 32]
    assert torch.equal(m1, m2)
    assert lib().nav_mlp_row_blocks(M1) == M1 // 32 and lib().nav_mlp_row_blocks(M2) == (M2 + 63) // 64


def test_twin_forward_and_target_smoothing(nav):
    from nav.mlp import forward
    c1, L1 = make_net(4, 1, 200, 3, 7)
    c2, L2 = make_net(4, 1, 200, 3, 8)
    M = 999
    x = torch.randn(M, 4) * 10
    o1, o2 = torch.zeros(M, 1, device=DEV), torch.zeros(M, 1, device=DEV)
    forward([c1, c2], x.to(DEV), 4, 0, [o1, o2], 1, 0, M)
    for o, L in ((o1, L1), (o2, L2)):
        r = torch_mlp(L, x)
        assert torch.allclose(o.cpu(), r, rtol=1e-4, atol=1e-5 * (r.abs().max() + 1))
    # robot.py:338-339 smoothing epilogue with injected eps
    a, La = make_net(2, 2, 200, 3, 9)
    s = torch.rand(M, 8) * 100
    eps = torch.randn(M, 2)
    out = torch.zeros(M, 4, device=DEV)
    forward([a], s.to(DEV), 8, 5, [out], 4, 2, M, out_mode=1, eps=eps.to(DEV))
    ref = (torch_mlp(La, s[:, 5:7]) + (eps * 0.2).clamp(-0.5, 0.5)).clamp(-5, 5)
    assert torch.allclose(out[:, 2:].cpu(), ref, rtol=1e-4, atol=1e-4)
    assert (out[:, :2] == 0).all()


def test_act_vs_reference_golden(nav, orc):
    """Robot.get_next_action_training/testing (robot.py:541-595) on the reference's goldens."""
    from nav._lib import lib, params_struct, ptr, stream_handle
    from nav.mlp import DeviceMLP
    from oracle.td3_oracle import make_mlp_params
    g = golden("actions.npz")
    actor = DeviceMLP(2, 2, 200, 3, DEV).load(make_mlp_params(int(g["actor_seed"]),
                                                               [2, 200, 200, 200, 2]))
    n = len(g["states"])
    st = torch.tensor(g["states"], device=DEV)
    gl = torch.tensor(g["goals"], device=DEV)
    sig = torch.tensor(g["sigmas"], device=DEV)
    z = torch.tensor(g["z"], device=DEV)
    act = torch.zeros(n, 2, dtype=torch.float64, device=DEV)
    res = torch.zeros(n, 2, device=DEV)
    p = params_struct()
    d = actor.desc()
    lib().nav_act(C.byref(p), C.byref(d), n, ptr(st), ptr(gl), ptr(sig), ptr(z), 0, 0, ptr(act),
                  ptr(res), stream_handle())
    r = res.cpu().numpy()
    assert np.allclose(r, g["residual"], rtol=2e-5, atol=1e-4)
    a = act.cpu().numpy()
    # epilogue exact given the residual the device computed
    for i in range(n):
        assert np.array_equal(a[i], orc.act_epilogue(g["states"][i], g["goals"][i], r[i],
                                                     g["sigmas"][i], g["z"][i]))
    assert np.allclose(a, g["action_train"], rtol=0, atol=2e-4)
    lib().nav_act(C.byref(p), C.byref(d), n, ptr(st), ptr(gl), None, None, 0, 1, ptr(act),
                  None, stream_handle())
    assert np.allclose(act.cpu().numpy(), g["action_test"], rtol=0, atol=2e-4)


def _grad_flat_vs_autograd(net, tl, gflat, d_in, d_out, nh):
    from nav.mlp import layer_offsets
    offs, _ = layer_offsets(d_in, d_out, net.hp, nh)
    for l, ((W, b), (w_off, b_off, fo, fi)) in enumerate(zip(tl, offs)):
        o, i = W.shape
        gW = gflat[w_off:w_off + fo * fi].view(fo, fi)
        tol = 1e-5 * (W.grad.abs().max() + 1e-6)
        assert torch.allclose(gW[:o, :i], W.grad, rtol=1e-3, atol=tol), l
        assert (gW[o:, :] == 0).all() and (gW[:, i:] == 0).all()
        gb = gflat[b_off:b_off + o]
        assert torch.allclose(gb, b.grad, rtol=1e-3, atol=1e-5 * (b.grad.abs().max() + 1e-6)), l
        assert (gflat[b_off + o:b_off + fo] == 0).all()


def relu_bits(masks, nh, hp, hidden, M):
    """The forward's ReLU bit image ([nh][M / 32 row tiles][hp / 32][64 lanes] u16 words, C
    layout: bit i of lane (l32, h) = row (i & 3) + 8 (i >> 2) + 4 h of the tile, column l32) as
    [nh][M][hidden] booleans."""
    nt = hp // 32
    w = masks.cpu().to(torch.int32) & 0xFFFF
    n_rt = w.numel() // (nh * nt * 64)
    bits = ((w.view(nh, n_rt, nt, 2, 32, 1) >> torch.arange(16)) & 1).bool()
    r = torch.arange(32)
    hh, ii = (r >> 2) & 1, (r & 3) + 4 * (r >> 3)  # lane half and element of tile row r
    b = bits.permute(0, 1, 3, 5, 2, 4)[:, :, hh, ii]  # [nh][n_rt][32 rows][nt][32 cols]
    return b.reshape(nh, n_rt * 32, nt * 32)[:, :M, :hidden]


@pytest.mark.parametrize("d_in,d_out,hidden,nh,M", [(4, 1, 200, 3, 100), (2, 2, 200, 3, 777),
                                                    (4, 1, 256, 2, 5000), (2, 2, 256, 2, 4096),
                                                    (4, 1, 64, 1, 300), (2, 2, 96, 4, 333),
                                                    # 32-row wave ranges ending mid-chunk
                                                    (4, 1, 200, 3, 33), (2, 2, 64, 3, 97),
                                                    # 64-row blocks (RT = 2, > 16 384 rows)
                                                    (4, 1, 256, 2, 16421), (2, 2, 200, 3, 16421),
                                                    (4, 1, 64, 1, 16421),
                                                    # factored weight gradient, 64-high n tiles
                                                    # (hp 192), and the f32 path at n_hidden 2
                                                    # with partial tiles (hp 96)
                                                    (4, 1, 192, 2, 3001), (2, 2, 96, 2, 1000)])
def test_backward_and_weight_grads_vs_autograd(nav, d_in, d_out, hidden, nh, M):
    """Row backward + per-block edge partials + recomputing hidden weight gradients + reduce
    against torch autograd; every gradient entry must be written (NaN-filled buffers)."""
    from nav._lib import descs, lib, parr, ptr, stream_handle
    from nav.mlp import forward
    net, layers = make_net(d_in, d_out, hidden, nh, 11)
    # seeded: ReLU's derivative is discontinuous, so a pre-activation within fp32 rounding of 0
    # can take the other branch in torch (different summation order) and move a dx row by a
    # whole unit's term; unseeded draws hit that about once in a few hundred runs
    g = torch.Generator().manual_seed(1000 + M)
    x = (torch.randn(M, d_in, generator=g) * 10).contiguous()
    dy = torch.randn(M, d_out, generator=g) / M
    out = torch.zeros(M, d_out, device=DEV)
    acts = torch.zeros(nh, M, net.hp, device=DEV)
    masks = net.mask_buffer(M)
    xd = x.to(DEV)
    forward([net], xd, d_in, 0, [out], d_out, 0, M, acts=[acts],
            save_mask=net.middle_layers() | net.top_layer(), masks=[masks])
    dz = torch.zeros(nh, M, net.hp, device=DEV)
    dx = torch.zeros(M, d_in, device=DEV)
    s = stream_handle()
    dyd = dy.to(DEV)
    L = lib()
    nblk = L.nav_mlp_row_blocks(M)
    eslab = torch.full((nblk, L.nav_mlp_edge_count(d_in, d_out, net.hp, nh)), float("nan"),
                       device=DEV)
    L.nav_mlp_backward(descs(net), 1, M, parr(dyd), d_out, parr(masks), ptr(xd), d_in, 0,
                       parr(acts[nh - 1]), parr(dz), net.middle_layers(), parr(dx), parr(eslab), s)
    splits = 7
    hs = torch.full((splits, max(4, L.nav_mlp_hidden_count(net.hp, nh))), float("nan"),
                    device=DEV)
    grad = torch.full((net.count,), float("nan"), device=DEV)
    L.nav_mlp_wgrad(descs(net), 1, M, ptr(xd), d_in, 0, parr(acts), parr(dz), parr(dyd), d_out,
                    parr(masks), parr(hs), splits, s)
    L.nav_grad_reduce(C.byref(net.desc()), ptr(hs), splits, ptr(eslab), nblk, ptr(grad), s)
    # torch autograd reference with the kernel's own ReLU decisions: a pre-activation within the
    # summation-order error bound of 0 (|z| <= K eps32 sum|w h|) may take the other branch in
    # torch's order and move a whole unit's term (at 16 421 rows one does: tools/dx_diag.py,
    # profiles/r02ag_dx_diag.log), so the reference multiplies by the forward's bit image, and
    # the bits must equal torch's (z > 0) everywhere outside that bound
    bits = relu_bits(masks, nh, net.hp, hidden, M)
    with torch.no_grad():
        h = x
        for L, (W, b) in enumerate(layers[:-1]):
            z = torch.nn.functional.linear(h, W, b)
            bound = W.shape[1] * 1.2e-7 * (h.abs() @ W.abs().t() + b.abs())
            assert torch.equal(bits[L][z.abs() > bound], (z > 0)[z.abs() > bound]), L
            h = torch.relu(z)
    tl = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in layers]
    xr = x.clone().requires_grad_(True)
    h = xr
    for L, (W, b) in enumerate(tl):
        h = torch.nn.functional.linear(h, W, b)
        if L < nh:
            h = h * bits[L].float()
    (h * dy).sum().backward()
    assert torch.allclose(dx.cpu(), xr.grad, rtol=1e-3, atol=1e-6 * (xr.grad.abs().max() + 1e-3))
    gflat = grad.cpu()
    assert torch.isfinite(gflat).all()
    _grad_flat_vs_autograd(net, tl, gflat, d_in, d_out, nh)


@pytest.mark.parametrize("hidden,nh,B", [(200, 3, 777), (256, 2, 4096), (64, 1, 100)])
def test_td3_critic_forward_gradients_vs_autograd(nav, hidden, nh, B):
    """train_critic's fused online forward (robot.py:341-361): TD target, MSE loss and gradient,
    then backward + weight gradients of both critics vs torch autograd of mse_loss(Q(s,a), y)."""
    from nav._lib import NavMlp, descs, lib, parr, ptr, stream_handle
    nets = [make_net(4, 1, hidden, nh, 31 + k) for k in range(2)]
    g = torch.Generator().manual_seed(5)
    batch = torch.zeros(B, 8)
    batch[:, :4] = torch.randn(B, 4, generator=g) * 10
    batch[:, 4] = torch.randn(B, generator=g) * 10
    batch[:, 7] = (torch.rand(B, generator=g) < 0.2).float()
    q1t, q2t = torch.randn(B, generator=g) * 20, torch.randn(B, generator=g) * 20
    y = batch[:, 4] + 0.99 * torch.min(q1t, q2t) * (1 - batch[:, 7])
    L = lib()
    bt, q1d, q2d = batch.to(DEV), q1t.to(DEV), q2t.to(DEV)
    nblk = L.nav_mlp_row_blocks(B)
    hp = nets[0][0].hp
    ec = L.nav_mlp_edge_count(4, 1, hp, nh)
    dq = [torch.zeros(B, device=DEV) for _ in range(2)]
    lp = torch.zeros(2, nblk, device=DEV)
    es = [torch.full((nblk, ec), float("nan"), device=DEV) for _ in range(2)]
    acts = [torch.zeros(nh, B, hp, device=DEV) for _ in range(2)]
    dz = [torch.zeros(nh, B, hp, device=DEV) for _ in range(2)]
    masks = [n.mask_buffer(B) for n, _ in nets]
    arr = lambda t: (C.c_void_p * 2)(*[x.data_ptr() for x in t])  # noqa: E731
    mid = nets[0][0].middle_layers()
    s = stream_handle()
    L.nav_td3_critic_forward((NavMlp * 2)(*[n.desc() for n, _ in nets]), B, ptr(bt), 8, 0,
                             ptr(bt), ptr(q1d), ptr(q2d), 0.99, arr(dq), arr([lp[0], lp[1]]),
                             arr(es), arr(acts), mid, arr(masks), s)
    splits = 5
    hs = [torch.zeros(splits, max(4, L.nav_mlp_hidden_count(hp, nh)), device=DEV)
          for _ in range(2)]
    dn = descs(*[n for n, _ in nets])
    L.nav_mlp_backward(dn, 2, B, parr(*dq), 1, parr(*masks), ptr(bt), 8, 0, None, parr(*dz),
                       mid, None, parr(*es), s)
    L.nav_mlp_wgrad(dn, 2, B, ptr(bt), 8, 0, parr(*acts), parr(*dz), parr(*dq), 1, parr(*masks),
                    parr(*hs), splits, s)
    for k, (net, layers) in enumerate(nets):
        grad = torch.full((net.count,), float("nan"), device=DEV)
        L.nav_grad_reduce(C.byref(net.desc()), ptr(hs[k]), splits, ptr(es[k]), nblk, ptr(grad), s)
        tl = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in layers]
        q = torch_mlp(tl, batch[:, :4])
        loss = torch.nn.functional.mse_loss(q, y.unsqueeze(1))
        loss.backward()
        got_loss = lp[k].sum().item() / B
        assert abs(got_loss - loss.item()) <= 1e-4 * loss.item()
        ref_dq = 2 * (q.detach().squeeze(1) - y) / B
        assert torch.allclose(dq[k].cpu(), ref_dq, rtol=1e-4, atol=1e-5 * ref_dq.abs().max())
        gflat = grad.cpu()
        assert torch.isfinite(gflat).all()
        _grad_flat_vs_autograd(net, tl, gflat, 4, 1, nh)


def test_adam_and_polyak_vs_oracle(nav):
    from nav.td3 import _Adam
    from oracle.td3_oracle import Adam
    net, layers = make_net(4, 1, 200, 3, 12)
    tgt, _ = make_net(4, 1, 200, 3, 13)
    opt = _Adam(net, 1e-3)
    ref_t = [t for W, b in layers for t in (W.clone(), b.clone())]
    ref_opt = Adam(ref_t, 1e-3)
    from nav.mlp import layer_offsets
    offs, _ = layer_offsets(4, 1, net.hp, 3)
    for step in range(3):
        grads = [torch.randn_like(t) for t in ref_t]
        flat = torch.zeros(net.count)
        for l, (w_off, b_off, fo, fi) in enumerate(offs):
            gW, gb = grads[2 * l], grads[2 * l + 1]
            flat[w_off:w_off + fo * fi].view(fo, fi)[:gW.shape[0], :gW.shape[1]] = gW
            flat[b_off:b_off + gb.shape[0]] = gb
        opt.step(flat.to(DEV))
        ref_opt.step(grads)
    got = net.export()
    for l, (W, b) in enumerate(got):
        assert torch.allclose(W, ref_t[2 * l], rtol=0, atol=2e-7)
        assert torch.allclose(b, ref_t[2 * l + 1], rtol=0, atol=2e-7)
    # packed images follow the params: a forward through the updated net matches torch
    from nav.mlp import forward
    x = torch.randn(300, 4)
    o = torch.zeros(300, 1, device=DEV)
    forward([net], x.to(DEV), 4, 0, [o], 1, 0, 300)
    ref = torch_mlp(got, x)
    assert torch.allclose(o.cpu(), ref, rtol=1e-4, atol=1e-5 * (ref.abs().max() + 1))
    # Polyak (robot.py:309)
    from nav._lib import lib, stream_handle
    before = [(W.clone(), b.clone()) for W, b in tgt.export()]
    lib().nav_polyak(C.byref(tgt.desc()), C.byref(net.desc()), 0.001, stream_handle())
    after = tgt.export()
    for (W0, b0), (W1, b1), (Ws, bs) in zip(before, after, got):
        assert torch.equal(W1, W0 * (1.0 - 0.001) + Ws * 0.001)
        assert torch.equal(b1, b0 * (1.0 - 0.001) + bs * 0.001)


def test_fused_reduce_adam_and_polyak_multi_bitwise(nav):
    """nav_grad_reduce_adam (2 nets, one launch) == nav_grad_reduce + nav_adam per net, and
    nav_polyak_multi == nav_polyak per pair, bit for bit (same op order)."""
    from nav._lib import descs, lib, parr, ptr, stream_handle
    L = lib()
    s = stream_handle()
    for hidden, nh in ((200, 3), (256, 2), (64, 1)):
        nets = [make_net(4, 1, hidden, nh, 40 + k)[0] for k in range(2)]
        twins = [make_net(4, 1, hidden, nh, 40 + k)[0] for k in range(2)]
        hp = nets[0].hp
        splits, nblk = 3, 5
        hc, ec = max(4, L.nav_mlp_hidden_count(hp, nh)), L.nav_mlp_edge_count(4, 1, hp, nh)
        hs = [torch.randn(splits, hc, device=DEV) for _ in range(2)]
        es = [torch.randn(nblk, ec, device=DEV) for _ in range(2)]
        m = [torch.randn(n.count, device=DEV) * 1e-3 for n in nets]
        v = [torch.rand(n.count, device=DEV) * 1e-4 for n in nets]
        m2, v2 = [x.clone() for x in m], [x.clone() for x in v]
        g_sep = [torch.zeros(n.count, device=DEV) for n in nets]
        g_fus = [torch.zeros(n.count, device=DEV) for n in nets]
        ss, bc = (C.c_float * 2)(1e-3, 2e-3), (C.c_float * 2)(0.5, 0.25)
        L.nav_grad_reduce_adam(descs(*nets), 2, parr(*hs), splits, parr(*es), nblk, parr(*g_fus),
                               parr(*m), parr(*v), 0.9, 0.999, 1e-8, ss, bc, s)
        for k in range(2):
            L.nav_grad_reduce(C.byref(twins[k].desc()), ptr(hs[k]), splits, ptr(es[k]), nblk,
                              ptr(g_sep[k]), s)
            L.nav_adam(C.byref(twins[k].desc()), ptr(g_sep[k]), ptr(m2[k]), ptr(v2[k]), 0.9,
                       0.999, 1e-8, ss[k], bc[k], s)
        for k in range(2):
            assert torch.equal(g_fus[k], g_sep[k])
            assert torch.equal(nets[k].params, twins[k].params)
            assert torch.equal(nets[k].packed, twins[k].packed)
            assert torch.equal(m[k], m2[k]) and torch.equal(v[k], v2[k])
        tg = [make_net(4, 1, hidden, nh, 50 + k)[0] for k in range(3)]
        tg2 = [make_net(4, 1, hidden, nh, 50 + k)[0] for k in range(3)]
        src = [nets[0], nets[1], twins[0]]
        L.nav_polyak_multi(descs(*tg), descs(*src), 3, 0.001, s)
        for t2, sr in zip(tg2, src):
            L.nav_polyak(C.byref(t2.desc()), C.byref(sr.desc()), 0.001, s)
        for t1, t2 in zip(tg, tg2):
            assert torch.equal(t1.params, t2.params) and torch.equal(t1.packed, t2.packed)


def test_td3_update_vs_oracle_and_reference(nav):
    """TD3.td3_update (robot.py:258-398) with the reference golden's weights, batches and noise:
    losses and post-update parameters vs the oracle (and the reference's own digests)."""
    from nav.td3 import TD3
    from nav import config as K
    from nav.mlp import DeviceMLP
    from nav.vec_env import ReplayRing
    from oracle.td3_oracle import TD3Oracle, make_mlp_params, param_digest
    g = golden("td3.npz")
    pa = make_mlp_params(21, [2, 200, 200, 200, 2])
    p1 = make_mlp_params(22, [4, 200, 200, 200, 1])
    p2 = make_mlp_params(23, [4, 200, 200, 200, 1])
    mk = lambda di, do, p: DeviceMLP(di, do, 200, 3, DEV).load(p)  # noqa: E731
    cfg = K.TD3Config(batch_size=int(g["B"]), num_epochs=int(g["epochs"]))
    td3 = TD3(cfg, DEV, actor=mk(2, 2, pa), critic1=mk(4, 1, p1), critic2=mk(4, 1, p2))
    S, A, R, S2, D = (g[k] for k in ("S", "A", "R", "S2", "D"))
    rep = ReplayRing(len(S), DEV)
    rows = np.concatenate([S, A, R[:, None], S2, D[:, None].astype(np.float64)], 1)
    rep.rows.copy_(torch.tensor(rows, dtype=torch.float32))
    rep.size = len(S)
    idx = [torch.tensor(i, dtype=torch.int64, device=DEV) for i in g["idx"]]
    eps = [torch.tensor(e, device=DEV) for e in g["noise"]]
    it = {"s": 0, "n": 0}

    def idx_fn():
        x = idx[it["s"]]; it["s"] += 1
        return x

    def eps_fn():
        x = eps[it["n"]]; it["n"] += 1
        return x

    td3.td3_update(rep, idx_fn=idx_fn, eps_fn=eps_fn, track_losses=True)
    torch.cuda.synchronize()
    closs = np.array(td3.critic_losses)
    np.testing.assert_allclose(closs, g["critic_loss"].mean(1), rtol=1e-4)
    np.testing.assert_allclose(np.array(td3.actor_losses), g["actor_loss"], rtol=1e-4)
    # oracle run on the same inputs, full parameter comparison
    ora = TD3Oracle(pa, p1, p2)
    it2 = {"s": 0, "n": 0}

    def sample():
        i = g["idx"][it2["s"]]; it2["s"] += 1
        return S[i], A[i], R[i], S2[i], D[i]

    def nz():
        x = g["noise"][it2["n"]]; it2["n"] += 1
        return x

    ora.td3_update(sample, nz, int(g["epochs"]))
    mine = td3.networks()
    for name, onet in ora.networks().items():
        got = mine[name].export()
        ref = onet.params
        for (W, b), (Wr, br) in zip(got, ref):
            # one Adam step moves a weight by ~lr = 1e-5; summation-order noise in the grads
            # only matters where |g| ~ eps: compare with an absolute bar well under lr
            assert torch.allclose(W, Wr, rtol=0, atol=2e-7), name
            assert torch.allclose(b, br, rtol=0, atol=2e-7), name
        # and the reference's own digests (sampled entries)
        dig = param_digest([t for wb in got for t in wb])
        for k, (_, _, ix, v) in enumerate(dig):
            assert (ix == g[name + "_idx"][k]).all()
            np.testing.assert_allclose(v, g[name + "_val"][k], rtol=0, atol=3e-7)


# 16 421 rows: the 64-row (RT = 2) form the bench's batch runs
# 333 / 2048: 32-row blocks with L2 warmer rows beside them (<= 128 compute workgroups); 4097:
# 32-row blocks without (129); 16421: 64-row blocks
@pytest.mark.parametrize("hidden,nh,B", [(200, 3, 333), (256, 2, 2048), (256, 2, 4097),
                                         (256, 2, 16421)])
def test_fused_row_kernels_match_unfused(nav, hidden, nh, B):
    """nav_td3_critic_rows / nav_td3_actor_rows (one launch each) produce bit-identical batches,
    targets, dq, losses, ReLU bits, dL/da and edge partials to the per-network kernels they
    fuse (same device code, same order)."""
    from nav._lib import NavReplay, descs, lib, parr, ptr, stream_handle
    from nav.mlp import forward
    L = lib()
    s = stream_handle()
    ta, _ = make_net(2, 2, hidden, nh, 61)
    tc = [make_net(4, 1, hidden, nh, 62 + k)[0] for k in range(2)]
    cr = [make_net(4, 1, hidden, nh, 64 + k)[0] for k in range(2)]
    actor, _ = make_net(2, 2, hidden, nh, 66)
    hp = ta.hp
    cap = 5000
    g = torch.Generator().manual_seed(9)
    rows = torch.randn(cap, 8, generator=g) * 10
    rows[:, 7] = (torch.rand(cap, generator=g) < 0.1).float()
    rows = rows.to(DEV)
    rd = NavReplay(rows.data_ptr(), cap)
    seed, counter = 1707366464, 3
    slo, shi = seed & 0xFFFFFFFF, seed >> 32
    mid = cr[0].middle_layers()
    nblk = L.nav_mlp_row_blocks(B)
    f = lambda *sh: torch.zeros(*sh, device=DEV)  # noqa: E731
    ec = L.nav_mlp_edge_count(4, 1, hp, nh)

    def critic_bufs():
        return dict(batch=f(B, 8), dq=[f(B), f(B)], lp=f(2, nblk), es=[f(nblk, ec), f(nblk, ec)],
                    acts=[f(nh, B, hp), f(nh, B, hp)], masks=[cr[0].mask_buffer(B) for _ in range(2)])
    u, v = critic_bufs(), critic_bufs()
    # unfused: sample, target actor with smoothing, twin targets, online twin with the TD loss
    L.nav_replay_sample(C.byref(rd), cap, B, None, slo, shi, 2 * counter, ptr(u["batch"]), s)
    tgt_in, q1t, q2t = f(B, 4), f(B), f(B)
    L.nav_strided_copy(ptr(u["batch"]), 8, 5, ptr(tgt_in), 4, 0, B, 2, s)
    forward([ta], u["batch"], 8, 5, [tgt_in], 4, 2, B, out_mode=1, seed=(slo, shi),
            counter=counter)
    forward(tc, tgt_in, 4, 0, [q1t, q2t], 1, 0, B)
    L.nav_td3_critic_forward(descs(*cr), B, ptr(u["batch"]), 8, 0, ptr(u["batch"]), ptr(q1t),
                             ptr(q2t), 0.99, parr(*u["dq"]), parr(u["lp"][0], u["lp"][1]),
                             parr(*u["es"]), parr(*u["acts"]), mid, parr(*u["masks"]), s)
    L.nav_td3_critic_rows(C.byref(ta.desc()), descs(*tc), descs(*cr), C.byref(rd), cap, B, None,
                          slo, shi, counter, None, 0.2, 0.5, 5.0, 0.99, ptr(v["batch"]),
                          parr(*v["dq"]), parr(v["lp"][0], v["lp"][1]), parr(*v["es"]),
                          parr(*v["acts"]), mid, parr(*v["masks"]), 0, None, 0, -1, s)
    # the same launch with each online critic's row backward fused in, against the separate
    # nav_mlp_backward of the unfused path (same device code, same order: same bits)
    w = critic_bufs()
    wdz = [f(nh, B, cr[0].hp), f(nh, B, cr[0].hp)]
    L.nav_td3_critic_rows(C.byref(ta.desc()), descs(*tc), descs(*cr), C.byref(rd), cap, B, None,
                          slo, shi, counter, None, 0.2, 0.5, 5.0, 0.99, ptr(w["batch"]),
                          parr(*w["dq"]), parr(w["lp"][0], w["lp"][1]), parr(*w["es"]),
                          parr(*w["acts"]), mid, parr(*w["masks"]), 1, parr(*wdz), mid, -1, s)
    udz = [f(nh, B, cr[0].hp), f(nh, B, cr[0].hp)]
    ues = [u["es"][0].clone(), u["es"][1].clone()]
    L.nav_mlp_backward(descs(*cr), 2, B, parr(*u["dq"]), 1, parr(*u["masks"]), ptr(u["batch"]),
                       8, 0, None, parr(*udz), mid, None, parr(*ues), s)
    torch.cuda.synchronize()
    assert torch.equal(u["batch"], v["batch"])
    assert torch.equal(u["lp"], v["lp"])
    for k in range(2):
        assert torch.equal(u["dq"][k], v["dq"][k])
        assert torch.equal(u["es"][k], v["es"][k])
        assert torch.equal(u["masks"][k], v["masks"][k])
        if mid:
            assert torch.equal(u["acts"][k], v["acts"][k])
        assert torch.equal(w["dq"][k], v["dq"][k])
        assert torch.equal(ues[k], w["es"][k])
        if mid:
            assert torch.equal(udz[k][1:nh - 1], wdz[k][1:nh - 1])
    # actor rows: sample, actor fwd, critic fwd, backward of -mean Q to the action, actor bwd
    eca = L.nav_mlp_edge_count(2, 2, hp, nh)
    save = actor.middle_layers() | actor.top_layer()

    def actor_bufs():
        return dict(batch=f(B, 8), q=f(B), da=f(B, 2), acts=f(nh, B, hp), dz=f(nh, B, hp),
                    ma=actor.mask_buffer(B), mc=cr[0].mask_buffer(B), es=f(nblk, eca))
    u, v = actor_bufs(), actor_bufs()
    L.nav_replay_sample(C.byref(rd), cap, B, None, slo, shi, 2 * counter + 1, ptr(u["batch"]), s)
    forward([actor], u["batch"], 8, 0, [u["batch"]], 8, 2, B, acts=[u["acts"]], save_mask=save,
            masks=[u["ma"]])
    forward([cr[0]], u["batch"], 8, 0, [u["q"]], 1, 0, B, masks=[u["mc"]])
    dqc = torch.full((1,), -1.0 / B, device=DEV)
    dx = f(B, 4)
    L.nav_mlp_backward(descs(cr[0]), 1, B, parr(dqc), 0, parr(u["mc"]), None, 0, 0, None, None, 0,
                       parr(dx), None, s)
    da = dx.view(-1)[2:]
    L.nav_mlp_backward(descs(actor), 1, B, parr(da), 4, parr(u["ma"]), ptr(u["batch"]), 8, 0,
                       parr(u["acts"][nh - 1]), parr(u["dz"]), actor.middle_layers(), None,
                       parr(u["es"]), s)
    L.nav_td3_actor_rows(C.byref(actor.desc()), C.byref(cr[0].desc()), C.byref(rd), cap, B, None,
                         slo, shi, counter, ptr(v["batch"]), ptr(v["q"]), ptr(v["da"]),
                         ptr(v["acts"]), save, ptr(v["dz"]), actor.middle_layers(), ptr(v["ma"]),
                         ptr(v["mc"]), ptr(v["es"]), s)
    torch.cuda.synchronize()
    assert torch.equal(u["batch"][:, :2], v["batch"][:, :2])
    assert torch.equal(u["batch"][:, 4:], v["batch"][:, 4:])
    assert torch.equal(u["q"], v["q"])
    assert torch.equal(dx[:, 2:], v["da"])
    assert torch.equal(u["ma"], v["ma"]) and torch.equal(u["mc"], v["mc"])
    assert torch.equal(u["acts"], v["acts"])
    assert torch.equal(u["es"], v["es"])
    if actor.middle_layers():
        assert torch.equal(u["dz"][1:nh - 1], v["dz"][1:nh - 1])


@pytest.mark.parametrize("hidden,nh,B", [(256, 2, 100), (256, 2, 2048), (200, 3, 777)])
def test_critic_rows_split_twins_bit_identical(nav, hidden, nh, B):
    """nav_td3_critic_rows with the twin online critics in separate workgroups (grid.y = 2, the
    small-batch form) and in one (grid.y = 1) at the same batch: batch rows, dq, loss partials,
    edge slabs, saved rows, ReLU bits and dz all bit-equal (same per-critic device code and
    order; the twin workgroups only repeat the target passes, and only y == 0 writes `batch`)."""
    from nav._lib import NavReplay, descs, lib, parr, ptr, stream_handle
    L = lib()
    s = stream_handle()
    ta, _ = make_net(2, 2, hidden, nh, 161)
    tc = [make_net(4, 1, hidden, nh, 162 + k)[0] for k in range(2)]
    cr = [make_net(4, 1, hidden, nh, 164 + k)[0] for k in range(2)]
    hp = ta.hp
    cap = 3000
    g = torch.Generator().manual_seed(19)
    rows = torch.randn(cap, 8, generator=g) * 10
    rows[:, 7] = (torch.rand(cap, generator=g) < 0.1).float()
    rows = rows.to(DEV)
    rd = NavReplay(rows.data_ptr(), cap)
    mid = cr[0].middle_layers()
    nblk = L.nav_mlp_row_blocks(B)
    f = lambda *sh: torch.full(sh, float("nan"), device=DEV)  # noqa: E731
    ec = L.nav_mlp_edge_count(4, 1, hp, nh)
    out = {}
    for split in (True, False):
        o = dict(batch=f(B, 8), dq=[f(B), f(B)], lp=f(2, nblk), es=[f(nblk, ec), f(nblk, ec)],
                 acts=[f(nh, B, hp), f(nh, B, hp)], dz=[f(nh, B, hp), f(nh, B, hp)],
                 masks=[cr[0].mask_buffer(B) for _ in range(2)])
        assert L.nav_td3_critic_rows(
            C.byref(ta.desc()), descs(*tc), descs(*cr), C.byref(rd), cap, B, None, 1707366464,
            0, 5, None, 0.2, 0.5, 5.0, 0.99, ptr(o["batch"]), parr(*o["dq"]),
            parr(o["lp"][0], o["lp"][1]), parr(*o["es"]), parr(*o["acts"]), mid,
            parr(*o["masks"]), 1, parr(*o["dz"]), mid, int(split), s) == 0
        out[split] = o
    torch.cuda.synchronize()
    a, b = out[True], out[False]
    assert torch.equal(a["batch"], b["batch"])
    assert torch.equal(a["lp"], b["lp"])
    for k in range(2):
        assert torch.equal(a["dq"][k], b["dq"][k]), k
        assert torch.equal(a["es"][k], b["es"][k]), k
        assert torch.equal(a["masks"][k], b["masks"][k]), k
        if mid:
            sel = [l for l in range(nh) if (mid >> l) & 1]
            assert torch.equal(a["acts"][k][sel], b["acts"][k][sel]), k
            assert torch.equal(a["dz"][k][sel], b["dz"][k][sel]), k


def test_reduce_adam_polyak_fused_bitwise(nav):
    """nav_grad_reduce_adam_polyak (the actor's reduce + Adam with the three soft updates of
    robot.py:283-285 in one launch) == nav_grad_reduce_adam then nav_polyak_multi, bit for bit:
    parameters, moments, targets and every packed image."""
    from nav._lib import descs, lib, parr, stream_handle
    L = lib()
    s = stream_handle()
    for hidden, nh, d_in, d_out in ((256, 2, 2, 2), (200, 3, 2, 2)):
        # two identical copies (index 0: unfused, 1: fused) of the actor, its target and the
        # critics' targets; the critics (sources) are shared
        a_net = [make_net(d_in, d_out, hidden, nh, 70)[0] for _ in range(2)]
        atgt = [make_net(d_in, d_out, hidden, nh, 72)[0] for _ in range(2)]
        crit = [make_net(4, 1, hidden, nh, 74 + k)[0] for k in range(2)]
        ctgt = [[make_net(4, 1, hidden, nh, 76 + k)[0] for k in range(2)] for _ in range(2)]
        hp = a_net[0].hp
        splits, nblk = 4, 37
        hc = max(4, L.nav_mlp_hidden_count(hp, nh))
        ec = L.nav_mlp_edge_count(d_in, d_out, hp, nh)
        hs = torch.randn(splits, hc, device=DEV)
        es = torch.randn(nblk, ec, device=DEV)
        m = [torch.randn(a_net[0].count, device=DEV) * 1e-3 for _ in range(2)]
        v = [torch.rand(a_net[0].count, device=DEV) * 1e-4 for _ in range(2)]
        m[1].copy_(m[0]); v[1].copy_(v[0])
        g = [torch.zeros(a_net[0].count, device=DEV) for _ in range(2)]
        ss, bc = (C.c_float * 1)(1e-3), (C.c_float * 1)(0.5)
        # unfused: reduce + Adam, then the soft updates of (actor, critic 1, critic 2)
        L.nav_grad_reduce_adam(descs(a_net[0]), 1, parr(hs), splits, parr(es), nblk, parr(g[0]),
                               parr(m[0]), parr(v[0]), 0.9, 0.999, 1e-8, ss, bc, s)
        L.nav_polyak_multi(descs(atgt[0], ctgt[0][0], ctgt[0][1]),
                           descs(a_net[0], crit[0], crit[1]), 3, 0.001, s)
        # fused
        L.nav_grad_reduce_adam_polyak(descs(a_net[1]), 1, parr(hs), splits, parr(es), nblk,
                                      parr(g[1]), parr(m[1]), parr(v[1]), 0.9, 0.999, 1e-8, ss, bc,
                                      descs(atgt[1]), descs(ctgt[1][0], ctgt[1][1]),
                                      descs(crit[0], crit[1]), 2, 0.001, s)
        torch.cuda.synchronize()
        assert torch.equal(g[0], g[1]) and torch.equal(m[0], m[1]) and torch.equal(v[0], v[1])
        assert torch.equal(a_net[0].params, a_net[1].params)
        assert torch.equal(a_net[0].packed, a_net[1].packed)
        for x, y in ((atgt[0], atgt[1]), (ctgt[0][0], ctgt[1][0]), (ctgt[0][1], ctgt[1][1])):
            assert torch.equal(x.params, y.params) and torch.equal(x.packed, y.packed)


@pytest.mark.parametrize("hidden,nh", [(256, 2), (200, 3), (96, 4), (64, 1)])
@pytest.mark.parametrize("M", [1, 1000, 20000])
def test_acting_forward_residual_bitwise(nav, hidden, nh, M):
    """nav_act's residual (the acting forward, robot.py:556, 598-624: input rows f32(state - goal)
    formed in the kernel, no masks) equals nav_mlp_forward's on the same f32 rows, bit for bit."""
    from nav._lib import lib, params_struct, ptr
    from nav.mlp import forward
    net, _ = make_net(2, 2, hidden, nh, 123)
    g = torch.Generator().manual_seed(M + nh)
    st = (torch.rand(M, 2, generator=g, dtype=torch.float64) * 100).to(DEV)
    gl = (torch.rand(M, 2, generator=g, dtype=torch.float64) * 100).to(DEV)
    act = torch.zeros(M, 2, dtype=torch.float64, device=DEV)
    res = torch.full((M, 2), float("nan"), device=DEV)
    p = params_struct()
    lib().nav_act(C.byref(p), C.byref(net.desc()), M, ptr(st), ptr(gl), None, None, 0, 1, ptr(act),
                  ptr(res), None)
    x = (st - gl).float().contiguous()
    out = torch.full((M, 2), float("nan"), device=DEV)
    forward([net], x, 2, 0, [out], 2, 0, M)
    torch.cuda.synchronize()
    assert torch.equal(res, out)


# ---- fp32 accuracy of the split GEMMs (the property behind the bench's "fp32" dtype) ----
def _f64_forward(layers, x):
    """fp64 forward of the same f32 weights; returns the output and every hidden pre-activation."""
    h, zs = x.double(), []
    for i, (W, b) in enumerate(layers):
        z = torch.nn.functional.linear(h, W.double(), b.double())
        if i < len(layers) - 1:
            zs.append(z)
            h = torch.relu(z)
        else:
            h = z
    return h, zs


@pytest.mark.parametrize("M", [4096, 16421])
def test_split_gemm_per_row_accuracy_rows_spanning_binades(nav, M):
    """Per-row accuracy of the split GEMM's A operand: the A scale is per 32-row
    tile, so a row far below its tile's maximum keeps fewer significant bits in the lo plane
    (fp16 subnormals). Rows of x scaled by 2^-u, u uniform in [0, 20] (biases zeroed, so the
    layer-1 input and output of a row scale with it): each row of h_1 against fp64, relative to
    that row's own max, within 4 (2^-22 + 2^(s - 37)) where 2^-s is the row's h_0 max over its
    tile's — the bound of the scaled two-plane split (the lo plane's absolute step is 2^-24 of a
    scaled maximum in [2^13, 2^14)). Rows near their tile's max meet f32-class accuracy; rows
    2^-20 below it ~2^-17."""
    from nav.mlp import DeviceMLP, forward
    from oracle.td3_oracle import make_mlp_params
    d_in, d_out, hidden, nh = 4, 1, 256, 2
    p = make_mlp_params(91, [d_in, hidden, hidden, d_out])
    p = [(W, b * 0) for W, b in p]
    net = DeviceMLP(d_in, d_out, hidden, nh, DEV).load(p)
    layers = [(torch.tensor(W), torch.tensor(b)) for W, b in p]
    g = torch.Generator().manual_seed(77 + M)
    u = torch.randint(0, 21, (M, 1), generator=g).float()
    x = (torch.randn(M, d_in, generator=g) * torch.pow(2.0, -u)).contiguous()
    out = torch.zeros(M, d_out, device=DEV)
    acts = torch.zeros(nh, M, net.hp, device=DEV)
    forward([net], x.to(DEV), d_in, 0, [out], d_out, 0, M, acts=[acts], save_mask=3)
    torch.cuda.synchronize()
    _, zs = _f64_forward(layers, x)
    h0 = torch.relu(zs[0])
    h1 = torch.relu(zs[1])
    got = acts[1].cpu().double()[:, :hidden]
    rmax0 = h0.abs().amax(1)
    tmax0 = rmax0.view(-1)[:M - M % 32].view(-1, 32).amax(1).repeat_interleave(32)
    tmax0 = torch.cat([tmax0, rmax0[M - M % 32:].max().expand(M % 32)]) if M % 32 else tmax0
    ok = rmax0 > 0
    s = torch.log2(tmax0[ok] / rmax0[ok]).clamp(min=0)
    err = (got[ok] - h1[ok]).abs().amax(1) / h1[ok].abs().amax(1).clamp(min=1e-300)
    bound = 4 * (2.0 ** -22 + torch.pow(2.0, s - 37))
    live = h1[ok].abs().amax(1) > 0
    assert bool((err[live] <= bound[live]).all()), float((err[live] / bound[live]).max())
    print("per-row err: max %.2e, median %.2e; rows with s > 12: max %.2e" % (
        err[live].max(), err[live].median(), err[live & (s > 12)].max()))


@pytest.mark.parametrize("d_in,d_out,hidden,nh", [(2, 2, 200, 3), (4, 1, 200, 3), (2, 2, 256, 2),
                                                  (4, 1, 256, 2), (4, 1, 192, 2)])
@pytest.mark.parametrize("M", [4097, 16421])
def test_split_gemm_f32_accuracy_vs_fp64(nav, d_in, d_out, hidden, nh, M):
    """nav_mlp_forward and the row backward (nav_mlp_backward: dz rows and dx) against an fp64
    reference of the same f32 weights and inputs: max |err| / max |ref| <= 2e-6 for every output,
    saved activation, dz row and dx. fp32 itself sits at ~1e-7 here; the three-plane bf16 split
    measured 3-4e-7, the scaled two-plane fp16 split (22 significant bits) 3-7e-7 in the probe, a
    two-plane bf16 split (a 16-bit-mantissa GEMM, narrower than fp32) 6-8e-6 — the rtol 1e-4 tests
    above pass all three, this one not the last. The row
    backward's reference uses the kernel's own ReLU bits (a kink within rounding of 0 may take the
    other branch in fp64; the bits are checked against the fp64 signs outside that band). Weight
    gradients (cross-row sums) are held to 1e-5 of their scale."""
    from nav._lib import descs, lib, parr, ptr, stream_handle
    from nav.mlp import forward
    net, layers = make_net(d_in, d_out, hidden, nh, 17)
    g = torch.Generator().manual_seed(2000 + M + nh)
    x = (torch.randn(M, d_in, generator=g) * 20).contiguous()
    dy = torch.randn(M, d_out, generator=g) / M
    xd, dyd = x.to(DEV), dy.to(DEV)
    out = torch.zeros(M, d_out, device=DEV)
    acts = torch.zeros(nh, M, net.hp, device=DEV)
    masks = net.mask_buffer(M)
    forward([net], xd, d_in, 0, [out], d_out, 0, M, acts=[acts], masks=[masks])
    L = lib()
    s = stream_handle()
    nblk = L.nav_mlp_row_blocks(M)
    eslab = torch.zeros((nblk, L.nav_mlp_edge_count(d_in, d_out, net.hp, nh)), device=DEV)
    dz = torch.zeros(nh, M, net.hp, device=DEV)
    dx = torch.zeros(M, d_in, device=DEV)
    L.nav_mlp_backward(descs(net), 1, M, parr(dyd), d_out, parr(masks), ptr(xd), d_in, 0,
                       parr(acts[nh - 1]), parr(dz), (1 << nh) - 1, parr(dx), parr(eslab), s)
    splits = 5
    hs = torch.zeros((splits, max(4, L.nav_mlp_hidden_count(net.hp, nh))), device=DEV)
    grad = torch.zeros(net.count, device=DEV)
    L.nav_mlp_wgrad(descs(net), 1, M, ptr(xd), d_in, 0, parr(acts), parr(dz), parr(dyd), d_out,
                    parr(masks), parr(hs), splits, s)
    L.nav_grad_reduce(C.byref(net.desc()), ptr(hs), splits, ptr(eslab), nblk, ptr(grad), s)
    torch.cuda.synchronize()

    def rel(a, ref):
        return float((a.double() - ref).abs().max() / ref.abs().max())

    errs = {}
    ref, zs = _f64_forward(layers, x)
    errs["out"] = rel(out.cpu(), ref)
    for l in range(nh):
        errs[f"h{l}"] = rel(acts[l].cpu()[:, :hidden], torch.relu(zs[l]))
    # fp64 row backward with the kernel's ReLU bits
    bits = relu_bits(masks, nh, net.hp, hidden, M)
    hs64 = [x.double()] + [torch.relu(z) for z in zs]
    for l in range(nh):
        W, b = layers[l]
        band = W.shape[1] * 1.2e-7 * (hs64[l].abs() @ W.double().abs().t() + b.double().abs())
        outside = zs[l].abs() > band
        assert torch.equal(bits[l][outside], (zs[l] > 0)[outside]), l
    gz = dy.double() @ layers[nh][0].double()                   # dL/dh_{nh-1}
    gW = {}
    for l in range(nh - 1, -1, -1):
        gz = gz * bits[l].double()                              # dL/dz_l
        errs[f"dz{l}"] = rel(dz[l].cpu()[:, :hidden], gz)
        gW[l] = gz.t() @ hs64[l]
        gz = gz @ layers[l][0].double()                         # dL/dh_{l-1} (l = 0: dL/dx)
    errs["dx"] = rel(dx.cpu(), gz)
    from nav.mlp import layer_offsets
    offs, _ = layer_offsets(d_in, d_out, net.hp, nh)
    gflat = grad.cpu()
    for l in range(1, nh):
        w_off, _, fo, fi = offs[l]
        errs[f"dW{l}"] = rel(gflat[w_off:w_off + fo * fi].view(fo, fi)[:hidden, :hidden], gW[l])
    print({k: f"{v:.2e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v <= (1e-5 if k.startswith("dW") else 2e-6), (k, v)


@pytest.mark.parametrize("d_in,d_out,hidden", [(4, 1, 256), (4, 1, 192), (2, 2, 256)])
@pytest.mark.parametrize("M,splits", [(1, 1), (31, 3), (33, 1), (100, 40), (2049, 7), (33001, 16)])
@pytest.mark.parametrize("dy_layout", ["packed", "misaligned", "strided"])
def test_weight_grads_2layer_edge_cases(nav, d_in, d_out, hidden, M, splits, dy_layout):
    """nav_mlp_wgrad of a 2-hidden-layer net (the factored path for d_out = 1: 128- or 64-high n
    tiles; the MFMA-operand path for d_out = 2) on ragged row counts (a single row, one partial
    32-row tile, a tile plus one row), more splits than rows, and dy rows that are packed,
    misaligned (not 16-B aligned: the element-load path) or strided (ld_dy = d_out + 1): the sum
    of the slabs against fp64 dW_1 = dz_1^T h_0 with the forward's own ReLU bits, within 1e-5 of
    its scale, and the padded entries exactly 0. 33 001 rows in 16 splits (2 112-row splits, 320
    rows per wave) give 384 / 256-row (factored path) and 448 / 192-row (operand path) wave ranges
    — whole tiles moved to the first wave of each SIMD pair — and a ragged last split of 1 321 rows
    that ends inside wave 3."""
    from nav._lib import descs, lib, parr, ptr, stream_handle
    from nav.mlp import forward
    nh = 2
    net, layers = make_net(d_in, d_out, hidden, nh, 40 + M)
    hp = net.hp
    g = torch.Generator().manual_seed(3000 + M)
    x = (torch.randn(M, d_in, generator=g) * 20).contiguous()
    dy = torch.randn(M, d_out, generator=g) / max(M, 1)
    xd = x.to(DEV)
    out = torch.zeros(M, d_out, device=DEV)
    acts = torch.zeros(nh, M, hp, device=DEV)
    masks = net.mask_buffer(M)
    forward([net], xd, d_in, 0, [out], d_out, 0, M, acts=[acts], masks=[masks])
    if dy_layout == "packed":
        ld, dyd = d_out, dy.to(DEV).contiguous()
        dyp = ptr(dyd)
    elif dy_layout == "misaligned":
        ld = d_out
        buf = torch.zeros(M * d_out + 1, device=DEV)
        buf[1:] = dy.reshape(-1).to(DEV)
        dyd, dyp = buf, buf.data_ptr() + 4
    else:
        ld = d_out + 1
        buf = torch.zeros(M, ld, device=DEV)
        buf[:, :d_out] = dy.to(DEV)
        dyd, dyp = buf, ptr(buf)
    L = lib()
    hc = max(4, L.nav_mlp_hidden_count(hp, nh))
    hs = torch.full((splits, hc), float("nan"), device=DEV)
    dz = torch.zeros(nh, M, hp, device=DEV)
    rc = L.nav_mlp_wgrad(descs(net), 1, M, ptr(xd), d_in, 0, parr(acts), parr(dz),
                         (C.c_void_p * 1)(dyp), ld, parr(masks), parr(hs), splits,
                         stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    del dyd
    got = hs.cpu().double().sum(0)[:hp * hp].view(hp, hp)
    assert torch.isfinite(got).all()
    bits = relu_bits(masks, nh, hp, hidden, M)
    _, zs = _f64_forward(layers, x)
    h0 = torch.relu(zs[0])
    dz1 = (dy.double() @ layers[nh][0].double()) * bits[1].double()
    ref = dz1.t() @ h0
    scale = ref.abs().max().item() + 1e-30
    err = (got[:hidden, :hidden] - ref).abs().max().item()
    assert err <= 1e-5 * scale, (err, scale)
    assert (got[hidden:, :] == 0).all() and (got[:, hidden:] == 0).all()


@pytest.mark.parametrize("d_in,d_out", [(4, 1), (2, 2)])
def test_weight_grads_tiny_inputs_stay_finite(nav, d_in, d_out):
    """Degenerate h_0 scale: every input row 0 and a tiny bias (|b0| ~ 1e-36) make
    the h_0 bound tiny, so its power-of-two scale is large; folded into large layer-0 weights
    (|W0| in [256, 400]) it would overflow them to inf and the zero inputs would give 0 * inf =
    NaN in the operand MFMAs. The scale is capped to keep those constants finite: both kernel
    paths (factored d_out = 1, operand d_out = 2) must match fp64 dW_1 within 1e-5 of scale."""
    from nav._lib import descs, lib, parr, ptr, stream_handle
    from nav.mlp import DeviceMLP, forward
    from oracle.td3_oracle import make_mlp_params
    nh, hidden, M, splits = 2, 256, 4096, 4
    p = make_mlp_params(77, [d_in, hidden, hidden, d_out])
    rng = np.random.default_rng(5)
    W0, b0 = p[0]
    p[0] = ((rng.uniform(256, 400, W0.shape) * rng.choice([-1, 1], W0.shape)).astype(np.float32),
            (rng.uniform(0.5, 1, b0.shape) * 1e-36 * rng.choice([-1, 1], b0.shape))
            .astype(np.float32))
    net = DeviceMLP(d_in, d_out, hidden, nh, DEV).load(p)
    layers = [(torch.tensor(W), torch.tensor(b)) for W, b in p]
    hp = net.hp
    x = torch.zeros(M, d_in)
    dy = torch.randn(M, d_out, generator=torch.Generator().manual_seed(9))
    xd, dyd = x.to(DEV), dy.to(DEV).contiguous()
    out = torch.zeros(M, d_out, device=DEV)
    acts = torch.zeros(nh, M, hp, device=DEV)
    masks = net.mask_buffer(M)
    forward([net], xd, d_in, 0, [out], d_out, 0, M, acts=[acts], masks=[masks])
    L = lib()
    hs = torch.full((splits, max(4, L.nav_mlp_hidden_count(hp, nh))), float("nan"), device=DEV)
    dz = torch.zeros(nh, M, hp, device=DEV)
    assert L.nav_mlp_wgrad(descs(net), 1, M, ptr(xd), d_in, 0, parr(acts), parr(dz), parr(dyd),
                           d_out, parr(masks), parr(hs), splits, stream_handle()) == 0
    torch.cuda.synchronize()
    got = hs.cpu().double().sum(0)[:hp * hp].view(hp, hp)
    assert torch.isfinite(got).all()
    bits = relu_bits(masks, nh, hp, hidden, M)
    _, zs = _f64_forward(layers, x)
    ref = ((dy.double() @ layers[nh][0].double()) * bits[1].double()).t() @ torch.relu(zs[0])
    scale = ref.abs().max().item()
    assert scale > 0
    assert (got[:hidden, :hidden] - ref).abs().max().item() <= 1e-5 * scale


def _fp16_image(packed, off, hp):
    """One fp16 B image (split_entry layout [2][hp/16][2][hp][8], then int32 exponents [hp]) as
    its two planes in fp32 [2][K][N] and the per-column exponents."""
    n = hp * hp
    raw = packed[off:off + n].contiguous().view(torch.float16).float()
    P = raw.view(2, hp // 16, 2, hp, 8).permute(0, 1, 2, 4, 3).reshape(2, hp, hp)
    e = packed[off + n:off + n + hp].contiguous().view(torch.int32)
    return P, e


def _pow2_exp(m):
    """mlp_common.h pow2_exp: e with m 2^e in [2^13, 2^14), clamped to +-126; 0 for 0 / inf."""
    import math
    if not (m > 0) or not math.isfinite(m) or m >= 3.0e38:
        return 0
    _, E = math.frexp(m)
    return max(-126, min(126, 14 - E))


def _assert_images_exact(net, tag):
    """Every hidden x hidden weight: the forward image (B[k][n] = W[n][k]) and the backward image
    (B[k][n] = W[k][n]; for d_out = 1 the top layer's is Wt[k][n] = Wo[k] W[k][n] in f32) hold, per column n with e_n = pow2_exp(max_k |B[k][n]|), hi =
    fp16_rne(B 2^e_n) and lo = fp16_rne(B 2^e_n - hi) bit for bit, and (hi + lo) 2^-e_n equals B
    within 2^-22 of the column's max (11 + 11 significant bits)."""
    hp, nh = net.hp, net.n_hidden
    pk = net.packed.detach().cpu()
    flat = net.params.detach().cpu()
    img = hp * hp + hp
    for L in range(1, nh):
        w_off = net.offsets[L][0]
        W = flat[w_off:w_off + hp * hp].view(hp, hp)
        Wb = W
        if net.d_out == 1 and L == nh - 1:  # the top layer's Wt image: Wo[k] * W[k][n] (f32)
            wo = flat[net.offsets[nh][0]:net.offsets[nh][0] + hp]
            Wb = wo[:, None] * W
        for which, off, Bk in (("fwd", (L - 1) * 2 * img, W.t()), ("bwd", (L - 1) * 2 * img + img, Wb)):
            P, e = _fp16_image(pk, off, hp)
            cmax = Bk.abs().max(0).values
            want = torch.tensor([_pow2_exp(float(m)) for m in cmax], dtype=torch.int32)
            assert torch.equal(e, want), (tag, L, which)
            sc = torch.pow(2.0, want.double())
            x = (Bk.double() * sc).float()  # exact: a power of two
            hi = x.half().float()
            assert torch.equal(P[0], hi), (tag, L, which)
            lo = (x - hi).half().float()
            assert torch.equal(P[1], lo), (tag, L, which)
            rec = (P[0].double() + P[1].double()) / sc
            tol = 2.0 ** -22 * cmax.double() + 1e-45
            assert ((rec - Bk.double()).abs() <= tol).all(), (tag, L, which)


@pytest.mark.parametrize("hidden,nh", [(256, 2), (200, 3), (96, 4)])
def test_packed_images_exact_after_pack_adam_polyak(nav, hidden, nh):
    """The fp16 B-operand images that the hidden GEMMs read follow the weights after every writer
    (the exact two-plane decomposition of _assert_images_exact): nav_mlp_pack, nav_adam,
    nav_polyak, and the product path's fused reduce + Adam + soft updates
    (nav_grad_reduce_adam_polyak), targets included."""
    from nav._lib import descs, lib, parr, ptr, stream_handle
    L = lib()
    s = stream_handle()
    net, _ = make_net(2, 2, hidden, nh, 301)
    _assert_images_exact(net, "pack")
    from nav.td3 import _Adam
    opt = _Adam(net, 1e-3)
    g = torch.Generator().manual_seed(7)
    opt.step((torch.randn(net.count, generator=g) * 1e-2).to(DEV))
    torch.cuda.synchronize()
    _assert_images_exact(net, "adam")
    tgt, _ = make_net(2, 2, hidden, nh, 302)
    L.nav_polyak(C.byref(tgt.desc()), C.byref(net.desc()), 0.37, s)
    torch.cuda.synchronize()
    _assert_images_exact(tgt, "polyak")
    crit = [make_net(4, 1, hidden, nh, 303 + k)[0] for k in range(2)]
    ctgt = [make_net(4, 1, hidden, nh, 305 + k)[0] for k in range(2)]
    hp = net.hp
    splits, nblk = 3, 9
    hs = torch.randn(splits, max(4, L.nav_mlp_hidden_count(hp, nh)), generator=g).to(DEV) * 1e-2
    es = torch.randn(nblk, L.nav_mlp_edge_count(2, 2, hp, nh), generator=g).to(DEV) * 1e-2
    m = torch.randn(net.count, device=DEV) * 1e-3
    v = torch.rand(net.count, device=DEV) * 1e-4
    gr = torch.zeros(net.count, device=DEV)
    assert L.nav_grad_reduce_adam_polyak(
        descs(net), 1, parr(hs), splits, parr(es), nblk, parr(gr), parr(m), parr(v), 0.9, 0.999,
        1e-8, (C.c_float * 1)(1e-2), (C.c_float * 1)(0.5), descs(tgt), descs(*ctgt),
        descs(*crit), 2, 0.25, s) == 0
    torch.cuda.synchronize()
    for t, tag in ((net, "reduce_adam"), (tgt, "own_target"), (ctgt[0], "pair0"),
                   (ctgt[1], "pair1")):
        _assert_images_exact(t, tag)


def _flat_to_tensors(net, flat):
    """Device-layout flat vector -> [W0, b0, W1, ...] at logical sizes (numpy)."""
    from nav.mlp import layer_offsets
    offs, _ = layer_offsets(net.d_in, net.d_out, net.hp, net.n_hidden)
    sizes = net.sizes()
    out = []
    for l, (w_off, b_off, fo, fi) in enumerate(offs):
        o, i = sizes[l + 1], sizes[l]
        out.append(flat[w_off:w_off + fo * fi].view(fo, fi)[:o, :i].numpy())
        out.append(flat[b_off:b_off + o].numpy())
    return out


def test_td3_gradients_vs_reference_grads(nav):
    """The learner's gradients against the REFERENCE's own param.grad (td3_grads.npz: the first
    loss.backward() of train_critic's two critics and of train_actor, robot.py:355-363, 393-395,
    3x200, B = 100) on the same weights, batch indices and smoothing noise: every compared entry
    within rtol 1e-4, the gradient scale within 1e-5 of 1 (a uniform scale error — a wrong 2/B,
    -1/B or split sum — would pass every parameter-level check, since Adam's first step is
    lr * sign(g))."""
    from conftest import golden_grad_check
    from nav import config as K
    from nav.mlp import DeviceMLP
    from nav.td3 import TD3
    from nav.vec_env import ReplayRing
    from oracle.td3_oracle import make_mlp_params
    g, gg = golden("td3.npz"), golden("td3_grads.npz")
    mk = lambda di, do, sd: DeviceMLP(di, do, 200, 3, DEV).load(  # noqa: E731
        make_mlp_params(sd, [di, 200, 200, 200, do]))
    td3 = TD3(K.TD3Config(batch_size=int(g["B"])), DEV, actor=mk(2, 2, 21), critic1=mk(4, 1, 22),
              critic2=mk(4, 1, 23))
    S, A, R, S2, D = (g[k] for k in ("S", "A", "R", "S2", "D"))
    rep = ReplayRing(len(S), DEV)
    rows = np.concatenate([S, A, R[:, None], S2, D[:, None].astype(np.float64)], 1)
    rep.rows.copy_(torch.tensor(rows, dtype=torch.float32))
    rep.size = len(S)
    T = lambda x, dt=None: torch.tensor(x, dtype=dt, device=DEV)  # noqa: E731
    gc = td3.critic_gradients(rep, idx=T(gg["critic_idx"], torch.int64), eps=T(gg["noise"]))
    gc = gc.cpu()
    cc = td3.critic_network_1.count
    for k, (name, net) in enumerate((("critic1", td3.critic_network_1),
                                     ("critic2", td3.critic_network_2))):
        sc = golden_grad_check(gg, name, _flat_to_tensors(net, gc[k * cc:(k + 1) * cc]), 1e-4,
                               1e-6)
        print(name, f"scale {sc:.8f}")
        assert abs(sc - 1) <= 1e-5, (name, sc)
    td3.critic_step()  # train_critic's Adam step, then train_actor's gradient on the new critic 1
    ga = td3.actor_gradients(rep, idx=T(gg["actor_idx"], torch.int64)).cpu()
    sc = golden_grad_check(gg, "actor", _flat_to_tensors(td3.actor_network, ga), 1e-4, 1e-6)
    print("actor", f"scale {sc:.8f}")
    assert abs(sc - 1) <= 1e-5, sc
