"""Device-resident ReLU MLP (robot.py:128-206) in libnavenv's padded flat layout.

Layout (include/navenv.h, nav_mlp): W0 [hp][d_in], b0 [hp], {W [hp][hp], b [hp]} x (n_hidden-1),
Wo [d_out][hp], bo [d_out], each segment rounded up to 4 floats; hidden width padded to hp (a
multiple of 32) with zeros, which is exact (relu(0) = 0 and zero rows/columns add nothing) and
stays zero under Adam/Polyak (their gradients are exactly zero). `packed` holds the MFMA B-operand
images of every hidden x hidden weight, refreshed by the library after each update.
"""
import ctypes as C
import math

import torch

from . import prof
from ._lib import NavMlp, lib, ptr


def _r4(x):
    return (x + 3) // 4 * 4


def layer_offsets(d_in, d_out, hp, n_hidden):
    offs, o = [], 0
    for l in range(n_hidden + 1):
        fi = d_in if l == 0 else hp
        fo = d_out if l == n_hidden else hp
        w = o
        o += _r4(fi * fo)
        b = o
        o += _r4(fo)
        offs.append((w, b, fo, fi))
    return offs, o


class DeviceMLP:
    def __init__(self, d_in, d_out, hidden, n_hidden, device="cuda"):
        self.d_in, self.d_out, self.hidden, self.n_hidden = d_in, d_out, hidden, n_hidden
        self.hp = (hidden + 31) // 32 * 32
        self.offsets, count = layer_offsets(d_in, d_out, self.hp, n_hidden)
        assert count == lib().nav_mlp_param_count(d_in, d_out, self.hp, n_hidden)
        self.count = count
        self.device = torch.device(device)
        self.params = torch.zeros(count, dtype=torch.float32, device=self.device)
        npk = lib().nav_mlp_packed_count(self.hp, n_hidden)
        self.packed = torch.zeros(max(npk, 4), dtype=torch.float32, device=self.device)
        self._desc = None

    # ---- descriptor for the C-ABI
    def desc(self):
        d = NavMlp(self.d_in, self.d_out, self.hidden, self.hp, self.n_hidden,
                   self.params.data_ptr(), self.packed.data_ptr())
        return d

    def middle_layers(self):
        """save_mask bits of the hidden layers 1 .. n_hidden-2: the only activations / dz rows the
        weight-gradient kernel reads (h_0 and the top dz are recomputed)."""
        return sum(1 << l for l in range(1, self.n_hidden - 1))

    def top_layer(self):
        return 1 << (self.n_hidden - 1)

    def mask_buffer(self, M):
        """ReLU-derivative bit image for M rows (nav_mlp_mask_count u16 words)."""
        n = lib().nav_mlp_mask_count(self.hp, self.n_hidden, M)
        return torch.zeros(n, dtype=torch.int16, device=self.device)

    def sizes(self):
        return [self.d_in] + [self.hidden] * self.n_hidden + [self.d_out]

    # ---- weights in torch nn.Linear layout (logical sizes) <-> device padded layout
    def load(self, layers, stream=None):
        """layers: list of (W [out, in], b [out]) arrays/tensors at logical sizes."""
        assert len(layers) == self.n_hidden + 1
        flat = torch.zeros(self.count, dtype=torch.float32)
        for l, (W, b) in enumerate(layers):
            w_off, b_off, fo, fi = self.offsets[l]
            W = torch.as_tensor(W, dtype=torch.float32).cpu()
            b = torch.as_tensor(b, dtype=torch.float32).cpu()
            o, i = W.shape
            view = flat[w_off:w_off + fo * fi].view(fo, fi)
            view[:o, :i] = W
            flat[b_off:b_off + o] = b
        self.params.copy_(flat.to(self.device))
        self.pack()
        return self

    def export(self):
        flat = self.params.detach().cpu()
        out = []
        sizes = self.sizes()
        for l in range(self.n_hidden + 1):
            w_off, b_off, fo, fi = self.offsets[l]
            o, i = sizes[l + 1], sizes[l]
            W = flat[w_off:w_off + fo * fi].view(fo, fi)[:o, :i].clone()
            b = flat[b_off:b_off + o].clone()
            out.append((W, b))
        return out

    def init_kaiming(self, generator=None):
        """robot.py:161-165: kaiming_uniform_(fan_in, relu) weights, zero biases."""
        layers = []
        sizes = self.sizes()
        for fi, fo in zip(sizes[:-1], sizes[1:]):
            bound = math.sqrt(6.0 / fi)
            W = (torch.rand(fo, fi, generator=generator) * 2 - 1) * bound
            layers.append((W, torch.zeros(fo)))
        return self.load(layers)

    def copy_from(self, other):
        self.params.copy_(other.params)
        self.packed.copy_(other.packed)
        return self

    def pack(self, stream=None):
        from ._lib import stream_handle
        d = self.desc()
        lib().nav_mlp_pack(C.byref(d), stream_handle(stream))

    def state_dict(self):
        return {"params": self.params.detach().cpu(), "meta": [self.d_in, self.d_out,
                                                               self.hidden, self.n_hidden]}

    def load_state_dict(self, sd):
        assert list(sd["meta"]) == [self.d_in, self.d_out, self.hidden, self.n_hidden]
        self.params.copy_(sd["params"].to(self.device))
        self.pack()


def forward(nets, inp, ld_in, in_col, outs, ld_out, out_col, M, out_mode=0, eps=None,
            policy_noise=0.2, noise_clip=0.5, max_action=5.0, seed=(0, 0), counter=0, acts=None,
            masks=None, save_mask=None, stream=None):
    """nav_mlp_forward for 1 or 2 networks sharing `inp`. With `acts`, hidden layer L is saved
    for bits L of save_mask (default: every layer)."""
    from ._lib import stream_handle
    n = len(nets)
    descs = (NavMlp * n)(*[x.desc() for x in nets])
    out_arr = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
    acts_arr = None
    if acts is not None:
        acts_arr = (C.c_void_p * n)(*[(a.data_ptr() if a is not None else None) for a in acts])
    masks_arr = None
    if masks is not None:
        masks_arr = (C.c_void_p * n)(*[(m.data_ptr() if m is not None else None) for m in masks])
    net = nets[0]
    if save_mask is None:
        save_mask = (1 << net.n_hidden) - 1 if acts is not None else 0
    flops = n * prof.mlp_fwd_flops(net.d_in, net.d_out, net.hidden, net.n_hidden, M)
    with prof.region("mlp_fwd", flops):
        lib().nav_mlp_forward(descs, n, M, ptr(inp), ld_in, in_col, out_arr, ld_out, out_col,
                              out_mode, ptr(eps), policy_noise, noise_clip, max_action,
                              seed[0], seed[1], counter, acts_arr, save_mask, masks_arr,
                              stream_handle(stream))
