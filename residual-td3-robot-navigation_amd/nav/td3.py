"""Residual-TD3 learner on the GPU (robot.py:209-398), every FLOP in libnavenv.so kernels.

Method names follow the reference: td3_update, train_critic, train_actor, soft_update. Networks
live as DeviceMLP flat buffers; Adam moments live beside them; torch only allocates memory and
provides the stream. Sampling: robot.py:98-115 draws `batch_size` rows without replacement from a
<=10 000-row buffer; here rows are drawn with replacement by Philox (NAV_TAG_SAMPLE) from the
device ring, or taken from an injected index tensor (parity tests, the N=1 drop-in).
"""
import ctypes as C
import math

import torch

from . import config as K
from . import prof
from ._lib import descs, lib, parr, ptr, stream_handle
from .mlp import DeviceMLP


class _Adam:
    """torch.optim.Adam state for one flat parameter buffer (robot.py:236-239)."""

    def __init__(self, net, lr, betas=(0.9, 0.999), eps=1e-8):
        self.net, self.lr, self.b1, self.b2, self.eps = net, lr, betas[0], betas[1], eps
        self.m = torch.zeros_like(net.params)
        self.v = torch.zeros_like(net.params)
        self.step_count = 0

    def advance(self):
        """Next step's (step_size, bc2_sqrt) = (lr / (1 - b1^t), sqrt(1 - b2^t))."""
        self.step_count += 1
        bc1 = 1 - self.b1 ** self.step_count
        bc2 = 1 - self.b2 ** self.step_count
        return self.lr / bc1, math.sqrt(bc2)

    def step(self, grad, stream=None):
        ss, bc2s = self.advance()
        d = self.net.desc()
        lib().nav_adam(C.byref(d), ptr(grad), ptr(self.m), ptr(self.v), self.b1, self.b2,
                       self.eps, ss, bc2s, stream_handle(stream))

    def state_dict(self):
        return {"m": self.m.cpu(), "v": self.v.cpu(), "t": self.step_count}

    def load_state_dict(self, sd):
        self.m.copy_(sd["m"]); self.v.copy_(sd["v"]); self.step_count = sd["t"]


class TD3:
    def __init__(self, cfg=None, device="cuda", seed=K.RANDOM_SEED, actor=None, critic1=None,
                 critic2=None, grad_hook=None, row_backward=True, fuse_soft_update=True,
                 wgrad_splits=None):
        self.cfg = cfg or K.TD3Config()
        c = self.cfg
        nc = c.net
        self.device = torch.device(device)
        mk = lambda di, do: DeviceMLP(di, do, nc.hidden, nc.n_hidden, self.device)  # noqa: E731
        g = torch.Generator().manual_seed(seed)
        self.actor_network = actor or mk(2, 2).init_kaiming(g)
        self.critic_network_1 = critic1 or mk(4, 1).init_kaiming(g)
        self.critic_network_2 = critic2 or mk(4, 1).init_kaiming(g)
        # robot.py:232-234 deep copies
        self.target_actor = mk(2, 2).copy_from(self.actor_network)
        self.target_critic_network_1 = mk(4, 1).copy_from(self.critic_network_1)
        self.target_critic_network_2 = mk(4, 1).copy_from(self.critic_network_2)
        self.actor_optimizer = _Adam(self.actor_network, c.actor_lr)
        self.critic_optimizer_1 = _Adam(self.critic_network_1, c.critic_lr)
        self.critic_optimizer_2 = _Adam(self.critic_network_2, c.critic_lr)
        self.seed = seed
        self.update_counter = 0  # Philox counter for sampling / smoothing noise
        # shared policy (BASELINE config 5): grad_hook(bucket) SUM-all-reduces a flat gradient
        # bucket in place (nav.dist.GradAllReduce: RCCL over xGMI) and Adam divides by the hook's
        # world_size. The contract is explicit: a hook without world_size is refused, since a
        # plain SUM callable would silently train on world_size x the mean gradient.
        self.grad_hook = grad_hook
        self.grad_div = 1.0
        if grad_hook is not None:
            ws = getattr(grad_hook, "world_size", None)
            if not isinstance(ws, int) or ws < 1:
                raise ValueError("grad_hook must carry an int world_size >= 1: it SUM-all-reduces "
                                 "the gradient bucket and Adam divides by world_size")
            self.grad_div = float(ws)
        # train_critic's row backward inside the critic_rows launch (False: its own launch; the
        # results are bit-identical, A/B only)
        self.row_backward = bool(row_backward)
        # a policy epoch's soft updates inside the actor's reduce + Adam launch (False: their own
        # launch; A/B only)
        self.fuse_soft_update = bool(fuse_soft_update)
        # row splits of the weight-gradient launches, (critic twins, actor); None = as many as
        # fill the chip (nav_mlp_wgrad_splits; tuning only)
        self.wgrad_splits = wgrad_splits
        # the twin online critics in separate workgroups: -1 = the library's choice by batch size
        # (1 / 0 force either form; the results are bit-identical)
        self.split_twins = -1
        self._B = 0
        # the per-epoch launches' constant ctypes arguments (_static), rebuilt when the batch
        # size, the seed or a hyper-parameter they carry changes (_static_key)
        self._st = None
        self._st_key = None
        self._rd = (None, None)
        # td3_update's collect_ready event while it is still to be recorded (_hook / the end)
        self._ready, self._ready_recorded = None, False
        self.actor_losses, self.critic_losses = [], []

    # ---- workspace, sized per batch
    def _workspace(self, B):
        if B == self._B:
            return
        d, hp, nh = self.device, self.actor_network.hp, self.actor_network.n_hidden
        f = lambda *s: torch.zeros(*s, dtype=torch.float32, device=d)  # noqa: E731
        L = lib()
        self.batch = f(B, 8)
        self.batch2 = f(B, 8)
        self.q1 = f(B)
        self.dq1, self.dq2 = f(B), f(B)
        # saved rows: only hidden layers 1 .. nh-2; h_0 and the top dz are recomputed by the
        # weight-gradient kernel, the top layer's dWo partials come from registers
        self.acts1, self.acts2, self.acts_a = f(nh, B, hp), f(nh, B, hp), f(nh, B, hp)
        self.dz1, self.dz2, self.dz_a = f(nh, B, hp), f(nh, B, hp), f(nh, B, hp)
        self.mask1 = self.critic_network_1.mask_buffer(B)
        self.mask2 = self.critic_network_1.mask_buffer(B)
        self.mask_a = self.actor_network.mask_buffer(B)
        self.da = f(B, 2)
        self.nblk = L.nav_mlp_row_blocks(B)
        self.loss_part = f(2, self.nblk)
        ec = L.nav_mlp_edge_count(4, 1, hp, nh)
        self.eslab1, self.eslab2 = f(self.nblk, ec), f(self.nblk, ec)
        self.eslab_a = f(self.nblk, L.nav_mlp_edge_count(2, 2, hp, nh))
        # row splits of the weight-gradient launch (partial slabs): critic twins and actor
        # separately, as many as fill the chip (wgrad_splits overrides; tuning only)
        sc = L.nav_mlp_wgrad_splits(2, self.critic_network_1.d_out, hp, nh, B)
        sa = L.nav_mlp_wgrad_splits(1, self.actor_network.d_out, hp, nh, B)
        if self.wgrad_splits:
            sc, sa = (max(1, min(int(v), max(1, B // 32))) for v in self.wgrad_splits)
        self.splits_c, self.splits_a = sc, sa
        hc = max(4, L.nav_mlp_hidden_count(hp, nh))
        self.hslab, self.hslab2 = f(max(sc, sa), hc), f(sc, hc)
        self.grad_a = f(self.actor_network.count)
        # the twin critics' flat gradients as ONE contiguous bucket (one all-reduce per epoch)
        cc = self.critic_network_1.count
        self.grad_c = f(2 * cc)
        self.grad_c1, self.grad_c2 = self.grad_c[:cc], self.grad_c[cc:]
        self._B = B
        self._st = None

    def _wgrad(self, nets, M, inp, ld_in, in_col, acts, dz, dy, ld_dy, masks, hslabs, s):
        """Hidden x hidden weight gradients of 1-2 same-shape nets: one MFMA launch writing
        `splits` partial slabs per net."""
        net = nets[0]
        splits = self.splits_a if net is self.actor_network else self.splits_c
        if net.n_hidden > 1:
            # k_wgrad_fact (d_out 1, 2 hidden layers, whole 64-wide tiles: 2 fp16 products per
            # f32 product) is timed apart from k_wgrad (3 products): their rooflines differ
            fact = net.d_out == 1 and net.n_hidden == 2 and net.hp % 64 == 0
            with prof.region("mlp_wgrad_fact" if fact else "mlp_wgrad",
                             len(nets) * prof.mlp_wgrad_flops(net.hidden, net.n_hidden, M)):
                lib().nav_mlp_wgrad(descs(*nets), len(nets), M, ptr(inp), ld_in, in_col,
                                    parr(*acts), parr(*dz), parr(*dy), ld_dy, parr(*masks),
                                    parr(*hslabs), splits, s)
        return splits

    def _reduce_bytes(self, nets, eslabs, splits, adam):
        return sum(4.0 * (splits * (x.count - e.shape[1]) + e.numel() +
                          (4 if adam else 1) * x.count) for x, e in zip(nets, eslabs))

    def _hook_and_adam(self, nets, opts, grads, s, stream, soft_update):
        self._hook(self.grad_c if len(nets) == 2 else grads[0], stream)
        self._adam(nets, opts, grads, s, self.grad_div)
        if soft_update:
            self.soft_update_all(stream)

    def _grads_and_step(self, nets, opts, M, inp, ld_in, in_col, acts, dz, dy, ld_dy, masks,
                        eslabs, grads, hslabs, s, stream, soft_update=False):
        """Weight gradients (nav_mlp_wgrad), then the fixed-order reduce of those and the fwd/bwd
        edge partials fused with each net's Adam step (robot.py:236-239) of 1-2 nets (and on a
        policy epoch the three soft updates). With a grad_hook (shared policy) the reduce writes
        the flat gradient bucket without Adam, the hook all-reduces it, and one multi-net Adam
        launch applies bucket / world_size."""
        splits = self._wgrad(nets, M, inp, ld_in, in_col, acts, dz, dy, ld_dy, masks, hslabs, s)
        if self.grad_hook is None:
            coeffs = [o.advance() for o in opts]
            args = (descs(*nets), len(nets), parr(*hslabs), splits, parr(*eslabs), self.nblk,
                    parr(*grads), parr(*[o.m for o in opts]), parr(*[o.v for o in opts]),
                    opts[0].b1, opts[0].b2, opts[0].eps,
                    (C.c_float * len(nets))(*[c[0] for c in coeffs]),
                    (C.c_float * len(nets))(*[c[1] for c in coeffs]))
            with prof.region("grad_reduce", self._reduce_bytes(nets, eslabs, splits, True)):
                if soft_update:  # the actor's step and all three soft updates in one launch
                    lib().nav_grad_reduce_adam_polyak(
                        *args, descs(self.target_actor),
                        descs(self.target_critic_network_1, self.target_critic_network_2),
                        descs(self.critic_network_1, self.critic_network_2), 2, self.cfg.tau, s)
                else:
                    lib().nav_grad_reduce_adam(*args, s)
            return
        with prof.region("grad_reduce", self._reduce_bytes(nets, eslabs, splits, False)):
            lib().nav_grad_reduce_multi(descs(*nets), len(nets), parr(*hslabs), splits,
                                        parr(*eslabs), self.nblk, parr(*grads), s)
        self._hook_and_adam(nets, opts, grads, s, stream, soft_update)

    def _adam(self, nets, opts, grads, s, grad_div=1.0):
        """One multi-net Adam launch on flat gradients (already reduced) / grad_div."""
        coeffs = [o.advance() for o in opts]
        n = len(nets)
        lib().nav_adam_multi(descs(*nets), n, parr(*grads), parr(*[o.m for o in opts]),
                             parr(*[o.v for o in opts]), opts[0].b1, opts[0].b2, opts[0].eps,
                             (C.c_float * n)(*[c[0] for c in coeffs]),
                             (C.c_float * n)(*[c[1] for c in coeffs]), float(grad_div), s)

    def _bwd(self, nets, M, dy, ld_dy, masks, s, inp=None, ld_in=0, in_col=0, h_top=None,
             dz=None, save_mask=0, dx=None, eslab=None):
        net = nets[0]
        n = len(nets)
        with prof.region("mlp_bwd", n * prof.mlp_bwd_flops(net.d_in, net.d_out, net.hidden,
                                                             net.n_hidden, M, dx is not None,
                                                             eslab is not None,
                                                             h_top is not None)):
            nil = [None] * n
            lib().nav_mlp_backward(descs(*nets), n, M, parr(*dy), ld_dy, parr(*masks), ptr(inp),
                                   ld_in, in_col, parr(*(h_top or nil)), parr(*(dz or nil)),
                                   save_mask, parr(*(dx or nil)), parr(*(eslab or nil)), s)

    # ---- the per-epoch launches with their constant arguments built once (the small-batch
    # learner of config 1 is bound by the host's issue of ~450 launches per td3_update)
    def _fast(self):
        return prof._active is None and self.row_backward

    def _static_key(self):
        c = self.cfg
        return (c.batch_size, self.seed, c.policy_noise, c.noise_clip, c.max_action, c.gamma,
                c.tau, self.split_twins)

    def _static(self):
        key = self._static_key()
        if self._st is not None and self._st_key == key:
            return self._st
        c = self.cfg
        B = c.batch_size
        c1, c2, a = self.critic_network_1, self.critic_network_2, self.actor_network
        ta, ca = self.target_actor.desc(), a.desc()
        c1d = c1.desc()
        mid, mida = c1.middle_layers(), a.middle_layers()
        oc, oa = (self.critic_optimizer_1, self.critic_optimizer_2), self.actor_optimizer
        seed = (self.seed & 0xFFFFFFFF, (self.seed >> 32) & 0xFFFFFFFF)
        st = {
            "keep": (ta, ca, c1d),
            "seed": seed,
            "cr_head": (C.byref(ta), descs(self.target_critic_network_1,
                                           self.target_critic_network_2), descs(c1, c2)),
            "cr_tail": (c.policy_noise, c.noise_clip, c.max_action, c.gamma, ptr(self.batch),
                        parr(self.dq1, self.dq2), parr(self.loss_part[0], self.loss_part[1]),
                        parr(self.eslab1, self.eslab2), parr(self.acts1, self.acts2), mid,
                        parr(self.mask1, self.mask2), 1, parr(self.dz1, self.dz2), mid,
                        self.split_twins),
            "ar_head": (C.byref(ca), C.byref(c1d)),
            "ar_tail": (ptr(self.batch2), ptr(self.q1), ptr(self.da), ptr(self.acts_a), mida,
                        ptr(self.dz_a), mida, ptr(self.mask_a), ptr(self.mask1),
                        ptr(self.eslab_a)),
        }
        wc = self._critic_wgrad_args()
        st["wg_c"] = (descs(c1, c2), 2, B, ptr(wc[0]), wc[1], wc[2], parr(*wc[3]), parr(*wc[4]),
                      parr(*wc[5]), wc[6], parr(*wc[7]), parr(self.hslab, self.hslab2),
                      self.splits_c)
        wa = self._actor_wgrad_args()
        st["wg_a"] = (descs(a), 1, B, ptr(wa[0]), wa[1], wa[2], parr(*wa[3]), parr(*wa[4]),
                      parr(*wa[5]), wa[6], parr(*wa[7]), parr(self.hslab), self.splits_a)
        st["red_c"] = (descs(c1, c2), 2, parr(self.hslab, self.hslab2), self.splits_c,
                       parr(self.eslab1, self.eslab2), self.nblk, parr(self.grad_c1, self.grad_c2),
                       parr(*[o.m for o in oc]), parr(*[o.v for o in oc]), oc[0].b1, oc[0].b2,
                       oc[0].eps)
        st["red_a"] = (descs(a), 1, parr(self.hslab), self.splits_a, parr(self.eslab_a),
                       self.nblk, parr(self.grad_a), parr(oa.m), parr(oa.v), oa.b1, oa.b2, oa.eps)
        st["poly"] = (descs(self.target_actor),
                      descs(self.target_critic_network_1, self.target_critic_network_2),
                      descs(c1, c2), 2, c.tau)
        # shared policy (grad_hook): reduce into the flat bucket, the hook's collective, then the
        # multi-net Adam on bucket / world_size and (policy epoch) the three soft updates
        st["redm_c"] = (descs(c1, c2), 2, parr(self.hslab, self.hslab2), self.splits_c,
                        parr(self.eslab1, self.eslab2), self.nblk, parr(self.grad_c1, self.grad_c2))
        st["adam_c"] = (descs(c1, c2), 2, parr(self.grad_c1, self.grad_c2),
                        parr(*[o.m for o in oc]), parr(*[o.v for o in oc]), oc[0].b1, oc[0].b2,
                        oc[0].eps)
        st["redm_a"] = (descs(a), 1, parr(self.hslab), self.splits_a, parr(self.eslab_a),
                        self.nblk, parr(self.grad_a))
        st["adam_a"] = (descs(a), 1, parr(self.grad_a), parr(oa.m), parr(oa.v), oa.b1, oa.b2,
                        oa.eps)

        st["wgrad"] = c1.n_hidden > 1
        self._st, self._st_key = st, key
        return st

    def _replay_ref(self, replay):
        if self._rd[0] is not replay:
            d = replay.desc()
            self._rd = (replay, (d, C.byref(d)))
        return self._rd[1][1]

    def _hook(self, bucket, stream):
        # the collective runs on torch's current stream: make it the launch stream, so it starts
        # after the reduce and Adam starts after it
        if self._ready is not None:  # the last epoch's replay reads and actor writes are issued
            self._ready.record(stream)
            self._ready, self._ready_recorded = None, True
        # region "allreduce": an event pair on the launch stream around the message (the
        # collective's stream waits for it and it for the collective), when a timer asks
        nbytes = bucket.numel() * bucket.element_size()
        if stream is None:
            with prof.region("allreduce", nbytes):
                self.grad_hook(bucket)
        else:
            with torch.cuda.stream(stream):
                with prof.region("allreduce", nbytes):
                    self.grad_hook(bucket)

    def _critic_epoch_fast(self, replay, idx, eps, s, stream):
        c = self.cfg
        B = c.batch_size
        self._workspace(B)
        st, L = self._static(), lib()
        L.nav_td3_critic_rows(*st["cr_head"], self._replay_ref(replay), len(replay), B,
                              None if idx is None else C.c_void_p(idx.data_ptr()), *st["seed"],
                              self.update_counter,
                              None if eps is None else C.c_void_p(eps.data_ptr()), *st["cr_tail"],
                              s)
        if st["wgrad"]:
            L.nav_mlp_wgrad(*st["wg_c"], s)
        o1, o2 = self.critic_optimizer_1.advance(), self.critic_optimizer_2.advance()
        ss, bc = (C.c_float * 2)(o1[0], o2[0]), (C.c_float * 2)(o1[1], o2[1])
        if self.grad_hook is None:
            L.nav_grad_reduce_adam(*st["red_c"], ss, bc, s)
            return
        L.nav_grad_reduce_multi(*st["redm_c"], s)
        self._hook(self.grad_c, stream)
        L.nav_adam_multi(*st["adam_c"], ss, bc, self.grad_div, s)

    def _actor_epoch_fast(self, replay, idx, s, stream, soft_update):
        c = self.cfg
        B = c.batch_size
        self._workspace(B)
        st, L = self._static(), lib()
        L.nav_td3_actor_rows(*st["ar_head"], self._replay_ref(replay), len(replay), B,
                             None if idx is None else C.c_void_p(idx.data_ptr()), *st["seed"],
                             self.update_counter, *st["ar_tail"], s)
        if st["wgrad"]:
            L.nav_mlp_wgrad(*st["wg_a"], s)
        o = self.actor_optimizer.advance()
        ss, bc = (C.c_float * 1)(o[0]), (C.c_float * 1)(o[1])
        if self.grad_hook is not None:
            L.nav_grad_reduce_multi(*st["redm_a"], s)
            self._hook(self.grad_a, stream)
            if soft_update:  # the actor's step and the three soft updates in one launch
                L.nav_adam_polyak_multi(*st["adam_a"], ss, bc, self.grad_div, *st["poly"], s)
            else:
                L.nav_adam_multi(*st["adam_a"], ss, bc, self.grad_div, s)
        elif soft_update:
            L.nav_grad_reduce_adam_polyak(*st["red_a"], ss, bc, *st["poly"], s)
        else:
            L.nav_grad_reduce_adam(*st["red_a"], ss, bc, s)

    # robot.py:312-366
    def _critic_rows(self, replay, idx, eps, s):
        c = self.cfg
        B = c.batch_size
        self._workspace(B)
        c1, c2 = self.critic_network_1, self.critic_network_2
        mid = c1.middle_layers()
        rd = replay.desc()
        # sample + target actor with smoothing noise + twin target critics + TD target + online
        # twin forward with the MSE gradient + each online critic's row backward: one launch,
        # rows in LDS throughout
        h, nh = c1.hidden, c1.n_hidden
        work = (prof.mlp_fwd_flops(2, 2, h, nh, B) + 4 * prof.mlp_fwd_flops(4, 1, h, nh, B) +
                2 * prof.mlp_bwd_flops(4, 1, h, nh, B, False, True))
        with prof.region("critic_rows", work):
            lib().nav_td3_critic_rows(
                C.byref(self.target_actor.desc()),
                descs(self.target_critic_network_1, self.target_critic_network_2),
                descs(c1, c2), C.byref(rd), len(replay), B, ptr(idx),
                self.seed & 0xFFFFFFFF, (self.seed >> 32) & 0xFFFFFFFF, self.update_counter,
                ptr(eps), c.policy_noise, c.noise_clip, c.max_action, c.gamma, ptr(self.batch),
                parr(self.dq1, self.dq2), parr(self.loss_part[0], self.loss_part[1]),
                parr(self.eslab1, self.eslab2), parr(self.acts1, self.acts2), mid,
                parr(self.mask1, self.mask2), int(self.row_backward), parr(self.dz1, self.dz2),
                mid, self.split_twins, s)
        if not self.row_backward:  # separate backward launch (A/B of the fusion)
            self._bwd([c1, c2], B, [self.dq1, self.dq2], 1, [self.mask1, self.mask2], s,
                      inp=self.batch, ld_in=8, in_col=0, dz=[self.dz1, self.dz2], save_mask=mid,
                      eslab=[self.eslab1, self.eslab2])

    def _critic_wgrad_args(self):
        return (self.batch, 8, 0, [self.acts1, self.acts2], [self.dz1, self.dz2],
                [self.dq1, self.dq2], 1, [self.mask1, self.mask2])

    def train_critic(self, replay, idx=None, eps=None, stream=None):
        s = stream_handle(stream)
        if self._fast():
            return self._critic_epoch_fast(replay, idx, eps, s, stream)
        self._critic_rows(replay, idx, eps, s)
        c1, c2 = self.critic_network_1, self.critic_network_2
        B = self.cfg.batch_size
        # both critics' weight gradients, then reduce + Adam: one launch each
        self._grads_and_step([c1, c2], [self.critic_optimizer_1, self.critic_optimizer_2], B,
                             *self._critic_wgrad_args(), [self.eslab1, self.eslab2],
                             [self.grad_c1, self.grad_c2], [self.hslab, self.hslab2], s, stream)

    def critic_gradients(self, replay, idx=None, eps=None, stream=None):
        """train_critic's gradient phase alone: both critics' flat gradients into the `grad_c`
        bucket ([critic 1 | critic 2], contiguous), no parameter changes. With critic_step this
        is train_critic's shared-policy path split where the collective goes."""
        s = stream_handle(stream)
        self._critic_rows(replay, idx, eps, s)
        c1, c2 = self.critic_network_1, self.critic_network_2
        splits = self._wgrad([c1, c2], self.cfg.batch_size, *self._critic_wgrad_args(),
                             [self.hslab, self.hslab2], s)
        lib().nav_grad_reduce_multi(descs(c1, c2), 2, parr(self.hslab, self.hslab2), splits,
                                    parr(self.eslab1, self.eslab2), self.nblk,
                                    parr(self.grad_c1, self.grad_c2), s)
        return self.grad_c

    def critic_step(self, grad_div=1.0, stream=None):
        """Adam on both critics from the `grad_c` bucket / grad_div (one launch)."""
        self._adam([self.critic_network_1, self.critic_network_2],
                   [self.critic_optimizer_1, self.critic_optimizer_2],
                   [self.grad_c1, self.grad_c2], stream_handle(stream), grad_div)

    def critic_loss_values(self):
        """(loss1, loss2) of the last train_critic (mean squared TD error), synchronising."""
        t = self.loss_part.sum(1) / self._B
        return t[0].item(), t[1].item()

    # robot.py:369-398
    def _actor_rows(self, replay, idx, s):
        c = self.cfg
        B = c.batch_size
        self._workspace(B)
        net = self.actor_network
        c1 = self.critic_network_1
        rd = replay.desc()
        h, nh = net.hidden, net.n_hidden
        # sample + actor forward + critic-1 forward + backward of -mean(Q) to the action + the
        # actor's row backward with its edge partials: one launch
        work = (prof.mlp_fwd_flops(2, 2, h, nh, B) + prof.mlp_fwd_flops(4, 1, h, nh, B) +
                prof.mlp_bwd_flops(4, 1, h, nh, B, True) +
                prof.mlp_bwd_flops(2, 2, h, nh, B, False, True, True))
        with prof.region("actor_rows", work):
            lib().nav_td3_actor_rows(
                C.byref(net.desc()), C.byref(c1.desc()), C.byref(rd), len(replay), B, ptr(idx),
                self.seed & 0xFFFFFFFF, (self.seed >> 32) & 0xFFFFFFFF, self.update_counter,
                ptr(self.batch2), ptr(self.q1), ptr(self.da), ptr(self.acts_a),
                net.middle_layers(), ptr(self.dz_a), net.middle_layers(),
                ptr(self.mask_a), ptr(self.mask1), ptr(self.eslab_a), s)

    def _actor_wgrad_args(self):
        return (self.batch2, 8, 0, [self.acts_a], [self.dz_a], [self.da], 2, [self.mask_a])

    def train_actor(self, replay, idx=None, stream=None, soft_update=False):
        """robot.py:369-398; with soft_update the three soft updates of robot.py:283-285 that
        follow it on a policy epoch ride in the actor's reduce + Adam launch."""
        s = stream_handle(stream)
        if self._fast():
            return self._actor_epoch_fast(replay, idx, s, stream, soft_update)
        self._actor_rows(replay, idx, s)
        self._grads_and_step([self.actor_network], [self.actor_optimizer], self.cfg.batch_size,
                             *self._actor_wgrad_args(), [self.eslab_a], [self.grad_a],
                             [self.hslab], s, stream, soft_update=soft_update)

    def actor_gradients(self, replay, idx=None, stream=None):
        """train_actor's gradient phase alone: the actor's flat gradient into `grad_a`."""
        s = stream_handle(stream)
        self._actor_rows(replay, idx, s)
        net = self.actor_network
        splits = self._wgrad([net], self.cfg.batch_size, *self._actor_wgrad_args(),
                             [self.hslab], s)
        lib().nav_grad_reduce_multi(descs(net), 1, parr(self.hslab), splits,
                                    parr(self.eslab_a), self.nblk, parr(self.grad_a), s)
        return self.grad_a

    def actor_step(self, grad_div=1.0, stream=None):
        self._adam([self.actor_network], [self.actor_optimizer], [self.grad_a],
                   stream_handle(stream), grad_div)

    def actor_loss_value(self):
        return -(self.q1.sum() / self._B).item()

    # robot.py:293-310
    def soft_update(self, target, source, tau, stream=None):
        lib().nav_polyak(C.byref(target.desc()), C.byref(source.desc()), tau,
                         stream_handle(stream))

    def soft_update_all(self, stream=None):
        """The three soft updates of robot.py:283-285 in one launch."""
        t = self.cfg.tau
        lib().nav_polyak_multi(
            descs(self.target_actor, self.target_critic_network_1, self.target_critic_network_2),
            descs(self.actor_network, self.critic_network_1, self.critic_network_2), 3, t,
            stream_handle(stream))

    # robot.py:258-285
    def td3_update(self, replay, num_epochs=None, idx_fn=None, eps_fn=None, stream=None,
                   track_losses=False, collect_ready=None):
        """`collect_ready` (a torch.cuda.Event, optional) is recorded on `stream` at the first
        point after which nothing this update still has to issue reads the replay ring or writes
        the actor: with a grad_hook and a final epoch that is not a policy epoch, just before
        that epoch's critic all-reduce (so the next collect can run beside the collective and
        the critics' Adam step), otherwise at the end."""
        n = self.cfg.num_epochs if num_epochs is None else num_epochs
        self._ready, self._ready_recorded = None, False
        try:
            self._update(replay, n, idx_fn, eps_fn, stream, track_losses, collect_ready)
        finally:
            self._ready = None
            if collect_ready is not None and not self._ready_recorded:
                collect_ready.record(stream)

    def _update(self, replay, n, idx_fn, eps_fn, stream, track_losses, collect_ready):
        if len(replay) < 1:
            return
        for epoch in range(n):
            if (collect_ready is not None and epoch == n - 1 and self.grad_hook is not None and
                    epoch % self.cfg.policy_update_delay != 0):
                self._ready = collect_ready
            self.train_critic(replay, idx=idx_fn() if idx_fn else None,
                              eps=eps_fn() if eps_fn else None, stream=stream)
            if track_losses:
                self.critic_losses.append(sum(self.critic_loss_values()) / 2)
            if epoch % self.cfg.policy_update_delay == 0:
                self.train_actor(replay, idx=idx_fn() if idx_fn else None, stream=stream,
                                 soft_update=self.fuse_soft_update)
                if track_losses:
                    self.actor_losses.append(self.actor_loss_value())
                if not self.fuse_soft_update:
                    self.soft_update_all(stream)
            self.update_counter += 1

    def networks(self):
        return {"actor": self.actor_network, "critic1": self.critic_network_1,
                "critic2": self.critic_network_2, "target_actor": self.target_actor,
                "target_critic1": self.target_critic_network_1,
                "target_critic2": self.target_critic_network_2}

    def state_dict(self):
        sd = {k: v.state_dict() for k, v in self.networks().items()}
        sd["opt"] = {k: o.state_dict() for k, o in (("actor", self.actor_optimizer),
                                                     ("critic1", self.critic_optimizer_1),
                                                     ("critic2", self.critic_optimizer_2))}
        sd["update_counter"] = self.update_counter
        return sd

    def load_state_dict(self, sd):
        for k, v in self.networks().items():
            v.load_state_dict(sd[k])
        self.actor_optimizer.load_state_dict(sd["opt"]["actor"])
        self.critic_optimizer_1.load_state_dict(sd["opt"]["critic1"])
        self.critic_optimizer_2.load_state_dict(sd["opt"]["critic2"])
        self.update_counter = sd["update_counter"]
