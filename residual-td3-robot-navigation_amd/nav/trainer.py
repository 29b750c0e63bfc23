"""Vectorised residual-TD3 training loop on one GPU (the MI355X form of robot-learning.py's
training mode, robot-learning.py:54-101, for n independent envs at once).

One `step()` = one vector tick: every env selects an action (actor MLP + baseline + exploration
noise) and takes one environment step with the fused reward / stuck / done / replay-push /
auto-reset tick, both in ONE launch (nav_act_tick), then the learner runs `updates_per_step`
TD3 epochs (robot.py:272-285: critic every epoch, actor + Polyak every `policy_update_delay`-th)
on batches sampled from the device replay ring. The reference's schedule (100 epochs of batch
100 at every episode end) does not map onto 65 536 asynchronous envs; the update-to-data ratio
here is updates_per_step * batch / n_envs sampled transitions per collected transition.
"""
import ctypes as C

import numpy as np
import torch

from . import config as K
from . import prof
from ._lib import lib, ptr, stream_handle
from .cem import cem_group_demo_sets
from .fields import make_field_device
from .td3 import TD3
from .vec_env import ReplayRing, VecEnv


class VecTrainer:
    def __init__(self, n_envs=65536, hidden=256, n_hidden=2, batch=32768, updates_per_step=2,
                 replay_capacity=None, seed=K.RANDOM_SEED, envs_per_group=1024, demos=True,
                 device="cuda", field=None, grad_hook=None, fuse_tick=True, overlap_collect=False):
        self.n = int(n_envs)
        self.device = torch.device(device)
        self.seed = int(seed)
        if field is None:  # set_dynamics on the device (nav_fields_generate)
            field = make_field_device(self.seed, self.device)
        self.field = field
        epg = int(envs_per_group) if envs_per_group else self.n
        self.env = VecEnv(self.n, field, seed=self.seed, envs_per_group=epg, demo_flag=demos,
                          device=self.device)
        if demos:
            G = (self.n + epg - 1) // epg
            firsts = torch.arange(G, device=self.device) * epg
            regions = self.env.region[firsts].cpu().numpy()
            goals = self.env.goal[firsts].cpu().numpy()
            # each group's 3 demonstrations from the batched GPU CEM (environment.py:140-179) +
            # their augmentations (robot.py:771-824), as the reference's robot acquires them
            pts, off = cem_group_demo_sets(self.field, regions, goals, self.seed,
                                           device=self.device)
            self.env.set_demo(pts, off if G > 1 else None)
        cfg = K.TD3Config(batch_size=int(batch), num_epochs=int(updates_per_step),
                          net=K.NetConfig(hidden=hidden, n_hidden=n_hidden))
        self.td3 = TD3(cfg, device=self.device, seed=self.seed, grad_hook=grad_hook)
        cap = replay_capacity or max(4 * self.n, 2 * int(batch), K.BUFFER_SIZE)
        self.replay = ReplayRing(cap, self.device)
        self.action = torch.zeros(self.n, 2, dtype=torch.float64, device=self.device)
        self.steps = 0
        self.updates_per_step = int(updates_per_step)
        # act + tick fused into one launch (False: the two launches; A/B and the fused-vs-unfused
        # parity test)
        self.fuse_tick = bool(fuse_tick)
        # shared policy: the next step's collect on a second stream beside the last epoch's
        # critic all-reduce and Adam step (bit-identical either way). Off by default: the two
        # cross-stream waits per step cost ~24 us on one MI355X (profiles/r05u_shared_policy_host
        # .json), so it pays only where the collective itself takes longer than that.
        self.overlap_collect = bool(overlap_collect)
        self._side = None
        self._collect_ready = None  # recorded by the last learn() (td3_update collect_ready)
        self._collected = None

    # robot.py:541-569 for every env
    def act(self, training=True, stream=None):
        net = self.td3.actor_network
        a = net.desc()
        with prof.region("act", prof.mlp_fwd_flops(2, 2, net.hidden, net.n_hidden, self.n)):
            lib().nav_act(C.byref(self.env.p), C.byref(a), self.n, ptr(self.env.state),
                          ptr(self.env.goal), ptr(self.env.noise_scale), None, self.steps,
                          0 if training else 1, ptr(self.action), None, stream_handle(stream))
        return self.action

    def collect(self, stream=None):
        if self.fuse_tick and (self.env.demo_xy is None or self.env.demo_index is not None):
            # one launch: action selection + the tick (nav_act_tick)
            self.env.act_tick(self.td3.actor_network, self.steps, self.replay,
                              action_out=self.action, stream=stream)
        else:
            self.act(True, stream)
            self.env.agent_step(self.action, self.replay, stream)
        self.steps += 1

    def learn(self, stream=None, collect_ready=None):
        if len(self.replay) >= self.td3.cfg.batch_size and self.updates_per_step > 0:
            self.td3.td3_update(self.replay, self.updates_per_step, stream=stream,
                                collect_ready=collect_ready)
        elif collect_ready is not None:
            collect_ready.record(stream)

    def step(self, stream=None):
        if not self.overlap_collect or prof._active is not None:
            self.sync_collect()
            self.collect(stream)
            self.learn(stream)
            return
        # overlapped form (shared policy): this collect reads only the actor and the env state
        # and writes the env state and the replay ring, so it may start once the previous learn
        # has issued its last replay read and actor write (td3_update's collect_ready: before
        # the final critic-only epoch's all-reduce); the learn waits for the collect
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
            self._collected = torch.cuda.Event()
        side = self._side
        if self._collect_ready is None:
            side.wait_stream(main)
        else:
            side.wait_event(self._collect_ready)
        self.collect(side)
        self._collected.record(side)
        main.wait_event(self._collected)
        if self._collect_ready is None:
            self._collect_ready = torch.cuda.Event()
        self.learn(main, self._collect_ready)

    def sync_collect(self):
        """Make the next step's collect wait for everything issued on the current stream (after
        host-side changes to the env state, the replay ring or the actor between steps)."""
        self._collect_ready = None

    def env_steps(self):
        return self.steps * self.n

    # ---- checkpoint / resume: every piece of state the next step reads
    ENV_STATE = ("state", "goal", "region", "hist", "meta", "plan_index", "path_length",
                 "episodes", "noise_scale")

    def state_dict(self):
        """The trainer's whole state as host tensors and plain values (torch.save-able, loadable
        with weights_only=True): per-env SoA state, field, demo set, replay ring, learner (nets,
        Adam moments, counters) and the step counter that keys the exploration noise. A trainer
        restored from it continues bit for bit as the original would have."""
        e = self.env
        return {
            "meta": {"n_envs": self.n, "seed": self.seed, "envs_per_group": e.envs_per_group,
                     "hidden": self.td3.actor_network.hidden,
                     "n_hidden": self.td3.actor_network.n_hidden,
                     "batch": self.td3.cfg.batch_size, "updates_per_step": self.updates_per_step,
                     "steps": self.steps},
            "env": {k: getattr(e, k).detach().cpu() for k in self.ENV_STATE},
            "field": self.field.detach().cpu(),
            "demo_xy": None if e.demo_xy is None else e.demo_xy.cpu(),
            "demo_off": None if e.demo_off is None else e.demo_off.cpu(),
            "replay": {"rows": self.replay.rows.cpu(), "position": self.replay.position,
                       "size": self.replay.size},
            "td3": self.td3.state_dict(),
        }

    def load_state_dict(self, sd):
        m = sd["meta"]
        assert (m["n_envs"], m["envs_per_group"]) == (self.n, self.env.envs_per_group)
        assert sd["replay"]["rows"].shape == self.replay.rows.shape
        for k in self.ENV_STATE:
            getattr(self.env, k).copy_(sd["env"][k].to(self.device))
        self.field.copy_(sd["field"].to(self.device))
        if sd["demo_xy"] is not None:
            self.env.set_demo(sd["demo_xy"], sd["demo_off"])
        self.replay.rows.copy_(sd["replay"]["rows"].to(self.device))
        self.replay.position = int(sd["replay"]["position"])
        self.replay.size = int(sd["replay"]["size"])
        self.td3.load_state_dict(sd["td3"])
        self.steps = int(m["steps"])
        self.updates_per_step = int(m["updates_per_step"])
        self.sync_collect()

    @classmethod
    def from_state_dict(cls, sd, device="cuda", grad_hook=None):
        """A trainer resumed from state_dict() without re-running the field generator or the CEM
        (their results are in the checkpoint)."""
        m = sd["meta"]
        t = cls(n_envs=m["n_envs"], hidden=m["hidden"], n_hidden=m["n_hidden"],
                batch=m["batch"], updates_per_step=m["updates_per_step"],
                replay_capacity=sd["replay"]["rows"].shape[0], seed=m["seed"],
                envs_per_group=m["envs_per_group"], demos=False, device=device,
                field=sd["field"].to(device), grad_hook=grad_hook)
        t.load_state_dict(sd)
        return t

    def save(self, path):
        torch.save(self.state_dict(), path)

    @classmethod
    def load(cls, path, device="cuda", grad_hook=None):
        return cls.from_state_dict(torch.load(path, weights_only=True), device, grad_hook)
