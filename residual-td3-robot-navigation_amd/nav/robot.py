"""Drop-in `robot.py` (ReplayBuffer, Residual_Actor_Network, Residual_Critic_Network, TD3, Robot)
on the MI355X kernels, for robot-learning.py's single-env loop.

Same class names, constructor arguments, attributes, method names, return types and numpy-stream
consumption as the reference (robot.py:58-824): every np.random draw the reference makes is made
here in the same order (exploration noise, replay sampling permutations, demonstration
augmentation), target-smoothing noise comes from the global torch generator as in robot.py:338.
The math runs in libnavenv.so: actor forward + action epilogue (nav_act), reward / stuck / done /
replay push (nav_transition, nav_demo_reward, nav_compute_reward, nav_check_if_stuck), the TD3
update (nav.td3 on MFMA). The control flow (get_next_action_type, Robot.reset) is the reference's.
"""
import ctypes as C

import numpy as np
import torch

from . import config as K
from ._lib import NavEnvSoa, NavReplay, NavStepOut, lib, params_struct, ptr, require_gpu, \
    stream_handle
from .demos import augment
from .mlp import DeviceMLP, forward
from .td3 import TD3 as _GpuTD3
from .vec_env import ReplayRing

# robot.py:21-54
NUM_DEMO, NUM_AUGMENTS, AUG_NOISE, AUG_INTERPOLATION = (K.NUM_DEMO, K.NUM_AUGMENTS, K.AUG_NOISE,
                                                        K.AUG_INTERPOLATION)
PATH_LENGTH, PATH_INCREASE = K.PATH_LENGTH, K.PATH_INCREASE
INITIAL_NOISE, NOISE_DECAY = K.INITIAL_NOISE, K.NOISE_DECAY
BUFFER_SIZE = K.BUFFER_SIZE
STUCK_THRESHOLD, STUCK_STEPS, STUCK_PENALTY = K.STUCK_THRESHOLD, K.STUCK_STEPS, K.STUCK_PENALTY
GOAL_REWARD, DEMO_PROXIMITY_FACTOR = K.GOAL_REWARD, K.DEMO_PROXIMITY_FACTOR
ACTOR_LR, CRITIC_LR, POLICY_UPDATE_DELAY = K.ACTOR_LR, K.CRITIC_LR, K.POLICY_UPDATE_DELAY
TARGET_POLICY_NOISE, NOISE_CLIP = K.TARGET_POLICY_NOISE, K.NOISE_CLIP
TD3_EPOCHS, TD3_BATCH_SIZE, GAMMA, TAU = K.TD3_EPOCHS, K.TD3_BATCH_SIZE, K.GAMMA, K.TAU

_DEV = "cuda"


class PathToDraw:
    """graphics.PathToDraw stand-in (visualisation data only; pyglet is not needed)."""

    def __init__(self, path, colour, width):
        self.path = path
        self.colour = colour
        self.width = width


class ReplayBuffer(ReplayRing):
    """robot.py:58-124 on a device ring of float32 rows (what train_critic feeds torch anyway)."""

    def __init__(self, capacity, device=_DEV):
        super().__init__(capacity, device)
        self._one = torch.zeros(5, 2, dtype=torch.float64, device=device)
        self._done = torch.zeros(1, dtype=torch.uint8, device=device)

    @property
    def buffer(self):
        return self.rows[:self.size]

    def push(self, state, action, reward, next_state, done):
        t = torch.tensor(np.stack([np.asarray(state, np.float64), np.asarray(action, np.float64),
                                   np.array([float(reward), 0.0]),
                                   np.asarray(next_state, np.float64), np.zeros(2)]))
        self._one.copy_(t)
        self._done.fill_(1 if done else 0)
        rd = self.desc()
        o = self._one
        lib().nav_replay_push(C.byref(rd), self.position, 1, ptr(o[0]), ptr(o[1]), ptr(o[2]),
                              ptr(o[3]), ptr(self._done), stream_handle())
        self.advance(1)

    def sample(self, batch_size):
        if self.size < batch_size:
            return None
        samples = np.random.choice(self.size, batch_size, replace=False)
        r = self.rows[torch.as_tensor(samples, device=self.rows.device)].cpu().numpy()
        r = r.astype(np.float64)
        return r[:, 0:2], r[:, 2:4], r[:, 4], r[:, 5:7], r[:, 7] > 0.5


def Residual_Actor_Network(hidden=200, n_hidden=3, generator=None, device=_DEV):
    """robot.py:128-165: 2 -> 200 x3 -> 2, ReLU, Kaiming-uniform weights, zero biases."""
    return DeviceMLP(2, 2, hidden, n_hidden, device).init_kaiming(generator)


def Residual_Critic_Network(hidden=200, n_hidden=3, generator=None, device=_DEV):
    """robot.py:168-206: cat(s, a) 4 -> 200 x3 -> 1."""
    return DeviceMLP(4, 1, hidden, n_hidden, device).init_kaiming(generator)


class TD3(_GpuTD3):
    """robot.py:209-398 with the reference's constructor and td3_update(replay_buffer)."""

    def __init__(self, actor_network, critic_network_1, critic_network_2, actor_lr=ACTOR_LR,
                 critic_lr=CRITIC_LR, gamma=GAMMA, tau=TAU, policy_noise=TARGET_POLICY_NOISE,
                 noise_clip=NOISE_CLIP, policy_update_delay=POLICY_UPDATE_DELAY,
                 num_epochs=TD3_EPOCHS, batch_size=TD3_BATCH_SIZE):
        net = K.NetConfig(hidden=actor_network.hidden, n_hidden=actor_network.n_hidden)
        cfg = K.TD3Config(actor_lr=actor_lr, critic_lr=critic_lr, gamma=gamma, tau=tau,
                          policy_noise=policy_noise, noise_clip=noise_clip,
                          policy_update_delay=policy_update_delay,
                          max_action=K.ROBOT_MAX_ACTION, batch_size=batch_size,
                          num_epochs=num_epochs, net=net)
        super().__init__(cfg, actor_network.device, actor=actor_network,
                         critic1=critic_network_1, critic2=critic_network_2)
        self.gamma, self.tau = gamma, tau
        self.policy_noise, self.noise_clip = policy_noise, noise_clip
        self.policy_update_delay = policy_update_delay
        self.max_action = K.ROBOT_MAX_ACTION
        self.num_epochs, self.batch_size = num_epochs, batch_size

    def td3_update(self, replay_buffer):
        """robot.py:258-285: the replay sampling permutations come from np.random exactly as
        ReplayBuffer.sample draws them (robot.py:111), one per train_critic and one per
        train_actor, in epoch order; the smoothing noise from torch.randn(B, 2) per critic epoch.
        Each epoch's draws are taken on the host right before its launches (the same streams, the
        same order) into pinned host slots that the row kernels read directly (zero-copy: 100
        indices and 200 noise values per epoch, no copy launch), so the host's sampling of epoch
        e+1 (numpy's full permutation of the buffer: the larger host cost) runs while the device
        works on epoch e; no host round trip between epochs. A slot is written once per update;
        the next update waits for the last launch of this one before reusing them."""
        B, dev = self.batch_size, self.device
        if len(replay_buffer) < B:
            raise TypeError("cannot unpack non-iterable NoneType object")  # robot.py:326
        # the reference's attributes are the live hyper-parameters (a caller may set them between
        # updates, as the reference's own td3_update reads self.* each time)
        c = self.cfg
        c.batch_size, c.gamma, c.tau = B, self.gamma, self.tau
        c.policy_noise, c.noise_clip = self.policy_noise, self.noise_clip
        c.policy_update_delay, c.num_epochs = self.policy_update_delay, self.num_epochs
        c.max_action = self.max_action  # robot.py:339's clamp
        L = len(replay_buffer)
        n_idx = self.num_epochs + (self.num_epochs + self.policy_update_delay - 1) // \
            self.policy_update_delay
        # the previous update's kernels read the pinned slots through raw pointers: wait for them
        # before the slots are rewritten OR freed (torch's caching host allocator may hand a freed
        # block straight to the next pin_memory())
        if getattr(self, "_pin_done", None) is not None:
            self._pin_done.synchronize()
            self._pin_done = None
        pin = getattr(self, "_pin", None)
        if pin is None or pin[0].shape != (n_idx, B) or pin[1].shape[0] != self.num_epochs:
            pin = (torch.empty(n_idx, B, dtype=torch.int64).pin_memory(),
                   torch.empty(self.num_epochs, B, 2).pin_memory())
            self._pin = pin
        h_idx, h_eps = pin
        cnt = {"i": 0, "e": 0}

        def idx_fn():
            k = cnt["i"]
            cnt["i"] += 1
            h_idx[k].numpy()[:] = np.random.choice(L, B, replace=False)
            return h_idx[k]

        def eps_fn():
            k = cnt["e"]
            cnt["e"] += 1
            h_eps[k].copy_(torch.randn(B, 2))
            return h_eps[k]
        super().td3_update(replay_buffer, self.num_epochs, idx_fn=idx_fn, eps_fn=eps_fn)
        self._pin_done = torch.cuda.Event()
        self._pin_done.record()


class Robot:
    def __init__(self, goal_state, device=_DEV):
        require_gpu()
        self.device = torch.device(device)
        self.goal_state = goal_state
        self.paths_to_draw = []
        self.demonstration_states = []
        self.demonstration_actions = []
        self.num_episodes = 0
        self.current_noise_scale = INITIAL_NOISE
        self.path_length = PATH_LENGTH
        self.plan_index = 0
        self.memory = ReplayBuffer(BUFFER_SIZE, device)
        self.td3_agent = TD3(actor_network=Residual_Actor_Network(device=device),
                             critic_network_1=Residual_Critic_Network(device=device),
                             critic_network_2=Residual_Critic_Network(device=device))
        self.goal_reached = False
        self.demo_flag = False
        self.stuck_flag = False
        # one-env device state for the per-step kernels
        d = self.device
        f64 = dict(dtype=torch.float64, device=d)
        self._p = params_struct()
        self._goal = torch.zeros(1, 2, **f64)
        self._hist = torch.zeros(5, 1, 2, **f64)
        self._meta = torch.zeros(1, dtype=torch.int32, device=d)
        self._plan = torch.zeros(1, dtype=torch.int32, device=d)
        self._path = torch.zeros(1, dtype=torch.int32, device=d)
        self._sas = torch.zeros(3, 1, 2, **f64)  # state, action, next state
        self._noise = torch.zeros(1, 2, **f64)
        self._sigma = torch.zeros(1, **f64)
        self._act = torch.zeros(1, 2, **f64)
        self._ns_out = torch.zeros(1, 2, **f64)
        self._gterm = torch.zeros(1, **f64)
        self._flags = torch.zeros(1, dtype=torch.uint8, device=d)
        self._reward = torch.zeros(1, **f64)
        self._stuck = torch.zeros(1, dtype=torch.uint8, device=d)
        self._demo = torch.zeros(0, 2, **f64)
        self._soa = NavEnvSoa(1, 0, self._goal.data_ptr(), 0, self._hist.data_ptr(),
                              self._meta.data_ptr(), self._plan.data_ptr(),
                              self._path.data_ptr(), 0, 0)
        self._out = NavStepOut(self._ns_out.data_ptr(), self._gterm.data_ptr(),
                               self._flags.data_ptr(), 0)

    # ---- robot.py:443-489 (control flow, verbatim semantics)
    def get_next_action_type(self, state, money_remaining):
        action_type = 'step'
        if (self.num_episodes <= NUM_DEMO) and not self.demo_flag:
            self.num_episodes += 1
            action_type = 'demo'
        if (self.num_episodes > NUM_DEMO) and not self.demo_flag:
            self.demo_flag = True
            self.num_episodes += 1
            action_type = 'reset'
        if self.plan_index == (self.path_length - 1) or self.goal_reached or self.stuck_flag:
            self.reset()
            self.td3_agent.td3_update(self.memory)
            action_type = 'reset'
        else:
            self.plan_index += 1
        return action_type

    # robot.py:492-506
    def reset(self):
        self.num_episodes += 1
        self.plan_index = 0
        self.goal_reached = False
        self.stuck_flag = False
        self.current_noise_scale *= NOISE_DECAY
        self.path_length += PATH_INCREASE

    @property
    def previous_states(self):
        """robot.py:425 view of the device history ring, oldest first."""
        meta = int(self._meta.item())
        cnt, head = (meta >> 8) & 7, (meta >> 12) & 7
        h = self._hist[:, 0].cpu().numpy()
        return [h[(head + i) % 5].copy() for i in range(cnt)]

    # robot.py:509-538
    def check_if_stuck(self, state):
        self._sas[0, 0] = torch.as_tensor(np.asarray(state, np.float64))
        lib().nav_check_if_stuck(C.byref(self._p), C.byref(self._soa), ptr(self._sas[0]),
                                 ptr(self._stuck), stream_handle())
        return bool(self._stuck.item())

    def _upload_goal(self):
        self._goal.copy_(torch.as_tensor(np.asarray(self.goal_state, np.float64)).view(1, 2))

    # robot.py:541-569
    def get_next_action_training(self, state, money_remaining):
        z = np.random.normal(0, 1, size=2)  # generate_noise's draws, scaled on the device
        return self._act_gpu(state, z)

    # robot.py:572-595
    def get_next_action_testing(self, state):
        return self._act_gpu(state, None)

    def _act_gpu(self, state, z):
        self._upload_goal()
        self._sas[0, 0] = torch.as_tensor(np.asarray(state, np.float64))
        self._sigma.fill_(float(self.current_noise_scale))
        if z is not None:
            self._noise.copy_(torch.as_tensor(z).view(1, 2))
        a = self.td3_agent.actor_network.desc()
        lib().nav_act(C.byref(self._p), C.byref(a), 1, ptr(self._sas[0]), ptr(self._goal),
                      ptr(self._sigma), ptr(self._noise) if z is not None else None, 0,
                      0 if z is not None else 1, ptr(self._act), None, stream_handle())
        return self._act.cpu().numpy()[0].copy()

    # robot.py:598-624
    def residual_action(self, state):
        x = torch.tensor(np.asarray(state, np.float32).reshape(1, 2), device=self.device)
        out = torch.zeros(1, 2, device=self.device)
        forward([self.td3_agent.actor_network], x, 2, 0, [out], 2, 0, 1)
        return out.cpu().numpy()[0]

    # robot.py:627-642
    def generate_noise(self, action):
        return np.random.normal(0, self.current_noise_scale * K.ROBOT_MAX_ACTION,
                                size=action.shape)

    def _sync_meta(self):
        bits = (1 if self.goal_reached else 0) | (2 if self.stuck_flag else 0) | \
               (4 if self.demo_flag else 0)
        self._meta.bitwise_and_(~7).bitwise_or_(bits)

    # robot.py:645-675
    def process_transition(self, state, action, next_state, money_remaining):
        self._upload_goal()
        self._sync_meta()
        self._plan.fill_(int(self.plan_index))
        self._path.fill_(int(self.path_length))
        self._sas.copy_(torch.as_tensor(np.stack([np.asarray(state, np.float64),
                                                  np.asarray(action, np.float64),
                                                  np.asarray(next_state, np.float64)]))
                        .view(3, 1, 2))
        rd = self.memory.desc()
        base = self.memory.position
        s = stream_handle()
        has_demo = self._demo.shape[0] > 0
        lib().nav_transition(C.byref(self._p), C.byref(self._soa), ptr(self._sas[0]),
                             ptr(self._sas[1]), ptr(self._sas[2]), C.byref(rd), base,
                             C.byref(self._out), int(has_demo), s)
        if has_demo:
            lib().nav_demo_reward(C.byref(self._p), 1, ptr(self._ns_out), ptr(self._gterm),
                                  ptr(self._flags), ptr(self._demo), None, self._demo.shape[0],
                                  1, C.byref(rd), base, None, None, s)
        self.memory.advance(1)
        meta = int(self._meta.item())
        self.goal_reached = bool(meta & 1)
        self.stuck_flag = bool(meta & 2)

    # robot.py:679-718
    def process_demonstration(self, demonstration_states, demonstration_actions,
                              money_remaining):
        self.demonstration_states.extend(demonstration_states)
        self.demonstration_actions.extend(demonstration_actions)
        self.augment_demonstration_data(demonstration_states, demonstration_actions)
        self.draw_path(demonstration_states, colour=[0, 255, 0], width=2)
        n = len(demonstration_states) - 1
        if n < 1:  # a 1-state demonstration has no transition: the reference pushes nothing
            self.goal_reached = False
            return
        ds = np.asarray(demonstration_states, np.float64)
        rewards = self._compute_rewards(ds[1:n + 1])
        done = np.zeros(n, np.uint8)
        done[n - 1] = 1
        d = self.device
        t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=d)  # noqa: E731
        st, ac = t(ds[:n]), t(np.asarray(demonstration_actions, np.float64)[:n])
        rw, s2, dn = t(rewards), t(ds[1:n + 1]), t(done)
        rd = self.memory.desc()
        lib().nav_replay_push(C.byref(rd), self.memory.position, n, ptr(st), ptr(ac), ptr(rw),
                              ptr(s2), ptr(dn), stream_handle())
        self.memory.advance(n)
        self.goal_reached = False

    def dynamics_model(self, state, action):  # robot.py:721-723 (unused by the reference)
        return state + action

    def _compute_rewards(self, next_states):
        """compute_reward([s']) for many s' at once (the demo set is fixed during the batch);
        sets goal_reached if any reached the goal, as the reference's per-call side effect."""
        self._upload_goal()
        ns = torch.as_tensor(np.ascontiguousarray(next_states, np.float64), device=self.device)
        n = ns.shape[0]
        goal = self._goal.expand(n, 2).contiguous()
        out = torch.zeros(n, dtype=torch.float64, device=self.device)
        hit = torch.zeros(n, dtype=torch.uint8, device=self.device)
        lib().nav_compute_reward(C.byref(self._p), n, ptr(ns), ptr(goal), ptr(self._demo),
                                 self._demo.shape[0], int(self.demo_flag), ptr(out), ptr(hit),
                                 stream_handle())
        if bool(hit.any().item()):
            self.goal_reached = True
        return out.cpu().numpy()

    # robot.py:727-762 (a path of several states averages the per-state minima)
    def compute_reward(self, path):
        path = [np.asarray(p, np.float64) for p in path]
        goal_distance_reward = -np.linalg.norm(path[-1] - self.goal_state)
        if goal_distance_reward >= -K.TEST_DISTANCE_THRESHOLD:
            self.goal_reached = True
            return GOAL_REWARD
        if not self.demonstration_states:
            return goal_distance_reward
        pts = torch.as_tensor(np.ascontiguousarray(path), device=self.device)
        mins = torch.zeros(len(path), dtype=torch.float64, device=self.device)
        lib().nav_demo_min(ptr(pts), len(path), ptr(self._demo), self._demo.shape[0], ptr(mins),
                           stream_handle())
        avg_min_distance = np.mean(mins.cpu().numpy())
        demo_proximity_reward = -avg_min_distance if self.demo_flag else 0
        return goal_distance_reward + (DEMO_PROXIMITY_FACTOR * demo_proximity_reward)

    def draw_path(self, path, colour=[255, 255, 255], width=2):
        self.paths_to_draw.append(PathToDraw(path, colour=colour, width=width))

    # robot.py:771-824
    def augment_demonstration_data(self, demonstration_states, demonstration_actions,
                                   noise_level=AUG_NOISE, interpolation_steps=AUG_INTERPOLATION,
                                   num_augmentations=NUM_AUGMENTS):
        for s, a in augment(demonstration_states, demonstration_actions, np.random, noise_level,
                            interpolation_steps, num_augmentations):
            self.draw_path(s, colour=[0, 0, 255], width=2)
            self.demonstration_states.extend(list(s))
            self.demonstration_actions.extend(list(a))
        self._demo = torch.as_tensor(
            np.asarray([np.asarray(x, np.float64) for x in self.demonstration_states]),
            device=self.device).reshape(-1, 2).contiguous()
