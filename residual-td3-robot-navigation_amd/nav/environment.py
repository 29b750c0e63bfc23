"""Drop-in `Environment` (environment.py:14-183) on the MI355X kernels.

Same constructor, attributes (robot_state, robot_init_region, goal_state, dynamics_speed,
dynamics_angle), methods and return conventions as the reference, numpy float64 in and out. All
random draws come from the global numpy legacy stream in the reference's order (so
`np.random.seed(RANDOM_SEED)` in robot-learning.py:19 gives the same goal, region, start states
and demonstrations); every arithmetic step — dynamics, step, reset, the CEM rollouts and their
path rewards — runs in libnavenv.so on the GPU. The dynamics fields come from nav.fields (the
`perlin_noise` package is absent: parity unpinned) unless injected.
"""
import ctypes as C

import numpy as np
import torch

from . import config as K
from ._lib import NavEnvSoa, lib, params_struct, ptr, require_gpu, stream_handle
from .fields import make_fields
from .vec_env import make_field


class Environment:
    def __init__(self, speed=None, angle=None, device="cuda"):
        require_gpu()
        self.device = torch.device(device)
        self._p = params_struct()
        d = self.device
        self._state = torch.zeros(1, 2, dtype=torch.float64, device=d)
        self._goal = torch.zeros(1, 2, dtype=torch.float64, device=d)
        self._region = torch.zeros(1, 4, dtype=torch.float64, device=d)
        self._u = torch.zeros(1, 2, dtype=torch.float64, device=d)
        self._a = torch.zeros(1, 2, dtype=torch.float64, device=d)
        self._soa = NavEnvSoa(1, self._state.data_ptr(), self._goal.data_ptr(),
                              self._region.data_ptr(), 0, 0, 0, 0, 0, 0)
        # environment.py:17-21
        self.robot_state = np.array([0.0, 0.0], dtype=np.float32)
        self.robot_init_region = np.array([0.0, 0.0, 0.0, 0.0], dtype=np.float32)
        self.goal_state = np.array([0.0, 0.0], dtype=np.float32)
        self.dynamics_speed = np.zeros([K.WORLD_SIZE, K.WORLD_SIZE], dtype=np.float32)
        self.dynamics_angle = np.zeros([K.WORLD_SIZE, K.WORLD_SIZE], dtype=np.float32)
        self.set_init_and_goal()
        if speed is not None:
            self.set_fields(speed, angle)
        else:
            self.set_dynamics()

    # ---- environment.py:28-56 (numpy draws, exactly the reference's sequence)
    def set_init_and_goal(self):
        r = np.random.choice([0, 1, 2, 3])
        S, W = K.INIT_REGION_SIZE, K.WORLD_SIZE
        if r == 0:
            l, rr = 0, S
            b = np.random.uniform(0, W - S)
            t = b + S
        elif r == 1:
            l = np.random.uniform(0, W - S)
            rr = l + S
            b, t = W - S, W
        elif r == 2:
            l, rr = W - S, W
            b = np.random.uniform(0, W - S)
            t = b + S
        else:
            l = np.random.uniform(0, W - S)
            rr = l + S
            b, t = 0, S
        distance = 0
        init_mid = np.array([0.5 * (l + rr), 0.5 * (b + t)])
        while distance < 90:
            random_goal = np.random.uniform(5, W - 5, 2)
            distance = np.linalg.norm(random_goal - init_mid)
        self.goal_state = random_goal
        self.robot_init_region = np.array([l, rr, b, t])
        self._goal.copy_(torch.from_numpy(np.asarray(self.goal_state, np.float64)[None]))
        self._region.copy_(torch.from_numpy(np.asarray(self.robot_init_region, np.float64)[None]))

    # ---- environment.py:59-95 (construction restated in nav.fields; parity unpinned)
    def set_dynamics(self):
        speed, angle = make_fields(K.RANDOM_SEED)
        self.set_fields(speed, angle)

    def set_fields(self, speed, angle):
        self.dynamics_speed = np.ascontiguousarray(speed, np.float32)
        self.dynamics_angle = np.ascontiguousarray(angle, np.float32)
        self._field = make_field(self.dynamics_speed, self.dynamics_angle, self.device)

    # ---- environment.py:98-119
    def dynamics(self, state, action):
        s = torch.tensor(np.asarray(state, np.float64).reshape(-1, 2), device=self.device)
        a = torch.tensor(np.asarray(action, np.float64).reshape(-1, 2), device=self.device)
        out = torch.empty_like(s)
        lib().nav_dynamics(ptr(self._field), ptr(s), ptr(a), ptr(out), s.shape[0],
                           stream_handle())
        out = out.cpu().numpy()
        return out[0] if np.ndim(state) == 1 else out

    # ---- environment.py:122-127: returns the committed state object (unchanged object if not)
    def step(self, action):
        self._state.copy_(torch.from_numpy(np.asarray(self.robot_state, np.float64)[None]))
        self._a.copy_(torch.from_numpy(np.asarray(action, np.float64).reshape(1, 2)))
        nxt = torch.empty_like(self._state)
        lib().nav_env_step(C.byref(self._p), C.byref(self._soa), ptr(self._field), ptr(self._a),
                           ptr(nxt), stream_handle())
        n = nxt.cpu().numpy()[0]
        if 0 <= n[0] < K.WORLD_SIZE and 0 <= n[1] < K.WORLD_SIZE:
            self.robot_state = n
        return self.robot_state

    # ---- environment.py:130-137
    def reset(self):
        self.robot_state = self.get_random_robot_init_state()
        return self.robot_state

    def get_random_robot_init_state(self):
        # np.random.uniform([l, b], [r, t], 2): two random_sample draws, low + (high-low)*u on GPU
        u = np.random.random_sample(2)
        self._u.copy_(torch.from_numpy(u[None]))
        lib().nav_env_reset(C.byref(self._p), C.byref(self._soa), None, ptr(self._u),
                            stream_handle())
        return self._state.cpu().numpy()[0].copy()

    # ---- environment.py:140-179: CEM, rollouts on the GPU
    def get_demonstration(self):
        I, P, T, E = (K.DEMOS_CEM_NUM_ITERATIONS, K.DEMOS_CEM_NUM_PATHS,
                      K.DEMOS_CEM_PATH_LENGTH, K.DEMOS_CEM_NUM_ELITES)
        planning_actions = np.zeros([I, P, T, 2], dtype=np.float32)
        planning_paths = np.zeros([I, P, T + 1, 2], dtype=np.float32)
        planning_path_rewards = np.zeros([I, P])
        start = self.get_random_robot_init_state()
        d = self.device
        st = torch.tensor(np.repeat(start[None], P, 0), device=d)
        paths = torch.zeros(P, T + 1, 2, dtype=torch.float64, device=d)
        rew = torch.zeros(P, dtype=torch.float64, device=d)
        goal = torch.tensor(np.asarray(self.goal_state, np.float64), device=d)
        mean = std = None
        for it in range(I):
            # the reference draws per (path, step) in this order; a size-(P,T,2) draw is the same
            # stream (legacy randint / polar gauss, element after element)
            if it == 0:
                acts = np.random.choice([-K.ROBOT_MAX_ACTION, K.ROBOT_MAX_ACTION], (P, T, 2))
                acts = acts.astype(np.float64)
            else:
                g = np.random.standard_normal((P, T, 2))
                acts = mean.astype(np.float64)[None] + std.astype(np.float64)[None] * g
            planning_actions[it] = acts
            a = torch.tensor(acts, device=d)
            lib().nav_rollout(ptr(self._field), P, T, ptr(st), ptr(a), ptr(paths), ptr(goal),
                              ptr(rew), stream_handle())
            planning_paths[it] = paths.cpu().numpy()
            planning_path_rewards[it] = rew.cpu().numpy()
            order = np.argsort(planning_path_rewards[it].copy())
            best = order[-E:]
            mean = np.mean(planning_actions[it, best], axis=0)
            std = np.std(planning_actions[it, best], axis=0)
        index_best_path = np.argmax(planning_path_rewards[-1])
        return planning_paths[-1, index_best_path, 0:T], planning_actions[-1, index_best_path]

    # environment.py:182-183
    def compute_reward(self, path):
        return -np.linalg.norm(path[-1] - self.goal_state)
