"""BASELINE config 1 end to end on one MI355X: the headless robot-learning.py loop (nav.driver)
through the drop-in Environment / Robot, budget disabled, until 200 episodes, with the
reference's own learner schedule (td3_update at every episode end: 100 epochs of batch 100,
3 x 200 MLPs). Prints one JSON line: wall time, env-steps, env-steps/s, and where the time went
(td3_update, CEM demonstrations, the per-step path), beside SURVEY §6's reference timing of the
same run in this container (215 s, 2 660 env-steps, 12.4 env-steps/s).

python tools/config1_run.py [episodes] [seed]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "residual-td3-robot-navigation_amd"))

import torch  # noqa: E402


class Timed:
    """wraps a bound method: synchronises the device after each call and sums the wall time"""

    def __init__(self, fn):
        self.fn, self.calls, self.s = fn, 0, 0.0

    def __call__(self, *a, **k):
        t0 = time.perf_counter()
        r = self.fn(*a, **k)
        torch.cuda.synchronize()
        self.s += time.perf_counter() - t0
        self.calls += 1
        return r


def main():
    from nav import driver
    from nav.environment import Environment
    from nav.robot import Robot
    episodes = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else None
    timers = {}

    class TimedRobot(Robot):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            for name in ("process_transition", "get_next_action_training"):
                timers[name] = Timed(getattr(self, name))
                setattr(self, name, timers[name])
            timers["td3_update"] = Timed(self.td3_agent.td3_update)
            self.td3_agent.td3_update = timers["td3_update"]

    class TimedEnvironment(Environment):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            for name in ("get_demonstration", "step", "reset"):
                timers[name] = Timed(getattr(self, name))
                setattr(self, name, timers[name])

    kw = {} if seed is None else {"seed": seed}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = driver.run(environment_cls=TimedEnvironment, robot_cls=TimedRobot, budget=False,
                   verbose=False, max_episodes=episodes, **kw)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    robot = r["robot"]
    out = {
        "workload": "config1: headless robot-learning.py loop, 1 env, budget off, "
                    f"{episodes} episodes, td3_update 100 epochs x batch 100 per episode end, "
                    "3x200 MLPs, generated fields",
        "episodes": robot.num_episodes, "ticks": r["ticks"], "env_steps": r["steps"],
        "resets": r["resets"], "demos": r["demos"], "wall_s": round(wall, 3),
        "env_steps_per_s": round(r["steps"] / wall, 1),
        "replay_rows": len(robot.memory),
        "time_s": {k: round(v.s, 3) for k, v in timers.items()},
        "calls": {k: v.calls for k, v in timers.items()},
        "per_call_ms": {k: round(1e3 * v.s / max(1, v.calls), 3) for k, v in timers.items()},
        "reference_same_run_this_container": {
            "wall_s": 215, "env_steps": 2660, "resets": 196, "demos": 3, "td3_update_s": 199,
            "env_steps_per_s": 12.4, "source": "SURVEY.md §6 (Intel Xeon, 8 cores, torch CPU)"},
        "note": "episode lengths and counts follow the policy being learned, so env_steps differs "
                "from the reference run; compare per-call costs and env-steps/s",
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
