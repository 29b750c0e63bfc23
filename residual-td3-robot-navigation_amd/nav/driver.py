"""Headless robot-learning.py (robot-learning.py:18-132 minus pyglet/graphics).

`run()` reproduces the reference's update() state machine: the money budget (demos 20, resets 5,
steps 0.01, wall-clock seconds 0.03; robot-learning.py:45-50), the training -> testing switch,
and the test episode (success at <= 5 from the goal, 100 s timeout). The 10 Hz pyglet clock
(robot-learning.py:129) is replaced by a plain loop; `tick_rate` re-imposes it when wanted.
Works with the reference's own Environment/Robot classes or with nav's drop-ins.
"""
import time

import numpy as np

from . import config as K


def run(environment_cls=None, robot_cls=None, seed=K.RANDOM_SEED, max_ticks=None,
        budget=True, test_timeout=K.TEST_TIMEOUT, tick_rate=None, verbose=True, env_kwargs=None,
        max_episodes=None):
    """max_episodes: end the run (in training mode) once robot.num_episodes reaches it — the
    SURVEY §6 config-1 timing ("200 episodes, budget disabled")."""
    if environment_cls is None:
        from .environment import Environment as environment_cls
    if robot_cls is None:
        from .robot import Robot as robot_cls
    log = print if verbose else (lambda *a, **k: None)
    np.random.seed(seed)  # robot-learning.py:19
    environment = environment_cls(**(env_kwargs or {}))
    state = environment.reset()
    robot = robot_cls(environment.goal_state)
    mode = "training"
    demos_bought = resets_bought = steps_bought = 0
    test_init_time = 0.0
    test_best_distance = np.inf
    penalty = False
    train_init_time = time.time()
    result = {"reached": False, "ticks": 0}

    def remaining():
        spent = (demos_bought * K.COST_PER_DEMO + resets_bought * K.COST_PER_RESET +
                 steps_bought * K.COST_PER_STEP +
                 (time.time() - train_init_time) * K.COST_PER_CPU_SECOND)
        return K.STARTING_MONEY - spent if budget else np.inf

    ticks = 0
    while max_ticks is None or ticks < max_ticks:
        t0 = time.time()
        ticks += 1
        if mode == "training":
            if max_episodes is not None and robot.num_episodes >= max_episodes:
                break
            money = remaining()
            action_type = robot.get_next_action_type(state, money)
            money = remaining()
            if money < 0:
                if money < -1.0:
                    log("You have overspent by more than £1! A 10% penalty will be applied to "
                        "the score.")
                    penalty = True
                state = environment.reset()
                mode = "testing"
                log("Training has finished, moving to testing.")
                test_init_time = time.time()
            elif action_type == "reset":
                if money >= K.COST_PER_RESET:
                    state = environment.reset()
                    resets_bought += 1
                else:
                    log("Insufficient money to buy a reset.")
            elif action_type == "demo":
                if money >= K.COST_PER_DEMO:
                    ds, da = environment.get_demonstration()
                    robot.process_demonstration(ds, da, money)
                    demos_bought += 1
                else:
                    log("Insufficient money to buy a demo.")
            elif action_type == "step":
                if money >= K.COST_PER_STEP:
                    action = robot.get_next_action_training(state, money)
                    next_state = environment.step(action)
                    robot.process_transition(state, action, next_state, money)
                    state = next_state
                    steps_bought += 1
            else:
                raise ValueError(f"Invalid value for action_type: {action_type}")
        else:
            action = robot.get_next_action_testing(state)
            next_state = environment.step(action)
            distance = np.linalg.norm(next_state - environment.goal_state)
            state = next_state
            test_time = time.time() - test_init_time
            if distance < test_best_distance:
                test_best_distance = distance
            if distance <= K.TEST_DISTANCE_THRESHOLD:
                log(f"The robot reached the goal! Time: {test_time}.")
                result["reached"] = True
                break
            if test_time >= test_timeout:
                log(f"The robot did not reach the goal in time. Best distance: "
                    f"{test_best_distance}.")
                break
        if tick_rate:
            time.sleep(max(0.0, 1.0 / tick_rate - (time.time() - t0)))
    result.update(ticks=ticks, mode=mode, demos=demos_bought, resets=resets_bought,
                  steps=steps_bought, penalty=penalty, best_distance=float(test_best_distance),
                  robot=robot, environment=environment)
    return result


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser(description="headless robot-learning.py on MI355X")
    ap.add_argument("--seed", type=int, default=K.RANDOM_SEED)
    ap.add_argument("--ticks", type=int, default=None)
    ap.add_argument("--episodes", type=int, default=None)
    ap.add_argument("--no-budget", action="store_true")
    a = ap.parse_args()
    r = run(seed=a.seed, max_ticks=a.ticks, budget=not a.no_budget, max_episodes=a.episodes)
    print({k: v for k, v in r.items() if k not in ("robot", "environment")})
