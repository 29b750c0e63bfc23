"""Import shim: `from robot import Robot` (robot-learning.py:15) resolves to the MI355X drop-in
when this directory is first on sys.path. Also re-exports the reference's other robot.py names."""
from nav.robot import (TD3, ReplayBuffer, Residual_Actor_Network,  # noqa: F401
                       Residual_Critic_Network, Robot)
