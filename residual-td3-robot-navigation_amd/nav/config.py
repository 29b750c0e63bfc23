"""Constants and hyper-parameters of the reference, in one place.

constants.py:6-53 (world, action bound, CEM sizes, costs, test threshold), configuration.py:26 (seed)
and robot.py:21-54 (demo augmentation, path length, exploration, replay, reward shaping, TD3).
"""
from dataclasses import dataclass, field

# constants.py
WORLD_SIZE = 100
ROBOT_MAX_ACTION = 5
INIT_REGION_SIZE = 25
UPDATE_RATE = 10
DEMOS_CEM_NUM_ITERATIONS = 4
DEMOS_CEM_NUM_PATHS = 100
DEMOS_CEM_PATH_LENGTH = 200
DEMOS_CEM_NUM_ELITES = 10
STARTING_MONEY = 100
COST_PER_STEP = 0.01
COST_PER_CPU_SECOND = 0.03
COST_PER_DEMO = 20
COST_PER_RESET = 5
TEST_DISTANCE_THRESHOLD = 5
TEST_TIMEOUT = 100

# configuration.py
RANDOM_SEED = 1707366464

# robot.py:21-54
NUM_DEMO = 3
NUM_AUGMENTS = 3
AUG_NOISE = 2.5
AUG_INTERPOLATION = 5
PATH_LENGTH = 50
PATH_INCREASE = 20
INITIAL_NOISE = 1
NOISE_DECAY = 0.75
BUFFER_SIZE = 10000
STUCK_THRESHOLD = 2
STUCK_STEPS = 5
STUCK_PENALTY = 50
GOAL_REWARD = 50
DEMO_PROXIMITY_FACTOR = 10
ACTOR_LR = 0.00001
CRITIC_LR = 0.00001
POLICY_UPDATE_DELAY = 2
TARGET_POLICY_NOISE = 0.2
NOISE_CLIP = 0.5
TD3_EPOCHS = 100
TD3_BATCH_SIZE = 100
GAMMA = 0.99
TAU = 0.001


@dataclass
class NetConfig:
    """Actor / critic width: 3 x 200 is the reference (robot.py:145-148, 185-188); 2 x 256 is the
    BASELINE config-3 throughput shape."""
    hidden: int = 200
    n_hidden: int = 3

    @property
    def hidden_pad(self):
        return (self.hidden + 31) // 32 * 32


@dataclass
class TD3Config:
    actor_lr: float = ACTOR_LR
    critic_lr: float = CRITIC_LR
    gamma: float = GAMMA
    tau: float = TAU
    policy_noise: float = TARGET_POLICY_NOISE
    noise_clip: float = NOISE_CLIP
    policy_update_delay: int = POLICY_UPDATE_DELAY
    max_action: float = ROBOT_MAX_ACTION
    batch_size: int = TD3_BATCH_SIZE
    num_epochs: int = TD3_EPOCHS
    net: NetConfig = field(default_factory=NetConfig)
