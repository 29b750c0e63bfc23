import cProfile, pstats, sys, os, time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/residual-td3-robot-navigation_amd")
import numpy as np, torch
from nav import robot
rb = robot.Robot(np.array([60.0, 40.0]))
rng = np.random.default_rng(0)
for s in rng.uniform(0, 100, (400, 2)):
    rb.memory.push(s, rng.uniform(-5, 5, 2), rng.uniform(-100, 0), s + 1, False)
for _ in range(3): rb.td3_agent.td3_update(rb.memory)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5): rb.td3_agent.td3_update(rb.memory)
torch.cuda.synchronize()
print("ms per update", (time.perf_counter() - t0) / 5 * 1e3)
pr = cProfile.Profile(); pr.enable()
for _ in range(5): rb.td3_agent.td3_update(rb.memory)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
