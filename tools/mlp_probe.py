"""Layer-scaling probe of the fused MLP forward (diagnostic): twin-critic forward time at growing
depth, so the marginal cost of one more hidden x hidden layer (GEMM + epilogue) separates from
the fixed per-network cost (layer 0, output layer, launch).

python tools/mlp_probe.py [--batch 32768] [--hidden 256]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "residual-td3-robot-navigation_amd"))

import torch  # noqa: E402

from tools.microbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--hidden", type=int, default=256)
    args = ap.parse_args()
    from nav.mlp import DeviceMLP, forward
    B, H = args.batch, args.hidden
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, 4, device="cuda") * 10
    res = {}
    for L in (1, 2, 3, 5):
        crit = [DeviceMLP(4, 1, H, L, "cuda").init_kaiming(g) for _ in range(2)]
        q = [torch.zeros(B, 1, device="cuda") for _ in range(2)]
        us = timeit(lambda: forward(crit, x, 4, 0, q, 1, 0, B), reps=30)
        res["twin_fwd_L%d" % L] = round(us, 2)
    per_layer = (res["twin_fwd_L5"] - res["twin_fwd_L2"]) / 3
    ideal = 2 * 2.0 * B * H * H / 155e12 * 1e6
    res["marginal_layer_us"] = round(per_layer, 2)
    res["marginal_layer_TFs"] = round(2 * 2.0 * B * H * H / per_layer / 1e6, 1)
    res["ideal_layer_us_155TF"] = round(ideal, 2)
    res["fixed_us"] = round(res["twin_fwd_L2"] - per_layer, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
