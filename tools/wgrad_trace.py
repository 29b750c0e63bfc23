"""Phase timing of the weight-gradient kernels at the bench shape (tuning probe, not a test).

Needs a library built with -DNAV_WGRAD_TRACE (tools/build_variant.sh wtrace learner
-DNAV_WGRAD_TRACE) bound through tools/withlib.py. Runs the bench trainer for a few steps, then
reads the s_memtime marks of 4 traced workgroups x 8 waves of k_wgrad_fact (critic twins) and
k_wgrad (actor) and prints each phase's mean duration in shader-clock cycles (s_memtime).

python tools/withlib.py abl/libnavenv_wtrace.so tools/wgrad_trace.py [--batch B]
"""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "residual-td3-robot-navigation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# (name, from mark, to mark) per kernel; k_wgrad has no table phase (no mark 1)
PHASES = {
    "k_wgrad_fact": [("table + barrier", 0, 1), ("constants", 1, 2), ("row maxima", 2, 3),
                     ("scales + row loop", 3, 4), ("tail tile + Wo epilogue", 4, 5),
                     ("LDS reduce + slab write", 5, 6)],
    "k_wgrad": [("constants", 0, 2), ("row maxima", 2, 3), ("scales + row loop", 3, 4),
                ("unscale", 4, 5), ("LDS reduce + slab write", 5, 6)],
}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--n-hidden", type=int, default=2)
    ap.add_argument("--n-envs", type=int, default=65536)
    args = ap.parse_args()
    from nav._lib import lib_path
    from nav.trainer import VecTrainer
    tr = VecTrainer(n_envs=args.n_envs, hidden=args.hidden, n_hidden=args.n_hidden, batch=args.batch, updates_per_step=2,
                    envs_per_group=1024)
    for _ in range(6):
        tr.step()
    torch.cuda.synchronize()
    raw = C.CDLL(lib_path())
    n = 2 * 4 * 8 * 8
    buf = (C.c_ulonglong * n)()
    assert raw.nav_wgrad_trace_read(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(2, 4, 8, 8).astype(np.int64)
    out = {"batch": args.batch, "unit": "shader-clock cycles (s_memtime)"}
    for kid, name in ((0, "k_wgrad_fact"), (1, "k_wgrad")):
        x = t[kid]
        res = {}
        for pname, a, b in PHASES[name] + [("total", 0, 6)]:
            ok = (x[:, :, a] > 0) & (x[:, :, b] > 0)
            res[pname] = round(float((x[:, :, b] - x[:, :, a])[ok].mean()), 1) if ok.any() else None
        # per traced block: each wave's marks relative to the block's earliest start
        res["waves"] = {}
        for b in range(4):
            if x[b, 0, 0] == 0:
                continue
            base = x[b, :, 0][x[b, :, 0] > 0].min()
            res["waves"][str(b)] = [[int(v - base) if v > 0 else None for v in x[b, w, :7]]
                                    for w in range(8)]
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
