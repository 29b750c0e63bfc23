"""Held shader clock of the MFMA kernels at the bench shape (tuning probe, not a test).

Needs a library built with -DNAV_CLOCK_STAMP (tools/build_variant.sh clock mlp8 -DNAV_CLOCK_STAMP),
bound through tools/withlib.py. Runs the bench trainer (BASELINE config 3: 65 536 envs, 2x256,
batch 32 768, UTD 1) back to back for --seconds (>= 2 s: MI355X_MICROARCH.md 'DVFS give-back' 6),
then reads the s_memtime / s_memrealtime stamps thread 0 of every workgroup wrote at the start and
the end of the last launch of k_td3_critic_rows, k_td3_actor_rows and the tick launch, and prints
per kernel the median (p10, p90) over workgroups of
    clock = d(s_memtime) / d(s_memrealtime) x 100 MHz
and the workgroup lifetime in shader cycles.

python tools/withlib.py abl/libnavenv_clock.so tools/clock_probe.py [--seconds 3]
"""
import ctypes as C
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "residual-td3-robot-navigation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

KERNELS = ["k_td3_critic_rows", "k_td3_actor_rows", "k_mlp_fwd<tick>"]
BLOCKS = 1024


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--batch", type=int, default=32768)
    args = ap.parse_args()
    from nav._lib import lib_path
    from nav.trainer import VecTrainer
    tr = VecTrainer(n_envs=65536, hidden=256, n_hidden=2, batch=args.batch, updates_per_step=2,
                    envs_per_group=1024)
    for _ in range(4):
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < args.seconds:
        for _ in range(50):
            tr.step()
        torch.cuda.synchronize()
        steps += 50
    wall = time.perf_counter() - t0
    raw = C.CDLL(lib_path())
    n = 3 * BLOCKS * 4
    buf = (C.c_ulonglong * n)()
    rc = raw.nav_clock_stamp_read(buf, n)
    assert rc == 0, rc
    t = np.frombuffer(buf, dtype=np.uint64).reshape(3, BLOCKS, 4).astype(np.float64)
    out = {"steps": steps, "seconds": round(wall, 3), "ms_per_step": round(1e3 * wall / steps, 4),
           "kernels": {}}
    for k, name in enumerate(KERNELS):
        dt = t[k, :, 2] - t[k, :, 0]
        dr = t[k, :, 3] - t[k, :, 1]
        ok = (dr > 0) & (t[k, :, 0] > 0)
        if not ok.any():
            continue
        mhz = dt[ok] / dr[ok] * 100.0
        # the whole launch: earliest start to latest end on the 100 MHz clock
        span_us = (t[k, ok, 3].max() - t[k, ok, 1].min()) / 100.0
        out["kernels"][name] = {
            "workgroups": int(ok.sum()),
            "clock_mhz_median": round(float(np.median(mhz)), 1),
            "clock_mhz_p10": round(float(np.percentile(mhz, 10)), 1),
            "clock_mhz_p90": round(float(np.percentile(mhz, 90)), 1),
            "wg_cycles_median": round(float(np.median(dt[ok])), 0),
            "wg_us_median": round(float(np.median(dr[ok])) / 100.0, 2),
            "launch_span_us": round(float(span_us), 2),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
