"""Phase timing of k_td3_critic_rows at the bench shape (tuning probe, not a test).

Needs a library built with -DNAV_PHASE_TRACE (tools/build_variant.sh trace mlp8 -DNAV_PHASE_TRACE)
bound through tools/withlib.py. Runs the bench trainer for a few steps, then reads the s_memtime marks of
4 traced workgroups (blocks 0, 1, 200, 511) x 4 waves and prints each phase's duration in
cycles of that counter, per wave, plus the per-phase mean over the 16 traced waves.

python tools/withlib.py abl/libnavenv_trace.so tools/phase_trace.py [--batch B] [--hidden H
    --n-hidden L --n-envs N]  (config 1's learner: --batch 100 --hidden 200 --n-hidden 3, a
    trace7 build)
(--batch 16448: 257 workgroups of 64 rows, so the traced ones run alone on their CU)
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

# mark -> name (k_td3_critic_rows; fwd_net / bwd_net marks are base + 0..5)
FWD = ["start", "layer0", "barrier", "gemm", "out_partials", "barrier"]
BWD = ["start", "top_unit", "barrier+edges", "gemm", "mask+store", "edges0"]


def mark_names():
    n = {0: "kernel start", 1: "sample + barrier"}
    for base, tag in ((2, "actor_t"), (9, "critic_t1"), (15, "critic_t2"), (22, "critic1"),
                      (36, "critic2")):
        for i, s in enumerate(FWD):
            n[base + i] = f"{tag} fwd {s}"
    n[8] = "target noise + barrier"
    n[21] = "TD target + barrier"
    for q in range(2):
        n[28 + 14 * q] = f"critic{q + 1} loss epilogue"
        for i, s in enumerate(BWD):
            n[29 + 14 * q + i] = f"critic{q + 1} bwd {s}"
        n[35 + 14 * q] = f"critic{q + 1} done"
    return n


def tick_names():
    # the fused act + tick launch (k_mlp_fwd OUT_TICK): fwd_net's marks from NAV_TICK_MK = 52
    n = {52 + i: f"act fwd {s}" for i, s in enumerate(FWD)}
    n.update({58: "tick preamble", 59: "action epilogue + agent tick (wave 0)",
              62: "demo: cell starts + length scan", 63: "demo: candidate trips",
              60: "demo: final barrier + rewards", 61: "block stats"})
    return n


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--tick", action="store_true", help="the fused act + tick launch's marks")
    ap.add_argument("--wide", action="store_true",
                    help="a -DNAV_TRACE_WIDE build: 64 blocks (0, 8, 16, ...), per block its start "
                         "and end relative to the earliest traced start, plus the phase means")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--n-hidden", type=int, default=2)
    ap.add_argument("--n-envs", type=int, default=65536)
    args = ap.parse_args()
    from nav._lib import lib_path
    from nav.trainer import VecTrainer
    tr = VecTrainer(n_envs=args.n_envs, hidden=args.hidden, n_hidden=args.n_hidden,
                    batch=args.batch, updates_per_step=2, envs_per_group=1024)
    for _ in range(4):
        tr.step()
    torch.cuda.synchronize()
    raw = C.CDLL(lib_path())
    nt = 64 if args.wide else 4
    buf = (C.c_ulonglong * (nt * 4 * 64))()
    rc = raw.nav_phase_trace_read(buf, nt * 4 * 64)
    assert rc == 0, rc
    t = np.frombuffer(buf, dtype=np.uint64).reshape(nt, 4, 64).astype(np.int64)
    names = tick_names() if args.tick else mark_names()
    # in time order (the demo pass's sub-phase marks 62, 63 come between 59 and 60)
    marks = sorted(names, key=lambda m: {62: 59.3, 63: 59.6}.get(m, m))
    live = [wg for wg in range(nt) if t[wg, 0, marks[0]] != 0]  # blocks past the grid: absent
    t = t[live]
    out = {"marks": {}, "total": {}}
    if args.wide:
        t0 = t[:, :, marks[0]].min()
        out["blocks"] = {str(8 * wg): {"start": int(t[i, :, marks[0]].min() - t0),
                                       "end": int(t[i, :, marks[-1]].max() - t0)}
                         for i, wg in enumerate(live)}
    for wg in range(t.shape[0]):
        for w in range(4):
            out["total"][f"wg{wg}w{w}"] = int(t[wg, w, marks[-1]] - t[wg, w, marks[0]])
    for a, b in zip(marks[:-1], marks[1:]):
        d = t[:, :, b] - t[:, :, a]
        out["marks"][f"{b:02d} {names[b]}"] = {"mean": float(d.mean()), "min": int(d.min()),
                                               "max": int(d.max())}
    if not args.tick and (t[:, :, 50] != 0).any():
        # a >= 3-layer forward's inner marks (the last forward of the block; twin 0 of block 0:
        # critic1, marks 24 .. 25): layer-1 product + bias, store_layer + barriers, top product
        w0 = t[0]
        out["inner_fwd"] = {"gemm1": (w0[:, 50] - w0[:, 24]).tolist(),
                            "store": (w0[:, 51] - w0[:, 50]).tolist(),
                            "gemm2": (w0[:, 25] - w0[:, 51]).tolist()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
