"""Frame-time model of a shard's sample chains with speculative sample starts (analysis only).

Reads a draw log (tools/chain_log.py), turns draws into shaded bounces (b = (draws - 2) / D),
runs tools/chain_sim.c for each policy and converts the runners-per-iteration curve into
time with a launch model of the wavefront loop: an iteration costs
max(floor, n * unit) while the live count n (scaled by the log's pixel stride) is above the
tail threshold, and `tail_round` per round below it. unit is set so the policy-free run of
the whole 1-GPU frame matches its measured time; floor / tail_round are the measured per
iteration floors.

  python tools/chain_model.py --log /tmp/chain_cfg4.npz
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = "/tmp/libchain_sim.so"


def sim_lib():
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", os.path.join(HERE, "chain_sim.c"), "-o", SO], check=True)
    L = ctypes.CDLL(SO)
    L.chain_sim.restype = ctypes.c_long
    L.chain_sim.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                                     ctypes.c_void_p]
    return L


def run(L, b, k_lo, k_hi, t_spec, pred=1, pred_mode=0, hist_len=20000):
    n, spp = b.shape
    hist = np.zeros(hist_len, np.int32)
    fin = np.zeros(n, np.int32)
    work = np.zeros(1, np.int64)
    tmax = L.chain_sim(b.ctypes.data, n, spp, k_lo, k_hi, t_spec, pred, pred_mode, hist.ctypes.data, hist_len,
                       fin.ctypes.data, work.ctypes.data)
    return hist[:tmax + 1], fin, int(work[0])


def frame_ms(hist, scale, unit_ns, floor_us, tail_n, tail_us):
    n = hist.astype(np.float64) * scale
    t = np.where(n > tail_n, np.maximum(floor_us * 1e-3, n * unit_ns * 1e-6), np.where(n > 0, tail_us * 1e-3, 0))
    return float(t.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", default="/tmp/chain_cfg4.npz")
    ap.add_argument("--D", type=int, default=7, help="RNG draws per shaded bounce (dragon: 7)")
    ap.add_argument("--t1-ms", type=float, default=1862.0, help="measured 1-GPU frame (cfg4)")
    ap.add_argument("--floor-us", type=float, default=150.0)
    ap.add_argument("--tail-n", type=float, default=8192)
    ap.add_argument("--tail-us", type=float, default=74.0)
    args = ap.parse_args()
    z = np.load(args.log)
    d = z["draws"].astype(np.int32)
    b = np.ascontiguousarray(((d - 2) // args.D).astype(np.uint16))
    world, every = int(z["world"]), int(z["every"])
    W, H, spp = int(z["W"]), int(z["H"]), int(z["spp"])
    scale = every
    L = sim_lib()
    chain = b.astype(np.int64).sum(1)
    print(json.dumps({"pixels": int(b.shape[0]), "chain_mean": float(chain.mean()), "chain_max": int(chain.max()),
                      "chain_p99": float(np.percentile(chain, 99)), "b_hist": np.bincount(b.ravel()).tolist()}))
    # unit: the 1-GPU frame's path steps (all pixels, mean chain) in t1
    steps_1gpu = W * H * chain.mean()
    unit_ns = args.t1_ms * 1e6 / steps_1gpu
    t_ideal = args.t1_ms / world
    out = []
    pols = [("base K=1", 1, 1, 0, 1, 0)]
    for t_spec in (0, 150, 220, 260, 300):
        for k in (2, 4, 8, 16):
            pols.append((f"K={k} from it {t_spec}", 1, k, t_spec, 1, 0))
            pols.append((f"K={k} from it {t_spec} last-b", 1, k, t_spec, 1, 1))
    for name, klo, khi, ts, pr, pm in pols:
        hist, fin, work = run(L, b, klo, khi, ts, pr, pm)
        ms = frame_ms(hist, scale, unit_ns, args.floor_us, args.tail_n, args.tail_us)
        r = {"policy": name, "iters": len(hist), "work_x": round(work / chain.sum(), 3), "ms": round(ms, 1),
             "eff": round(t_ideal / ms, 3)}
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
