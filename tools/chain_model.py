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
    ap.add_argument("--out", default="")
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
    for t_spec in (0, 260, 300):
        for k in (2, 4, 8):
            pols.append((f"window K={k} from it {t_spec}, b=1", 1, k, t_spec, 1, 0))
            pols.append((f"window K={k} from it {t_spec}, last b", 1, k, t_spec, 1, 1))
    for name, klo, khi, ts, pr, pm in pols:
        hist, fin, work = run(L, b, klo, khi, ts, pr, pm)
        ms = frame_ms(hist, scale, unit_ns, args.floor_us, args.tail_n, args.tail_us)
        r = {"policy": name, "iters": len(hist), "work_x": round(work / chain.sum(), 3), "ms": round(ms, 1),
             "eff": round(t_ideal / ms, 3)}
        out.append(r)
        print(json.dumps(r), flush=True)
    L.lattice_sim.restype = ctypes.c_long
    L.lattice_sim.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                                       ctypes.c_void_p]
    for t0 in (266, 500, 873):
        for R in (4, 8, 16, 32):
            hist = np.zeros(20000, np.int32)
            fin = np.zeros(b.shape[0], np.int32)
            work = np.zeros(1, np.int64)
            tm = L.lattice_sim(b.ctypes.data, b.shape[0], b.shape[1], R, t0, 8, hist.ctypes.data, 20000,
                               fin.ctypes.data, work.ctypes.data)
            hist = hist[:tm + 1]
            ms = frame_ms(hist, scale, unit_ns, args.floor_us, args.tail_n, args.tail_us)
            r = {"policy": f"lattice R={R} from it {t0}", "iters": int(tm), "work_x": round(int(work[0]) / chain.sum(), 3),
                 "ms": round(ms, 1), "eff": round(t_ideal / ms, 3)}
            out.append(r)
            print(json.dumps(r), flush=True)
    if args.out:
        summary = {"what": "per-pixel sample-chain model of an N-way row shard (tools/chain_model.py on tools/chain_log.py's "
                           "per-sample draw counts from the CPU restatement; analysis only)",
                   "log": {"config": str(z.get("config", "cfg4")), "world": world, "rank": int(z["rank"]), "every": every,
                           "pixels": int(b.shape[0])},
                   "chains": {"mean": float(chain.mean()), "p99": float(np.percentile(chain, 99)), "max": int(chain.max()),
                              "b_hist": np.bincount(b.ravel()).tolist()},
                   "time_model": {"unit_ns_per_path_step": round(unit_ns, 4), "floor_us": args.floor_us,
                                  "tail_below_paths": args.tail_n, "tail_round_us": args.tail_us, "t1_ms": args.t1_ms},
                   "policies": out}
        with open(args.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
