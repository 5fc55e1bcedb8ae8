"""Does the order of a k_trace launch's queries matter? The rays of one
dense iteration of a cfg2 frame (every walk of the stats render's first iterations, from the
walk log, rt_test_walk_log) are walked by the product's quad walk (rt_device_queries,
k_query_quad: 16 consecutive queries per wave, like k_trace's chunks) in several orders:
  pixel    the queue order of the product (kind by kind, path slot = pixel order in each)
  random   a random permutation (the lower bound on locality)
  octant   8 pixel-order groups x 8 direction octants (the binning item 5 proposes)
  morton   direction octant, then the Morton code of the origin on a 1024^3 grid
and the mean launch time is compared (the answers must agree bit for bit). Every order is
kind-major, like the product's queues (k_trace walks one kind's shards after another).

  python tools/order_probe.py [--iteration 2] [--config cfg2] [--out gpurun_out/order_probe.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def morton3(q: np.ndarray) -> np.ndarray:
    """30-bit Morton codes of [n, 3] integer cells in [0, 1024)."""
    def spread(v):
        v = v.astype(np.uint64) & 0x3FF
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        v = (v | (v << 2)) & 0x09249249
        return v
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def orders(log: np.ndarray, rng) -> dict:
    n = log.shape[0]
    o, d, slot = log["o"], log["d"], log["slot"].astype(np.int64)
    octant = ((d[:, 0] < 0).astype(np.int64) | ((d[:, 1] < 0).astype(np.int64) << 1) |
              ((d[:, 2] < 0).astype(np.int64) << 2))
    kind = log["kind"].astype(np.int64)
    out = {"pixel": np.lexsort((slot, kind)), "random": rng.permutation(n)}
    grp = (slot * 8) // (slot.max() + 1)
    out["octant"] = np.lexsort((slot, octant, grp, kind))
    lo, hi = o.min(0), o.max(0)
    cell = np.clip(((o - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.int64), 0, 1023)
    out["morton"] = np.lexsort((morton3(cell), octant, kind))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--iteration", type=int, default=2)
    ap.add_argument("--capacity", type=int, default=20 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "order_probe.json"))
    args = ap.parse_args()
    import torch

    import bench
    import rt_amd
    from rt_amd import _capi
    from rt_amd.dist import ShardedFrame

    scene, sky_kind, cam, W, H, spp, nb, desc = bench.CONFIGS[args.config]
    P, sky, cam17 = bench.build_inputs(args.config)
    rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=0)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    rk.set_lanes(1)  # (one lane: the iteration's queries are one launch's)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    fr = ShardedFrame(rk, 0, 1, device=dev)
    rk.set_stats(True)
    rk.test_walk_log(1, args.capacity)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    log, total = rk.walk_log()
    rk.set_stats(False)
    rk.test_walk_log(0, 0)
    sel = log[(log["iter"] == args.iteration) & (log["where"] == 0)]
    res = {"config": args.config, "iteration": args.iteration, "walks_logged": int(log.shape[0]),
           "walks_total": int(total), "orders": {}}
    rng = np.random.default_rng(7)
    L = _capi.lib()
    for role, kinds, mode in (("closest", (0, 1, 2, 3), 4), ("occlusion", (4, 5), 5)):
        part = sel[np.isin(sel["kind"], kinds)]
        n = part.shape[0]
        res["orders"][role] = {"queries": int(n)}
        ref = None
        for name, perm in orders(part, rng).items():
            rays = np.zeros((n, 8), np.float32)
            rays[:, 0:3] = part["o"][perm]
            rays[:, 4:7] = part["d"][perm]
            t = np.zeros(n, np.float32)
            k = np.zeros(n, np.int32)
            ms = ctypes.c_double()
            rc = L.rt_device_queries(rk.ctx, mode, _capi.ptr(rays), n, args.reps, _capi.ptr(t), _capi.ptr(k),
                                     ctypes.byref(ms))
            assert rc == 0, rc
            inv = np.empty(n, np.int64)
            inv[perm] = np.arange(n)
            tt = t[inv]
            if ref is None:
                ref = tt
            same = bool(np.array_equal(tt.view(np.uint32), ref.view(np.uint32)))
            res["orders"][role][name] = {"ms": round(ms.value, 4), "mrays_per_s": round(n / ms.value / 1e3, 1),
                                         "answers_equal": same}
            print(role, name, res["orders"][role][name], flush=True)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
