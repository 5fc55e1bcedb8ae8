"""Per-iteration profile of one render (RT_ITER_LOG), one lane: where the frame
time goes as the live-path count falls. Renders rank 0's rows of an N-way
strong-scaling split (--world N; 1 = the whole frame) twice: a stats render
(per-iteration query / live counts) and a timed render (HIP events around each
launch), then prints time per live-count band and the tail kernel's share.

  python tools/iter_profile.py [--config cfg2] [--world 1] [--out gpurun_out/iter]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--lanes", type=int, default=1)
    ap.add_argument("--fast-k", type=int, default=0, help="fast lane paths (0 off: r04-comparable bands; -1 product)")
    ap.add_argument("--out", default="gpurun_out/iter")
    ap.add_argument("--raw", action="store_true", help="add the per-iteration arrays")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    prefix = f"{args.out}_{args.config}_w{args.world}"
    os.environ["RT_ITER_LOG"] = prefix
    import numpy as np
    import torch
    import bench
    import rt_amd
    from rt_amd.dist import ShardedFrame
    scene, sky_kind, cam, W, H, spp, nb, desc = bench.CONFIGS[args.config]
    P, sky, cam17 = bench.build_inputs(args.config)
    rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=0)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    rk.set_lanes(args.lanes)
    rk.test_schedule(fast_k=args.fast_k)
    dev = torch.device("cuda", 0)
    fr = ShardedFrame(rk, 0, args.world, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rk.set_stats(True)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    rk.set_stats(False)
    fr.render(stream)  # warm
    torch.cuda.synchronize(dev)
    rk.kernel_timing(1)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    kt = rk.kernel_timing(0)
    frame_ms = rk.device_last_kernel_ms()
    cnt = np.loadtxt(prefix + ".counts", ndmin=2)
    ms = np.loadtxt(prefix + ".ms", ndmin=2)
    # counts: i, queries, live (k_step n) | tail: rounds; ms: i, trace_ms, step_ms
    n_it = ms.shape[0]
    live = cnt[:n_it, 2]
    bands = [(1 << 30, 1 << 20), (1 << 20, 1 << 18), (1 << 18, 1 << 16), (1 << 16, 1 << 14), (1 << 14, 0)]
    out = {"config": args.config, "world": args.world, "lanes": args.lanes, "frame_ms": round(frame_ms, 2),
           "iterations": int(n_it), "kernel_ms": {k: round(v[0], 2) for k, v in kt.items()}, "bands": []}
    for hi, lo in bands:
        sel = (live <= hi) & (live > lo)
        out["bands"].append({"live": f"({lo}, {hi}]", "iters": int(sel.sum()),
                             "trace_ms": round(float(ms[sel, 1].sum()), 2), "step_ms": round(float(ms[sel, 2].sum()), 2),
                             "queries": int(cnt[:n_it][sel, 1].sum()),
                             # the longest walk of each launch (quad_visit calls, closest / occlusion), band mean
                             "max_visits_c": round(float(cnt[:n_it][sel, 3].mean()), 1) if sel.any() else 0.0,
                             "max_visits_a": round(float(cnt[:n_it][sel, 4].mean()), 1) if sel.any() else 0.0,
                             "walks_over_8_calls": int(cnt[:n_it][sel, 5].sum()),
                             "us_per_trace": round(float(ms[sel, 1].sum()) * 1e3 / max(1, int(sel.sum())), 1)})
    # the tail launch: rounds of its longest pool loop, 100 MHz ticks / 16 in steps and in walks (summed over waves)
    ti = int(cnt.shape[0]) - 1
    out["tail_row"] = [int(v) for v in cnt[ti]] if cnt.shape[0] > n_it else None
    if args.raw:  # per-iteration arrays: live slots, queries, fallbacks (stats render), trace / step ms (timed)
        out["raw"] = {"live": [int(v) for v in live], "queries": [int(v) for v in cnt[:n_it, 1]],
                      "fallbacks": [int(v) for v in cnt[:n_it, 6]] if cnt.shape[1] > 6 else None,
                      "trace_ms": [round(float(v), 4) for v in ms[:, 1]], "step_ms": [round(float(v), 4) for v in ms[:, 2]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
