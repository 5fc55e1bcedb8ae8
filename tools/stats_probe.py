"""Counters of one render (rt_set_stats): how the k_trace quad slots split between the
streams and their drains, walk visits, fallbacks, path steps. One GPU.

  python tools/stats_probe.py [--config cfg2] [--world 1]   (world > 1: rank 0's rows of that split)
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
    args = ap.parse_args()
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
    dev = torch.device("cuda", 0)
    fr = ShardedFrame(rk, 0, args.world, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rk.set_stats(True)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    s = rk.stats()
    rk.set_stats(False)
    out = {"config": args.config, "world": args.world, "counters": s,
           "drain_slot_fraction": round(s["drain_slots"] / max(1, s["wave_slots"] + s["drain_slots"]), 4),
           "simt_stream": round((s["quad_visits"]) / max(1, s["wave_slots"]), 4),
           "simt_drain": round(s["drain_visits"] / max(1, s["drain_slots"]), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
