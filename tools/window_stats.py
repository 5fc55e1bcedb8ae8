"""Traversal counters of one cfg2 render (stats kernels) with the library RT_HIP_LIB points at:
box / triangle / verification tests, fallbacks to the exact walk (RT_T2_WINDOW sweeps).

  RT_HIP_LIB=... python tools/window_stats.py [--config cfg2]
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
    fr = ShardedFrame(rk, 0, 1, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rk.set_stats(True)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    st = rk.stats()
    print(json.dumps({"lib": os.environ.get("RT_HIP_LIB", "default"), "config": args.config, "stats": st}))


if __name__ == "__main__":
    main()
