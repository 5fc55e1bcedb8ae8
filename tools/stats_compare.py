"""Work counters of one cfg2 render (rt_set_stats) for the loaded library build
(RT_HIP_LIB selects another): box / triangle tests and fallbacks, one JSON line.

  RT_HIP_LIB=... python tools/stats_compare.py [--config cfg2]
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
    import bench
    import rt_amd
    _, _, _, W, H, spp, nb, _ = bench.CONFIGS[args.config]
    P, sky, cam17 = bench.build_inputs(args.config)
    fb = rt_amd.Image(W, H)
    rk = rt_amd.RenderKernel(W, H, spp, nb, fb, P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky), None)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    rk.set_stats(True)
    rk.render()
    st = rk.stats()
    print(json.dumps({"lib": os.environ.get("RT_HIP_LIB", "default"), **{k: int(v) for k, v in st.items()}}))


if __name__ == "__main__":
    main()
