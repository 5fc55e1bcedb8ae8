"""Per-variant frame time of the cfg5 sweep on one GPU (BASELINE config 5: 16 material
variants, 1920x1080x1024spp x8), through rt_render_variants one variant at a time, and
the static 8-GPU assignment it implies for bench.py's variant order (CFG5_ORDER).

  python tools/sweep_probe.py [--out profiles/r03_sweep_variant_ms.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/sweep_variant_ms.json")
    args = ap.parse_args()
    import torch

    import bench
    import rt_amd
    _, _, _, W, H, spp, nb, desc = bench.CONFIGS["cfg5sweep"]
    P, sky, cam17 = bench.build_inputs("cfg5sweep")
    tables = bench.cfg5_tables(P)
    rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=0)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    buf = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0")
    rk.render_variants([tables[0]], device_ptrs=[buf.data_ptr()])  # warm
    ms = []
    for v, t in enumerate(tables):
        t0 = time.perf_counter()
        rk.render_variants([t], device_ptrs=[buf.data_ptr()])
        ms.append(round((time.perf_counter() - t0) * 1e3, 1))
        print(json.dumps({"variant": v, "grid": bench.CFG5_GRID[v], "ms": ms[-1]}), flush=True)
    out = {"what": "cfg5 sweep: one variant per rt_render_variants call on one MI355X (3 lanes)", "desc": desc,
           "ms": ms, "grid": bench.CFG5_GRID, "total_ms": round(sum(ms), 1)}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
