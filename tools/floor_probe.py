"""Per-iteration floor of the wavefront loop: a render of a few pixels with the tail kernel off,
so every iteration is a k_trace + k_step pair over a handful of paths (HIP events per launch).

  python tools/floor_probe.py [--px 1] [--spp 64]
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
    ap.add_argument("--px", type=int, default=1, help="pixels per side")
    ap.add_argument("--spp", type=int, default=64)
    args = ap.parse_args()
    import torch
    import bench
    import rt_amd
    from rt_amd.dist import ShardedFrame
    P, sky, cam17 = bench.build_inputs("cfg2")
    W = H = args.px
    rk = rt_amd.RenderKernel(W, H, args.spp, 8, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=0)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    rk.test_schedule(tail_paths=0, lanes=1, fast_k=0)  # (no tail kernel: every iteration a k_trace + k_step pair)
    dev = torch.device("cuda", 0)
    fr = ShardedFrame(rk, 0, 1, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    fr.render(stream)
    torch.cuda.synchronize(dev)
    plain = rk.device_last_kernel_ms()  # (no per-launch events)
    plain_iters = rk.last_iterations()
    rk.kernel_timing(1)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    kt = rk.kernel_timing(0)
    frame = rk.device_last_kernel_ms()
    out = {"pixels": W * H, "spp": args.spp, "frame_ms": round(frame, 3), "kernel_ms": {k: [round(v[0], 3), int(v[1])] for k, v in kt.items()}}
    n = max(1, kt["trace"][1])
    out["plain_frame_ms"] = round(plain, 3)
    out["plain_per_iteration_us"] = round(plain * 1e3 / max(1, plain_iters), 1)
    out["per_iteration_us"] = {"trace": round(kt["trace"][0] * 1e3 / n, 1), "step": round(kt["step"][0] * 1e3 / n, 1),
                               "frame": round(frame * 1e3 / n, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
