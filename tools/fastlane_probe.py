"""Per-iteration latency of a small render while a full frame renders beside it.

Question behind it: could a few thousand long-chain paths, stepped in a
wavefront of their own beside the frame's lanes, advance much faster than one step per
dense iteration (~1.2 ms)? Context B renders a thin row shard of cfg2 (rows y % world
== 0, one lane, HIP events around its launches) alone, then again while context A
renders the full cfg2 frame in a loop on another host thread (ctypes drops the GIL),
and the probe prints B's iterations, frame time and ms per iteration both ways.

  python tools/fastlane_probe.py [--world 100] [--out gpurun_out/fastlane.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=100)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "fastlane.json"))
    args = ap.parse_args()
    import torch

    import bench
    import rt_amd
    from rt_amd.dist import ShardedFrame

    scene, sky_kind, cam, W, H, spp, nb, desc = bench.CONFIGS["cfg2"]
    P, sky, cam17 = bench.build_inputs("cfg2")

    def kernel():
        rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                                 P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                                 rt_amd.Image.from_rgb(sky), None, device=0)
        rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
        return rk

    dev = torch.device("cuda", 0)
    ka, kb = kernel(), kernel()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    fa = ShardedFrame(ka, 0, 1, device=dev)
    fb = ShardedFrame(kb, 0, args.world, device=dev)
    kb.set_lanes(1)
    for f, s in ((fa, sa), (fb, sb)):  # warm
        f.render(s.cuda_stream)
    torch.cuda.synchronize(dev)

    def timed_b():
        kb.kernel_timing(1)
        t0 = time.perf_counter()
        fb.render(sb.cuda_stream)
        sb.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        kt = kb.kernel_timing(0)
        return ms, kb.last_iterations(), kt

    alone = timed_b()
    stop = threading.Event()
    a_frames = []

    def loop_a():
        while not stop.is_set():
            t0 = time.perf_counter()
            fa.render(sa.cuda_stream)
            sa.synchronize()
            a_frames.append((time.perf_counter() - t0) * 1e3)

    th = threading.Thread(target=loop_a)
    th.start()
    time.sleep(0.05)  # (A's dense phase under way)
    loaded = timed_b()
    stop.set()
    th.join()
    out = {"config": "cfg2", "b_rows": fb.rows, "b_pixels": fb.rows * W, "world": args.world,
           "b_alone": {"ms": round(alone[0], 2), "iters": alone[1], "ms_per_iter": round(alone[0] / max(alone[1], 1), 4),
                       "kernel_ms": alone[2]},
           "b_beside_full_frame": {"ms": round(loaded[0], 2), "iters": loaded[1],
                                   "ms_per_iter": round(loaded[0] / max(loaded[1], 1), 4), "kernel_ms": loaded[2]},
           "a_frame_ms": [round(x, 2) for x in a_frames]}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
