"""Per-rank render time of a row shard, on one GPU (multi-GPU scaling probe).

Renders the shares (rows y % N == r) of a config for N in --worlds — every rank's
with --all-ranks, else rank 0's — and prints the time per render, the per-GPU rate
and the strong-scaling efficiency it implies, T_1 / (N * max_r T_N,r) (the slowest
rank sets the frame); the RCCL gather is not included (it is ~0.1 ms at 1080p,
DESIGN.md §6).

  python tools/shard_probe.py [--config cfg2] [--worlds 1,2,4,8] [--reps 2] [--all-ranks]
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
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--all-ranks", action="store_true")
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
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = {"config": args.config, "desc": desc, "runs": []}
    t1 = None
    for n in [int(x) for x in args.worlds.split(",")]:
        per_rank = []
        for rank in (range(n) if args.all_ranks else [0]):
            fr = ShardedFrame(rk, rank, n, device=dev)
            fr.render(stream)
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                fr.render(stream)
                torch.cuda.synchronize(dev)
                ts.append(time.perf_counter() - t0)
            per_rank.append((min(ts), fr.rows, rk.last_iterations()))
        t = max(p[0] for p in per_rank)
        t1 = t if n == 1 else t1
        rows = per_rank[0][1]
        samples = rows * W * spp
        r = {"world": n, "rows": rows, "ms": round(t * 1e3, 2), "iters": max(p[2] for p in per_rank),
             "msamples_per_s_per_gpu": round(samples / t / 1e6, 1)}
        if len(per_rank) > 1:
            r["ms_per_rank"] = [round(p[0] * 1e3, 2) for p in per_rank]
            r["slowest_rank"] = int(max(range(len(per_rank)), key=lambda i: per_rank[i][0]))
        if t1 is not None:
            r["strong_eff_vs_1"] = round(t1 / (n * t), 3)
        out["runs"].append(r)
        print(json.dumps(r), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
