"""Launch timeline of one render with every lane on one clock (RT_TIMELINE, run_wave).

Renders a config's frame (or one rank's row shard) with the default lanes and HIP events
around every launch, then reports what the GPU ran over time: per lane its first and
last launch, the k_trace / k_step / tail-kernel time, and the frame split into the
intervals where 3, 2, 1 or 0 lanes had work queued, and the time in each lane's tail
kernel. Events on the lanes' streams add a little time to the render (not a bench
figure).

  python tools/timeline.py [--config cfg2] [--world 1 --rank 0] [--out gpurun_out/tl_cfg2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)


def summarize(rows: np.ndarray) -> dict:
    """rows: lane, iter, trace start, trace end, step end, flag (1 tail kernel, 2 the fast lane's kernel) (ms)."""
    fast = rows[rows[:, 5] == 2]  # (the fast lane's kernel: start, end)
    rows = rows[rows[:, 5] != 2]
    lanes = sorted(set(int(x) for x in rows[:, 0]))
    out = {"lanes": []}
    if len(fast):
        out["fast_lane"] = {"start_ms": round(float(fast[0, 2]), 2), "end_ms": round(float(fast[0, 3]), 2),
                            "ms": round(float(fast[0, 3] - fast[0, 2]), 2)}
    ev = []  # (time, +1 / -1) per lane busy interval (first launch .. last)
    for l in lanes:
        r = rows[rows[:, 0] == l]
        tail = r[r[:, 5] == 1]
        tr = float(np.sum(r[:, 3] - r[:, 2]))
        st = float(np.sum((r[:, 4] - r[:, 3])[r[:, 5] == 0]))
        tk = float(np.sum(tail[:, 4] - tail[:, 3])) if len(tail) else 0.0
        d = {"lane": l, "iters": int(len(r)), "first_ms": round(float(r[:, 2].min()), 3),
             "last_ms": round(float(r[:, 4].max()), 3), "trace_ms": round(tr, 2), "step_ms": round(st, 2),
             "tail_ms": round(tk, 2), "tail_start_ms": round(float(tail[0, 3]), 2) if len(tail) else None}
        out["lanes"].append(d)
        for a, b in zip(r[:, 2], r[:, 4]):
            ev.append((a, 1))
            ev.append((b, -1))
    ev.sort()
    busy = {}
    cur, last = 0, ev[0][0]
    for t, dlt in ev:
        busy[cur] = busy.get(cur, 0.0) + (t - last)
        cur += dlt
        last = t
    out["frame_ms"] = round(float(max(rows[:, 4].max(), fast[:, 3].max() if len(fast) else 0.0) - rows[:, 2].min()), 3)
    out["ms_with_n_lanes_busy"] = {str(k): round(v, 2) for k, v in sorted(busy.items())}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "timeline"))
    args = ap.parse_args()
    import torch

    import bench
    import rt_amd
    from rt_amd.dist import ShardedFrame

    scene, sky_kind, cam, W, H, spp, nb, desc = bench.CONFIGS[args.config]
    P, sky, cam17 = bench.build_inputs(args.config)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    os.environ["RT_TIMELINE"] = args.out + ".txt"  # (read when the context is created; written by timed renders)
    rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=0)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    fr = ShardedFrame(rk, args.rank, args.world, device=dev)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fr.render(stream)
    torch.cuda.synchronize(dev)
    plain_ms = (time.perf_counter() - t0) * 1e3
    rk.kernel_timing(1)
    t0 = time.perf_counter()
    fr.render(stream)
    torch.cuda.synchronize(dev)
    timed_ms = (time.perf_counter() - t0) * 1e3
    rk.kernel_timing(0)
    rows = np.loadtxt(args.out + ".txt", ndmin=2)
    s = summarize(rows)
    s.update({"config": args.config, "world": args.world, "rank": args.rank, "render_ms": round(plain_ms, 2),
              "render_ms_with_events": round(timed_ms, 2)})
    with open(args.out + ".json", "w") as f:
        json.dump(s, f, indent=1)
    print(json.dumps(s))


if __name__ == "__main__":
    main()
