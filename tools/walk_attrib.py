"""Attribution of the long search-BVH walks: a stats render of one rank's
shard with the walk log on (rt_test_walk_log), every walk of at least --min-calls quad_visit
calls recorded (a row trip counts 2), then histograms by where it ran (k_trace quads, a drain's
rows, k_tail), ray kind, calls, iteration, and where the ray starts and ends on the dragon
stand-in (tools/scenes.py: a deformed UV sphere about (0, 1.6, 0), y scaled by 0.8, whose two
poles are fans of 1000 sliver triangles each, on a 40 x 40 ground quad at y = 0).

  python tools/walk_attrib.py [--config cfg4] [--world 8] [--rank 1] [--min-calls 24]
                              [--out gpurun_out/walk_attrib]

Writes OUT.json (histograms) and OUT_sample.npy (up to 200 K records, for offline study).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)

import numpy as np

KINDS = ["cont", "light_shadow", "brdf_light", "camera", "env_shadow", "brdf_env"]
WHERE = ["k_trace_quads", "k_trace_drain_rows", "k_tail"]
CENTER = np.array([0.0, 1.6, 0.0], np.float32)


def region(p: np.ndarray) -> dict:
    """Where points lie on the stand-in: ground, pole caps (theta of the undeformed
    parameterisation within 2 / 10 degrees of a pole), or the rest of the dragon, by theta band."""
    rel = (p - CENTER).astype(np.float64)
    rel[:, 1] /= 0.8
    r = np.linalg.norm(rel, axis=1)
    th = np.degrees(np.arccos(np.clip(rel[:, 1] / np.maximum(r, 1e-12), -1, 1)))
    ground = np.abs(p[:, 1]) < 1e-3
    out = {"ground": ground}
    d = ~ground
    out["pole_2deg"] = d & ((th < 2) | (th > 178))
    out["pole_10deg"] = d & ((th < 10) | (th > 170)) & ~out["pole_2deg"]
    for lo in range(10, 170, 20):
        out[f"theta_{lo}_{lo + 20}"] = d & (th >= lo) & (th < lo + 20) & ~out["pole_2deg"] & ~out["pole_10deg"]
    out["theta"] = th
    out["r"] = r
    return out


def hist(mask_dict: dict, n: int) -> dict:
    return {k: int(v.sum()) for k, v in mask_dict.items() if isinstance(v, np.ndarray) and v.dtype == bool and n}


def analyse(log: np.ndarray, total: int, min_calls: int) -> dict:
    n = log.shape[0]
    calls = log["calls"]
    res = {"walks_logged": int(n), "walks_qualified": int(total), "min_calls": min_calls}
    res["calls_quantiles"] = {q: int(np.quantile(calls, q)) for q in (0.5, 0.9, 0.99, 0.999, 1.0)} if n else {}
    edges = [min_calls, 32, 48, 64, 80, 96, 128, 192, 256, 1 << 30]
    res["calls_hist"] = {f"{a}-{b - 1}": int(((calls >= a) & (calls < b)).sum()) for a, b in zip(edges, edges[1:]) if b > a}
    res["by_where"] = {w: int((log["where"] == i).sum()) for i, w in enumerate(WHERE)}
    res["by_kind"] = {k: int((log["kind"] == i).sum()) for i, k in enumerate(KINDS)}
    o = log["o"]
    ro = region(o)
    res["origin_region"] = hist(ro, n)
    # camera rays start at the eye: their interesting end is the hit
    t = log["t"]
    closest = np.isin(log["kind"], [0, 1, 2, 3])
    hit = closest & (t > 0)
    p = o + np.maximum(t, 0)[:, None] * log["d"]
    rh = region(p[hit])
    res["closest_hit_region"] = hist(rh, int(hit.sum()))
    res["closest_outcome"] = {"hit": int(hit.sum()), "miss": int((closest & (t == -1)).sum()),
                              "exact_walk": int((closest & (t == -2)).sum())}
    occ = ~closest
    res["occlusion_outcome"] = {"occluded": int((occ & (t == 1)).sum()), "open": int((occ & (t == 0)).sum()),
                                "exact_walk": int((occ & (t == -2)).sum())}
    # grazing: the angle between the direction and the stand-in's radial direction at a dragon origin
    dr = ~ro["ground"] & (log["kind"] != 3)
    rel = (o[dr] - CENTER)
    rel[:, 1] /= 0.8
    rad = rel / np.maximum(np.linalg.norm(rel, axis=1, keepdims=True), 1e-12)
    cosr = np.abs((rad * log["d"][dr]).sum(1))
    res["dragon_origin_abs_cos_to_radial"] = {f"{a:.1f}-{b:.1f}": int(((cosr >= a) & (cosr < b)).sum())
                                              for a, b in zip(np.arange(0, 1.0, 0.1), np.arange(0.1, 1.01, 0.1))}
    # the same for the hardest walks alone
    top = calls >= np.quantile(calls, 0.99) if n else calls > 0
    res["top1pct"] = {"min_calls": int(calls[top].min()) if top.any() else 0,
                      "by_kind": {k: int((log["kind"][top] == i).sum()) for i, k in enumerate(KINDS)},
                      "origin_region": hist({k: v[top] for k, v in ro.items() if v.dtype == bool}, int(top.sum())),
                      "closest_hit_region": hist(region(p[top & hit]), int((top & hit).sum()))}
    # distinct paths (pixels) and how persistent long walks are along a path
    slots, counts = np.unique(log["slot"], return_counts=True)
    res["distinct_paths"] = int(slots.size)
    res["walks_per_path_quantiles"] = {q: int(np.quantile(counts, q)) for q in (0.5, 0.9, 0.99, 1.0)} if n else {}
    fbk = log["t"] == -2
    if fbk.any():  # walks left to the exact walk: their triangle field says why
        res["exact_walk_reasons"] = {name: {KINDS[k]: int((fbk & (log["tri"] == code) & (log["kind"] == k)).sum())
                                            for k in range(6) if (fbk & (log["tri"] == code) & (log["kind"] == k)).any()}
                                     for code, name in ((1, "tie"), (2, "chain_check"), (3, "stack_overflow"))}
    it = log["iter"]
    res["by_iteration_band"] = {f"{a}-{b - 1}": int(((it >= a) & (it < b)).sum())
                                for a, b in zip([0, 100, 200, 300, 400, 500, 600, 800], [100, 200, 300, 400, 500, 600, 800, 1 << 20])}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--min-calls", type=int, default=24)
    ap.add_argument("--capacity", type=int, default=4 << 20)
    ap.add_argument("--sample-every", type=int, default=1, help="keep every k-th walk by a hash (all walks: --min-calls 1); -1: only the walks left to the exact walk")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "walk_attrib"))
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
    fr = ShardedFrame(rk, args.rank, args.world, device=dev)
    rk.set_stats(True)
    rk.test_walk_log(args.min_calls, args.capacity, args.sample_every)
    fr.render(stream)
    torch.cuda.synchronize(dev)
    st = rk.stats()
    log, total = rk.walk_log()
    res = {"config": args.config, "world": args.world, "rank": args.rank, "iterations": rk.last_iterations(),
           "queries": int(st["rays"] + st["any_rays"]), "sample_every": args.sample_every, **analyse(log, total, args.min_calls)}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out + ".json", "w") as f:
        json.dump(res, f, indent=1)
    rng = np.random.default_rng(0)
    keep = log if log.shape[0] <= 200000 else log[np.sort(rng.choice(log.shape[0], 200000, replace=False))]
    np.save(args.out + "_sample.npy", keep)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
