"""Far-origin probe of the search-BVH front end.

Rays are aimed at uniform random points of uniformly chosen triangles of a scene from
distance D along random directions (``--mode random``), or along directions within a
few degrees of the triangle's plane (``--mode grazing``). The fast query the render's
k_trace stage runs (rt_fast.h fast_query_closest, compiled for the host:
rt_hostsim_fast_queries) is compared with the exact octree walk (rt_intersect,
rt_traverse.h, the reference's bvh.h:127-209 walk): a ray the fast query settles with
another (t, triangle) than the exact walk is a wrong answer; a ray it hands to the exact
walk (-2) is not.

    python tools/far_probe.py --scene dragon --d 10 100 1000 10000 --n 200000 [--near-scale -1]

--near-scale: rt_test_schedule("near_scale", x) (x < 0: the product's default; a huge
value turns the far-origin routing off, to measure the unguarded walk). Prints one JSON
line per (scene, mode, D).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sycl-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import rt_amd  # noqa: E402
from rt_amd import _capi  # noqa: E402
import scenes  # noqa: E402


def kernel(scene: str, hostsim: bool = True):
    P = rt_amd.parse_obj(scenes.scene_path(scene))
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(np.ones((8, 16, 3), np.float32)), None, hostsim=hostsim)
    return P, rk


def far_rays(tris: np.ndarray, D: float, n: int, mode: str, rng: np.random.Generator) -> np.ndarray:
    """rays[n][6]: origin P + D u, direction -u, P a uniform point of a uniformly
    chosen triangle; u uniform on the sphere (random) or within ~3 degrees of the
    triangle's plane (grazing)."""
    a, b, c = tris[:, 0:3].astype(np.float64), tris[:, 3:6].astype(np.float64), tris[:, 6:9].astype(np.float64)
    cr = np.cross(b - a, c - a)
    area = np.linalg.norm(cr, axis=1)
    k = rng.integers(0, len(tris), size=n)  # every triangle alike (the dragon's, not the ground's area)
    r1, r2 = rng.random(n), rng.random(n)
    s = np.sqrt(r1)
    P = (1 - s)[:, None] * a[k] + (s * (1 - r2))[:, None] * b[k] + (s * r2)[:, None] * c[k]
    if mode == "random":
        u = rng.normal(size=(n, 3))
    else:  # grazing: an in-plane direction tilted by up to ~3 degrees out of the plane
        nrm = cr[k] / np.maximum(area[k], 1e-300)[:, None]
        t = rng.normal(size=(n, 3))
        t -= (t * nrm).sum(1)[:, None] * nrm
        t /= np.linalg.norm(t, axis=1)[:, None]
        u = t + rng.uniform(-0.05, 0.05, n)[:, None] * nrm
    u /= np.linalg.norm(u, axis=1)[:, None]
    o = P + D * u
    rays = np.empty((n, 6), np.float32)
    rays[:, 0:3] = o
    rays[:, 3:6] = -u
    return rays


def compare(rk, rays: np.ndarray) -> dict:
    n = rays.shape[0]
    t = np.zeros(n, np.float32)
    k = np.zeros(n, np.int32)
    L = _capi.lib(hostsim=True)
    assert L.rt_hostsim_fast_queries(rk.ctx, _capi.ptr(rays), n, _capi.ptr(t), _capi.ptr(k)) == 0
    ex = rk.intersect(rays)
    want_t = np.where(ex[:, 0] == 1, ex[:, 2].view(np.float32), -1.0).astype(np.float32)
    want_k = np.where(ex[:, 0] == 1, ex[:, 1], -1)
    settled = t != -2.0
    wrong = settled & ((t.view(np.uint32) != want_t.view(np.uint32)) | (k != want_k))
    miss_wrong = wrong & (t == -1.0) & (want_t != -1.0)
    out = {"rays": int(n), "settled": int(settled.sum()), "to_exact": int((~settled).sum()), "wrong": int(wrong.sum()),
           "wrong_miss": int(miss_wrong.sum())}
    if wrong.any():
        i = int(np.flatnonzero(wrong)[0])
        out["example"] = {"ray": rays[i].tolist(), "fast": [float(t[i]), int(k[i])],
                          "exact": [float(want_t[i]), int(want_k[i])]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--d", type=float, nargs="+", default=[10, 100, 1000, 10000, 100000])
    ap.add_argument("--n", type=int, default=200000)
    ap.add_argument("--mode", choices=["random", "grazing"], nargs="+", default=["random"])
    ap.add_argument("--near-scale", type=float, default=-1.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=200000)
    ap.add_argument("--label", default="product")
    a = ap.parse_args()
    P, rk = kernel(a.scene)
    if a.near_scale >= 0:
        rk.test_schedule(near_scale=a.near_scale)
    for mode in a.mode:
        for D in a.d:
            rng = np.random.default_rng([a.seed, int(D * 1000), 0 if mode == "random" else 1])
            tot = {}
            t0 = time.time()
            left = a.n
            while left > 0:
                m = min(left, a.chunk)
                r = compare(rk, far_rays(P.triangles, D, m, mode, rng))
                for key, v in r.items():
                    if key == "example":
                        tot.setdefault("example", v)
                    else:
                        tot[key] = tot.get(key, 0) + v
                left -= m
            print(json.dumps({"label": a.label, "lib": os.path.basename(_capi.HOSTSIM), "scene": a.scene,
                              "mode": mode, "D": D, "near_scale": a.near_scale,
                              "s": round(time.time() - t0, 1), **tot}), flush=True)


if __name__ == "__main__":
    main()
