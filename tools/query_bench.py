"""Search-BVH query micro-benchmark on the dragon stand-in (GPU box).

Rays: bounce-like rays from points on the scene's triangles (offset 1e-4
along the face normal, cosine-weighted directions about it) in triangle-index
order, so neighbouring lanes start near each other like a wavefront queue in
pixel order. Runs every walk variant of rt_device_queries (closest and any),
checks that the variants agree bit for bit wherever none of them needs the
exact walk, and checks the closest answers against the exact octree walk
(rt_intersect) on a subset.

  python tools/query_bench.py [--n 1000000] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def make_rays(tris: np.ndarray, n: int, seed: int = 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.integers(0, tris.shape[0], n))
    t = tris[idx].reshape(-1, 3, 3).astype(np.float64)
    r1, r2 = rng.random(n), rng.random(n)
    s = np.sqrt(r1)
    p = (1 - s)[:, None] * t[:, 0] + (s * (1 - r2))[:, None] * t[:, 1] + (s * r2)[:, None] * t[:, 2]
    nrm = np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True) + 1e-30
    # cosine-weighted direction about the normal, on a random side
    side = np.where(rng.random(n) < 0.5, 1.0, -1.0)[:, None]
    nz = nrm * side
    a = np.where(np.abs(nz[:, :1]) > 0.9, np.array([[0, 1.0, 0]]), np.array([[1.0, 0, 0]]))
    tx = np.cross(nz, a)
    tx /= np.linalg.norm(tx, axis=1, keepdims=True)
    ty = np.cross(nz, tx)
    u1, u2 = rng.random(n), rng.random(n)
    rr, ph = np.sqrt(u1), 2 * np.pi * u2
    d = (rr * np.cos(ph))[:, None] * tx + (rr * np.sin(ph))[:, None] * ty + np.sqrt(1 - u1)[:, None] * nz
    o = p + nz * 1e-4
    out = np.zeros((n, 8), dtype=np.float32)
    out[:, 0:3] = o
    out[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="0,2,4,6,1,3,5,7")
    args = ap.parse_args()
    import bench
    import rt_amd
    from rt_amd import _capi

    P, sky, cam17 = bench.build_inputs("cfg2")
    rk = rt_amd.RenderKernel(64, 64, 1, 1, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=0)
    rays = make_rays(np.asarray(P.triangles, dtype=np.float32).reshape(-1, 9), args.n)
    L = _capi.lib()
    res = {}
    names = {0: "closest/node-walk", 1: "any/node-walk", 2: "closest/item-walk", 3: "any/item-walk",
             4: "closest/quad-walk", 5: "any/quad-walk", 6: "closest/quad-walk@8w", 7: "any/quad-walk@8w",
             8: "closest/row-walk (16 lanes, 16-wide BVH)", 9: "any/row-walk (16 lanes, 16-wide BVH)"}
    for m in [int(x) for x in args.modes.split(",")]:
        t = np.zeros(args.n, dtype=np.float32)
        k = np.zeros(args.n, dtype=np.int32)
        ms = ctypes.c_double()
        rc = L.rt_device_queries(rk.ctx, m, _capi.ptr(rays), args.n, args.reps, _capi.ptr(t), _capi.ptr(k),
                                 ctypes.byref(ms))
        assert rc == 0, (rc, L.rt_last_error(rk.ctx))
        res[m] = (t, k)
        fb = int((t == -2.0).sum())
        line = {"mode": m, "name": names[m], "ms": round(ms.value, 3), "mrays_per_s": round(args.n / ms.value / 1e3, 1),
                "fallback": fb, "hits": int((t > 0).sum())}
        print(json.dumps(line), flush=True)
    # agreement between walks
    for a, b in ((0, 2), (1, 3), (0, 4), (1, 5), (0, 6), (1, 7), (4, 8), (5, 9)):
        if a in res and b in res:
            ta, ka = res[a]
            tb, kb = res[b]
            ok = (ta != -2.0) & (tb != -2.0)
            same = (ta[ok].view(np.int32) == tb[ok].view(np.int32)) & (ka[ok] == kb[ok])
            print(json.dumps({"agree": f"{names[a]} vs {names[b]}", "compared": int(ok.sum()),
                              "mismatch": int((~same).sum())}), flush=True)
    # closest vs the exact octree walk on a subset
    sub = np.arange(0, args.n, max(1, args.n // 20000))
    ex = rk.intersect(rays[sub][:, [0, 1, 2, 4, 5, 6]])
    for m in (0, 2, 4, 8):
        if m not in res:
            continue
        t, k = res[m]
        ok = t[sub] != -2.0
        et = ex[:, 2].view(np.float32)
        same = np.where(ex[ok, 0] == 1, t[sub][ok].view(np.int32) == ex[ok, 2], t[sub][ok] == -1.0)
        print(json.dumps({"exact_check": names[m], "compared": int(ok.sum()), "mismatch": int((~same).sum()),
                          "exact_hits": int((et > 0).sum())}), flush=True)
        assert same.all()


if __name__ == "__main__":
    main()
