"""Tie settlement on the GPU against the exact octree walk (debug tool): camera-like rays of the
cfg2 view (a dense jittered grid: edge hits tie) and the reference-pinned tie-prone rays,
walked by the quad walk (mode 4) and the row walk (mode 8) of rt_device_queries; every settled
answer must equal the exact walk's (rt_intersect). Mismatches are saved for study.

  python tools/tie_debug.py [--n 4000000] [--out gpurun_out/tie_debug.npz]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4 << 20)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "tie_debug.npz"))
    args = ap.parse_args()
    import bench
    import rt_amd
    from rt_amd import _capi
    from conftest import load_golden

    P, sky, cam17 = bench.build_inputs("cfg2")
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky), None,
                             device=0)
    m = cam17[:16].reshape(4, 4)
    o = m[:3, 3]
    rng = np.random.default_rng(3)
    # camera rays through a jittered grid around the view direction (as get_camera_ray would)
    xn = rng.uniform(-1.8, 1.8, args.n).astype(np.float32)
    yn = rng.uniform(-1, 1, args.n).astype(np.float32)
    p = np.stack([xn, yn, np.full(args.n, cam17[16], np.float32), np.ones(args.n, np.float32)], 1) @ m.T
    d = p[:, :3] - o[None, :]
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    sets = {"camera": (np.tile(o[None], (args.n, 1)).astype(np.float32), d)}
    g = load_golden("rays_dragon.npz")["rays"].astype(np.float32)
    sets["tie_prone"] = (g[:, 0:3], g[:, 3:6])
    out, bad_all = {}, {}
    for name, (ro, rd) in sets.items():
        n = ro.shape[0]
        r8 = np.zeros((n, 8), np.float32)
        r8[:, 0:3] = ro
        r8[:, 4:7] = rd
        res = {}
        for mode in (4, 8):
            t = np.zeros(n, np.float32)
            k = np.zeros(n, np.int32)
            ms = ctypes.c_double()
            assert _capi.lib().rt_device_queries(rk.ctx, mode, _capi.ptr(r8), n, 1, _capi.ptr(t), _capi.ptr(k),
                                                 ctypes.byref(ms)) == 0
            res[mode] = (t, k)
        ex = rk.intersect(np.concatenate([ro, rd], 1))
        want_t = np.where(ex[:, 0] == 1, ex[:, 2].view(np.float32), -1.0).astype(np.float32)
        rep = {"rays": int(n)}
        for mode, (t, k) in res.items():
            ok = t != -2.0
            bad_t = ok & (t.view(np.uint32) != want_t.view(np.uint32))
            bad = bad_t | (ok & (ex[:, 0] == 1) & (k != ex[:, 1]))
            rep[f"mode{mode}"] = {"settled": int(ok.sum()), "unsettled": int((~ok).sum()), "t_mismatch": int(bad_t.sum()),
                                  "triangle_mismatch": int((bad & ~bad_t).sum())}
            if bad.any():
                bad_all[f"{name}_mode{mode}"] = np.concatenate([ro[bad], rd[bad], t[bad, None], want_t[bad, None]], 1)
        out[name] = rep
        print(name, json.dumps(rep), flush=True)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    np.savez(args.out, **bad_all) if bad_all else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
