"""Per-sample bounce counts of a frame's pixels (analysis for the speculative
sample-chain schedule; see chain_probe.cpp). Writes an npz with h[n, spp] and
q[n, spp] for every k-th row and column of the frame."""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests")]
import conftest  # noqa: E402
import rt_cases  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="cfg2_dragon")
    ap.add_argument("--step", type=int, default=8)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--out", default="/tmp/chains.npz")
    a = ap.parse_args()
    so = "/tmp/libchain_probe.so"
    subprocess.run(["g++", "-std=gnu++20", "-O2", "-fopenmp", "-ffp-contract=off", "-fPIC", "-shared",
                    os.path.join(HERE, "chain_probe.cpp"), "-o", so], check=True)
    import json
    man = json.load(open(os.path.join(REPO, "tests", "golden", "manifest.json")))
    e = dict(man["renders"][a.case])
    cams = np.load(os.path.join(REPO, "tests", "golden", "cameras.npz"))
    cam = cams[e["camera"]]
    P = conftest.parsed_scene(e["scene"])
    mats, mi, sph = rt_cases.sphere_buffers(e, P, rt_cases.materials_for(e, P))
    env = np.ascontiguousarray(rt_cases.sky(e["sky"]), np.float32)
    L = ctypes.CDLL(so)
    V = ctypes.c_void_p
    L.oracle_scene_create.restype = V
    L.oracle_scene_create.argtypes = [V, ctypes.c_int, V, V, ctypes.c_int, V, ctypes.c_int, V, ctypes.c_int,
                                      V, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.probe_chains.argtypes = [V, V, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               V, ctypes.c_long, V, V]
    p = lambda x: None if x is None else x.ctypes.data_as(V)  # noqa: E731
    tris = np.ascontiguousarray(P.triangles, np.float32)
    mi = np.ascontiguousarray(mi, np.int32)
    mats = np.ascontiguousarray(mats, np.float32)
    em = np.ascontiguousarray(P.emissive_triangle_indices, np.int32)
    sphz = np.zeros((0, 5), np.float32) if sph is None else np.ascontiguousarray(sph, np.float32)
    s = L.oracle_scene_create(p(tris), tris.shape[0], p(mi), p(mats), mats.shape[0], p(em), em.shape[0],
                              p(sphz), sphz.shape[0], p(env), env.shape[1], env.shape[0], 32, 8)
    W, H, spp, nb = e["W"], e["H"], a.spp or e["spp"], e["bounces"]
    ys, xs = np.mgrid[0:H:a.step, 0:W:a.step]
    px = np.ascontiguousarray(np.stack([xs.ravel(), ys.ravel()], 1), np.int32)
    n = px.shape[0]
    hs = np.zeros((n, spp), np.uint8)
    qs = np.zeros((n, spp), np.uint8)
    view = np.ascontiguousarray(cam[:16], np.float32)
    import time
    t0 = time.time()
    L.probe_chains(s, p(view), float(np.float32(cam[16])), W, H, spp, nb, p(px), n, p(hs), p(qs))
    print(f"{n} pixels x {spp} spp in {time.time() - t0:.1f} s")
    np.savez_compressed(a.out, h=hs, q=qs, px=px, W=W, H=H, spp=spp, bounces=nb, emissive=em.shape[0])


if __name__ == "__main__":
    main()
