"""ctypes bindings to oracle/liboracle.so — the CPU restatement of the
reference render path (oracle/cpu_oracle.cpp).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / baseline, never as the
thing measured.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "-s"], check=True)
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        L.oracle_scene_create.restype = P
        L.oracle_scene_create.argtypes = [P, ctypes.c_int, P, P, ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int,
                                          P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_scene_destroy.argtypes = [P]
        L.oracle_set_use_bvh.argtypes = [P, ctypes.c_int]
        L.oracle_bvh_dump.restype = ctypes.c_long
        L.oracle_bvh_dump.argtypes = [P, P, ctypes.c_long]
        L.oracle_intersect.argtypes = [P, P, ctypes.c_int, P, P]
        L.oracle_render.restype = ctypes.c_double
        L.oracle_render.argtypes = [P, P, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    P, ctypes.c_long, P, ctypes.c_int, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleScene:
    """Scene inputs exactly as the reference RenderKernel receives them
    (render_kernel.h:24-46): triangles [N,9], material indices, materials
    [M,10] (emission rgba, diffuse rgba, metalness, roughness), emissive
    triangle ids, spheres [S,5] (cx,cy,cz,r,prim), env RGB [H,W,3]."""

    def __init__(self, tris, mat_idx, mats, emissive, env=None, spheres=None, max_depth=32, leaf_max=8):
        self.tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        self.mat_idx = np.ascontiguousarray(mat_idx, dtype=np.int32)
        self.mats = np.ascontiguousarray(mats, dtype=np.float32).reshape(-1, 10)
        self.emissive = np.ascontiguousarray(emissive, dtype=np.int32)
        self.spheres = np.ascontiguousarray(spheres if spheres is not None else np.zeros((0, 5)), dtype=np.float32)
        self.env = None if env is None else np.ascontiguousarray(env, dtype=np.float32)
        eh, ew = (0, 0) if env is None else self.env.shape[:2]
        assert self.mat_idx.shape[0] >= self.tris.shape[0] + self.spheres.shape[0], "one material index per primitive"
        self.h = lib().oracle_scene_create(
            _p(self.tris), self.tris.shape[0], _p(self.mat_idx), _p(self.mats), self.mats.shape[0],
            _p(self.emissive), self.emissive.shape[0], _p(self.spheres), self.spheres.shape[0],
            _p(self.env), ew, eh, max_depth, leaf_max)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_scene_destroy(self.h)
            self.h = None

    def set_use_bvh(self, use_bvh: bool):
        """USE_BVH (render_kernel.h:13): False = the brute-force intersect_scene loop."""
        lib().oracle_set_use_bvh(self.h, 1 if use_bvh else 0)

    def octree_dump(self) -> bytes:
        n = lib().oracle_bvh_dump(self.h, None, 0)
        buf = ctypes.create_string_buffer(n)
        lib().oracle_bvh_dump(self.h, buf, n)
        return buf.raw

    def intersect(self, rays, counters=False):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        out = np.zeros((rays.shape[0], 11), dtype=np.int32)
        cnt = np.zeros(5, dtype=np.uint64)
        lib().oracle_intersect(self.h, _p(rays), rays.shape[0], _p(out), _p(cnt) if counters else None)
        return (out, cnt) if counters else out

    def render(self, camera17, W, H, spp, bounces, pixels=None, fb=None, threads=0, counters=False):
        """camera17 = 16 floats row-major view matrix + fov_dist. Returns (fb or
        pixel colours, seconds[, counters])."""
        cam = np.ascontiguousarray(camera17[:16], dtype=np.float32)
        fov = float(np.float32(camera17[16]))
        if fb is None:
            fb = np.zeros((H, W, 4), dtype=np.float32)
            fb[..., 3] = 1.0
        px = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int32).reshape(-1, 2)
        cnt = np.zeros(5, dtype=np.uint64)
        sec = lib().oracle_render(self.h, _p(cam), fov, W, H, spp, bounces, _p(px), 0 if px is None else px.shape[0],
                                  _p(fb), threads, _p(cnt) if counters else None)
        res = fb if px is None else fb[px[:, 1], px[:, 0]]
        return (res, sec, cnt) if counters else (res, sec)
