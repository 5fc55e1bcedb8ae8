"""Row walks (rt_row.h: 16 lanes per query over the 16-wide search BVH) against the
quad walks (rt_quad.h) and the exact octree walk, on the dragon stand-in.

The row walk must give the rt_fast.h answer exactly: the same closest (t, k) or
occluded flag, and the same "needs the exact walk" verdict (-2), for every ray —
tie-prone rays of the reference-pinned fixture (tests/golden/rays_dragon.npz,
answers of the reference's own BVH::intersect), rays leaving the surface in
cosine-distributed directions (the secondary-ray mix) and camera rays."""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np
import pytest

from conftest import load_golden, parsed_scene

import rt_amd
from rt_amd import _capi

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _queries(rk, mode, rays8):
    n = rays8.shape[0]
    t = np.zeros(n, dtype=np.float32)
    k = np.zeros(n, dtype=np.int32)
    ms = ctypes.c_double()
    rc = _capi.lib().rt_device_queries(rk.ctx, mode, _capi.ptr(rays8), n, 1, _capi.ptr(t), _capi.ptr(k),
                                       ctypes.byref(ms))
    assert rc == 0, _capi.lib().rt_last_error(rk.ctx)
    return t, k


def _rays8(o, d):
    r = np.zeros((o.shape[0], 8), np.float32)
    r[:, 0:3] = o
    r[:, 4:7] = d
    return r


@pytest.mark.gpu
def test_gpu_row_walks_match_quad_walks_and_octree():
    import query_bench
    P = parsed_scene("dragon")
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(np.ones((8, 16, 3), np.float32)), None)
    g = load_golden("rays_dragon.npz")["rays"].astype(np.float32)
    sets = {"tie_prone": _rays8(g[:, 0:3], g[:, 3:6]),
            "surface": query_bench.make_rays(np.asarray(P.triangles, np.float32).reshape(-1, 9), 1 << 16)}
    rng = np.random.default_rng(7)
    cam = rt_amd.Camera.preset("dragon")
    o = np.tile(cam.view_matrix[:3, 3][None], (4096, 1)).astype(np.float32)
    d = rng.normal(size=(4096, 3)).astype(np.float32) * np.float32(0.15) + np.float32([0, -0.45, -1.0])
    sets["camera"] = _rays8(o, (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32))
    seen_unoccluded = False
    for name, rays in sets.items():
        tq, kq = _queries(rk, 4, rays)   # closest, quad walk
        tr, kr = _queries(rk, 8, rays)   # closest, row walk
        np.testing.assert_array_equal(tr.view(np.uint32), tq.view(np.uint32), err_msg=f"{name}: closest t")
        np.testing.assert_array_equal(kr, kq, err_msg=f"{name}: closest k")
        aq, _ = _queries(rk, 5, rays)    # occlusion, quad walk
        ar, _ = _queries(rk, 9, rays)    # occlusion, row walk
        np.testing.assert_array_equal(ar.view(np.uint32), aq.view(np.uint32), err_msg=f"{name}: occlusion")
        assert (tr > 0).any() and (ar == 1.0).any(), name
        seen_unoccluded = seen_unoccluded or bool((ar == 0.0).any())
        # the settled closest answers against the exact octree walk (BVH::intersect)
        ok = tr != -2.0
        ex = rk.intersect(rays[ok][:, [0, 1, 2, 4, 5, 6]])
        np.testing.assert_array_equal(np.where(ex[:, 0] == 1, ex[:, 2].view(np.float32), -1.0).astype(np.float32)
                                      .view(np.uint32), tr[ok].view(np.uint32), err_msg=f"{name}: vs octree")
        # ... and the triangle (rows and quads settle same-leaf ties the way the octree walk does)
        np.testing.assert_array_equal(np.where(ex[:, 0] == 1, ex[:, 1], -1), kr[ok], err_msg=f"{name}: k vs octree")
    assert seen_unoccluded
