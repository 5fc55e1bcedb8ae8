"""Far ray origins (DESIGN.md §4 "Far origins and grazing hits").

The reference's Moller-Trumbore test (triangle.h:24-44) accepts rays that pass outside a
triangle by ~eps |o - a| / (sin(alpha) cos(theta)): far origins and grazing angles widen it
beyond the search BVH's padded boxes. A query whose origin lies outside the near box (the
scene's box widened by its largest extent) is answered by the exact octree walk.

Fixtures (tools/gen_golden_far.py, written by the compiled reference):
* far_rays_{cornell,dragon}.npz: rays aimed at surface points from D = 1e2 ... 1e5 along
  random and grazing directions (and two near distances), with BVH::intersect's answers;
* far_render_{cornell,dragon}_tele.npz: whole frames from telephoto cameras 1000x farther
  than the presets (RenderKernel::render).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import golden_io as gio
from conftest import load_golden, parsed_scene

import rt_amd
import rt_cases
from rt_amd import _capi


def _kernel(scene: str, hostsim: bool, W=4, H=4, spp=1, nb=1, sky="S"):
    P = parsed_scene(scene)
    return rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(W, H), P.triangles, P.materials,
                               P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                               rt_amd.Image.from_rgb(rt_cases.sky(sky)), None, hostsim=hostsim)


def _want(g):
    h = g["hits"]
    t = np.where(h["found"] == 1, h["t"], np.float32(-1.0)).astype(np.float32)
    k = np.where(h["found"] == 1, h["prim"], -1).astype(np.int32)
    return t, k


def _near(scene, o, scale=0.5):
    """Origins inside the near box (rt_view_near: the scene's box widened on every side by
    scale x its largest extent; RT_NEAR_SCALE 0.5), with a 1e-3 guard band either way."""
    v = np.asarray(parsed_scene(scene).triangles, np.float64).reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    w = scale * (hi - lo).max()
    inside = ((o >= lo - w + 1e-3) & (o <= hi + w - 1e-3)).all(1)
    outside = ((o < lo - w - 1e-3) | (o > hi + w + 1e-3)).any(1)
    return inside, outside


def _check_settled(t, k, g, name, scene):
    """Every settled answer (t != -2) is the reference's, bit for bit; every origin outside
    the near box (all of D >= 100) is left to the exact walk; inside, the search BVH
    settles almost all."""
    wt, wk = _want(g)
    ok = t != -2.0
    np.testing.assert_array_equal(t[ok].view(np.uint32), wt[ok].view(np.uint32), err_msg=f"{name}: t")
    np.testing.assert_array_equal(k[ok], wk[ok], err_msg=f"{name}: triangle")
    inside, outside = _near(scene, g["rays"][:, 0:3].astype(np.float64))
    assert outside[g["dist"] >= 100.0].all()
    assert (t[outside] == -2.0).all(), f"{name}: far origins settled by the search BVH"
    assert inside.sum() >= 512 and ok[inside].mean() > 0.9, \
        f"{name}: near rays left to the exact walk: {(~ok[inside]).sum()} of {inside.sum()}"


@pytest.mark.parametrize("scene", ["cornell", "dragon"])
def test_hostsim_fast_query_far_origins(scene):
    """The search-BVH query of the render's k_trace stage (rt_fast.h fast_query_closest,
    hostsim) on the far-origin fixture: far origins go to the exact walk, near ones settle
    with the reference's (t, triangle)."""
    g = load_golden(f"far_rays_{scene}.npz")
    rk = _kernel(scene, hostsim=True)
    rays = np.ascontiguousarray(g["rays"], np.float32)
    n = rays.shape[0]
    t = np.zeros(n, np.float32)
    k = np.zeros(n, np.int32)
    L = _capi.lib(hostsim=True)
    assert L.rt_hostsim_fast_queries(rk.ctx, _capi.ptr(rays), n, _capi.ptr(t), _capi.ptr(k)) == 0
    _check_settled(t, k, g, scene, scene)


@pytest.mark.parametrize("scene", ["cornell", "dragon"])
def test_hostsim_intersect_far_origins(scene):
    """rt_intersect (BVH::intersect + the sphere loop) on the far-origin fixture: every
    field of every answer bit for bit (hit flag, primitive, t, point, normal)."""
    g = load_golden(f"far_rays_{scene}.npz")
    rk = _kernel(scene, hostsim=True)
    ex = rk.intersect(np.ascontiguousarray(g["rays"], np.float32))
    h = g["hits"]
    np.testing.assert_array_equal(ex[:, 0], h["found"])
    hit = h["found"] == 1
    np.testing.assert_array_equal(ex[hit, 1], h["prim"][hit])
    np.testing.assert_array_equal(ex[hit, 2].view(np.float32).view(np.uint32), h["t"][hit].view(np.uint32))
    np.testing.assert_array_equal(ex[hit, 3:6].view(np.float32).view(np.uint32), h["p"][hit].view(np.uint32))
    np.testing.assert_array_equal(ex[hit, 6:9].view(np.float32).view(np.uint32), h["n"][hit].view(np.uint32))


def _render_tele(name, hostsim):
    import json
    man = json.load(open(os.path.join(gio.GOLDEN, "far_manifest.json")))["renders"][name]
    g = load_golden(f"far_render_{name}.npz")
    rk = _kernel(man["scene"], hostsim, man["W"], man["H"], man["spp"], man["bounces"], man["sky"])
    cam = g["camera"]
    rk.set_camera(rt_amd.Camera(cam[:16], cam[16]))
    rk.render()
    return rk.frame_buffer.pixels, g["rgba"]


@pytest.mark.parametrize("name", ["cornell_tele", "dragon_tele"])
def test_hostsim_far_telephoto_render(name):
    """A whole frame from a camera 1000x farther than the preset (every camera ray from
    outside the near box, so every one takes the exact walk), bit for bit."""
    got, want = _render_tele(name, hostsim=True)
    assert gio.compare_rgb(got, want)["bitwise_fraction"] == 1.0
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_far_fixtures_see_the_scene():
    """The telephoto frames show the scene (not only sky) and the far rays hit it."""
    for name in ("cornell_tele", "dragon_tele"):
        rgb = load_golden(f"far_render_{name}.npz")["rgba"][..., :3]
        assert np.unique(rgb.reshape(-1, 3), axis=0).shape[0] > 100, name
    for sc in ("cornell", "dragon"):
        g = load_golden(f"far_rays_{sc}.npz")
        assert g["hits"]["found"].mean() > 0.99, sc


def test_near_scale_changes_no_answer():
    """The near box only decides which walk answers: with near_scale 0 (the scene's own box)
    and 1e30 (no routing) every near ray the fast query settles still gets the reference's
    answer, and with 0 nothing 10 or more units away is settled."""
    g = load_golden("far_rays_cornell.npz")
    rays = np.ascontiguousarray(g["rays"], np.float32)
    n = rays.shape[0]
    L = _capi.lib(hostsim=True)
    for scale in (0.0, 1e30):
        rk = _kernel("cornell", hostsim=True)
        rk.test_schedule(near_scale=scale)
        t = np.zeros(n, np.float32)
        k = np.zeros(n, np.int32)
        assert L.rt_hostsim_fast_queries(rk.ctx, _capi.ptr(rays), n, _capi.ptr(t), _capi.ptr(k)) == 0
        wt, wk = _want(g)
        ok = t != -2.0
        near = g["dist"] < 100.0
        np.testing.assert_array_equal(t[ok & near].view(np.uint32), wt[ok & near].view(np.uint32))
        if scale == 0.0:
            assert not ok[g["dist"] >= 10.0].any()


def test_schedule_rejects_non_finite_values():
    rk = _kernel("cornell", hostsim=True)
    L = _capi.lib(hostsim=True)
    for key, v in (("lanes", float("nan")), ("lanes", 1e12), ("near_scale", float("inf")), ("fast_k", -3e9)):
        assert L.rt_test_schedule(rk.ctx, key.encode(), ctypes.c_double(v)) == rt_amd.RT_ERR_ARG, key
    assert L.rt_test_schedule(rk.ctx, b"near_scale", ctypes.c_double(2.5)) == 0


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_tele", "dragon_tele"])
def test_gpu_far_telephoto_render(name):
    """The product (gfx950) on the telephoto frames: bitwise equal to the reference's."""
    got, want = _render_tele(name, hostsim=False)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), gio.compare_rgb(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["cornell", "dragon"])
def test_gpu_far_origin_queries(scene):
    """The device's search-BVH walks on the far-origin fixture (rt_device_queries: one lane,
    quads, rows): far origins go to the exact walk (-2), near ones settle with the
    reference's (t, triangle); rt_intersect answers all of them bit for bit."""
    g = load_golden(f"far_rays_{scene}.npz")
    rk = _kernel(scene, hostsim=False)
    rays8 = np.zeros((g["rays"].shape[0], 8), np.float32)
    rays8[:, 0:3] = g["rays"][:, 0:3]
    rays8[:, 4:7] = g["rays"][:, 3:6]
    n = rays8.shape[0]
    for mode in (0, 4, 8):  # closest: one lane, quad walk, row walk
        t = np.zeros(n, np.float32)
        k = np.zeros(n, np.int32)
        ms = ctypes.c_double()
        rc = _capi.lib().rt_device_queries(rk.ctx, mode, _capi.ptr(rays8), n, 1, _capi.ptr(t), _capi.ptr(k),
                                           ctypes.byref(ms))
        assert rc == 0
        _check_settled(t, k, g, f"{scene} mode {mode}", scene)
    ex = rk.intersect(np.ascontiguousarray(g["rays"], np.float32))
    wt, wk = _want(g)
    np.testing.assert_array_equal(np.where(ex[:, 0] == 1, ex[:, 2].view(np.float32), -1.0).astype(np.float32)
                                  .view(np.uint32), wt.view(np.uint32))
    np.testing.assert_array_equal(np.where(ex[:, 0] == 1, ex[:, 1], -1), wk)
