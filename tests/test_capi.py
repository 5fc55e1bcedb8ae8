"""The C-ABI boundary (include/rt_hip.h): the product library loads, exports
every declared symbol, rejects bad arguments with RT_ERR_* codes, and its
host-side helpers (OBJ ingest, camera presets, env CDF, octree build)
reproduce the reference's host prerequisites bit for bit (golden fixtures
written by the compiled reference, tools/gen_golden.py)."""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np
import pytest

import golden_io as gio
import scenes
from conftest import REPO, load_golden, parsed_scene

import rt_amd
from rt_amd import _capi


def header_symbols():
    src = open(os.path.join(REPO, "include", "rt_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_table():
    assert header_symbols() == sorted(_capi.EXPORTS)


@pytest.mark.parametrize("which", ["product", "hostsim"])
def test_library_exports_every_symbol(which):
    L = _capi.lib(hostsim=(which == "hostsim"))
    missing = [s for s in header_symbols() if getattr(L, s, None) is None]
    assert not missing, missing


def test_product_exports_device_extras():
    L = _capi.lib()
    for s in ("rt_device_libm", "rt_device_last_kernel_ms"):
        assert getattr(L, s, None) is not None


def test_product_has_no_cpu_path():
    """librt_hip.so must fail loudly without a device, never fall back."""
    if os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd"):
        pytest.skip("a GPU may be visible here")
    L = _capi.lib()
    h = ctypes.c_void_p()
    rc = L.rt_create(0, ctypes.byref(h))
    assert rc == -5, rc
    assert b"no HIP device" in L.rt_last_error(None)


def test_version():
    assert _capi.lib().rt_version() == _capi.lib(hostsim=True).rt_version() >= 10000


def test_argument_errors():
    L = _capi.lib(hostsim=True)
    h = ctypes.c_void_p()
    assert L.rt_create(0, ctypes.byref(h)) == 0
    try:
        tri = np.zeros((1, 9), np.float32)
        mats = rt_amd.make_materials([((0, 0, 0), (1, 1, 1), 0.0, 0.5)])
        bad_mi = np.array([3], np.int32)
        assert L.rt_set_scene(h, _capi.ptr(tri), 1, _capi.ptr(bad_mi), 1, _capi.ptr(mats), 1, None, 0, None, 0) == -1
        assert b"material index" in L.rt_last_error(h)
        fb = np.zeros((4, 4, 4), np.float32)
        assert L.rt_render(h, 4, 4, 1, 1, _capi.ptr(fb)) == -3  # no scene yet
        mi = np.array([0], np.int32)
        assert L.rt_set_scene(h, _capi.ptr(tri), 1, _capi.ptr(mi), 1, _capi.ptr(mats), 1, None, 0, None, 0) == 0
        assert L.rt_build_bvh(h, 33, 8) == -1  # deeper than the device stack bound
        assert L.rt_build_bvh(h, 32, 8) == 0
        assert L.rt_render(h, 4, 4, 1, 1, _capi.ptr(fb)) == -3  # no env
        sky = np.ones((2, 2, 3), np.float32)
        assert L.rt_set_env(h, _capi.ptr(sky), 2, 2, 5, None) == -1
        assert L.rt_set_env(h, _capi.ptr(sky), 2, 2, 3, None) == 0
        assert L.rt_render(h, 4, 4, 1, 1, _capi.ptr(fb)) == -3  # no camera
        cam = np.eye(4, dtype=np.float32)
        assert L.rt_set_camera(h, _capi.ptr(cam), 1.0) == 0
        assert L.rt_render(h, 0, 4, 1, 1, _capi.ptr(fb)) == -1
        # seed 31 + x*y*spp must fit an int (render_kernel.cpp:77)
        assert L.rt_render(h, 50000, 50000, 2, 1, _capi.ptr(fb)) == -1
        assert L.rt_render(h, 4, 4, 1, 1, _capi.ptr(fb)) == 0
        xy = np.array([[4, 0]], np.int32)
        rgba = np.zeros((1, 4), np.float32)
        assert L.rt_render_pixels(h, 4, 4, 1, 1, _capi.ptr(xy), 1, _capi.ptr(rgba)) == -1
    finally:
        L.rt_destroy(h)


# ----------------------------------------------------------- host ingest
@pytest.mark.parametrize("scene", ["cornell12", "cornell", "mis"])
def test_parse_obj_matches_reference(scene):
    """Utils::parse_obj (utils.cpp:16-98) incl. rapidobj triangulation."""
    P = parsed_scene(scene)
    g = load_golden(f"parse_{scene if scene != 'cornell' else 'cornell'}.npz")
    np.testing.assert_array_equal(P.triangles.view(np.uint32), g["tris"].view(np.uint32))
    np.testing.assert_array_equal(P.material_indices, g["mat_idx"])
    np.testing.assert_array_equal(P.materials.view(np.uint32), g["mats"].view(np.uint32))
    np.testing.assert_array_equal(P.emissive_triangle_indices, g["emissive"])


@pytest.mark.parametrize("scene", ["cornell12", "cornell", "mis"])
def test_octree_matches_reference(scene):
    """BVH ctor (bvh.cpp:19-60, bvh.h:55-125, child-min quirk included)."""
    P = parsed_scene(scene)
    d = rt_amd.octree_dump(P.triangles)
    g = load_golden(f"octree_{scene}.npz")["dump"].tobytes()
    assert d == g


def test_camera_presets_match_reference(cameras):
    """Camera presets (camera.cpp:3-8, mat.cpp) composed on the host."""
    for name, want in cameras.items():
        c = rt_amd.Camera.preset(name)
        np.testing.assert_array_equal(c.as17().view(np.uint32), want.view(np.uint32), err_msg=name)


def test_env_cdf_matches_reference(manifest):
    """compute_env_map_cdf (utils.cpp:126-142): sequential float prefix sum of
    the double-evaluated luminance (image.h:80-85)."""
    g = load_golden("skyS_cdf.npz")
    img = rt_amd.Image.from_rgb(scenes.make_sky("S"))
    np.testing.assert_array_equal(rt_amd.compute_env_map_cdf(img).view(np.uint32), g["cdf"].view(np.uint32))
    np.testing.assert_array_equal(rt_amd.luminance_of_pixels(img).view(np.uint32), g["lum"].view(np.uint32))
    imgL = rt_amd.Image.from_rgb(scenes.make_sky("L"))
    assert gio.sha256(rt_amd.compute_env_map_cdf(imgL)) == manifest["skyL"]["cdf_sha256"]


def test_bvh_preorder_roundtrip():
    """rt_set_bvh_preorder accepts a caller's pre-order walk of BVH::_root."""
    P = parsed_scene("mis")
    dump = rt_amd.octree_dump(P.triangles)
    sky = rt_amd.Image.from_rgb(scenes.make_sky("S"))
    fb = rt_amd.Image(8, 8)
    rk = rt_amd.RenderKernel(8, 8, 1, 2, fb, P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles, preorder=dump), sky, None, hostsim=True)
    assert rk.bvh_dump() == dump
    info = rk.bvh_info()
    assert info["octree_nodes"] == 5049 and info["max_depth"] <= 32
    with pytest.raises(rt_amd.RtError):
        rt_amd.RenderKernel(8, 8, 1, 2, fb, P.triangles, P.materials, P.emissive_triangle_indices,
                            P.material_indices, None, rt_amd.BVH(P.triangles, preorder=dump[:-7]), sky, None,
                            hostsim=True)


def test_mesh_load_missing_file():
    with pytest.raises(rt_amd.RtError):
        rt_amd.parse_obj("/nonexistent/scene.obj")
