"""USE_BVH 0 (render_kernel.h:13): INTERSECT_SCENE as the brute-force loop
(render_kernel.cpp:453-483 — closest by strict `<` in buffer order, the
lowest index wins a tie).

Pinned to the REFERENCE itself (tools/gen_golden_brute.py, tests/golden/brute_*):
ray answers of the public RenderKernel::intersect_scene (render_kernel.h:65) and
renders of the reference's render_kernel.cpp compiled with USE_BVH 0
(oracle/ref/render_kernel_brute.cpp). The oracle's restatement of the loop is
checked against the same fixtures, then used for the random-pixel cases. Host
(hostsim) and gfx950 (gpu marker) variants."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import golden_io as gio
import rt_cases
from conftest import load_golden, parsed_scene

import rt_amd

with open(os.path.join(gio.GOLDEN, "brute_manifest.json")) as _f:
    BRUTE = json.load(_f)
CORNELL_RAYS = ["cornell_regression", "cornell_edges", "cornell_edges_spheres"]
CORNELL_RENDERS = ["cfg1_cornell12_64", "cornell32_64", "cornell32_8spp", "mis_512", "spheres_cornell32_64"]


def _ray_kernel(entry, hostsim):
    """A context over the entry's scene (+ its analytic spheres), brute-force INTERSECT_SCENE."""
    P = parsed_scene(entry["scene"])
    mats, mi, spheres = rt_cases.sphere_buffers(entry, P, P.materials.copy())
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, mats, P.emissive_triangle_indices, mi,
                             spheres, rt_amd.BVH(P.triangles), rt_amd.Image(1, 1), None, hostsim=hostsim)
    rk.set_use_bvh(False)
    return rk


def _check_ref_rays(name, hostsim):
    """rt_intersect (USE_BVH 0) against RenderKernel::intersect_scene's own answers:
    found, primitive, t, point, normal bit for bit."""
    entry = BRUTE["rays"][name]
    g = load_golden(f"brute_rays_{name}.npz")
    got = _ray_kernel(entry, hostsim).intersect(g["rays"])
    want = np.ascontiguousarray(g["hits"]).view(np.int32).reshape(-1, 11)
    np.testing.assert_array_equal(got[:, :9], want[:, :9])
    assert int(got[:, 0].sum()) == entry["found"]


def _ref_render(name, hostsim):
    """A brute-force render fixture of the reference (USE_BVH 0 build) through the product."""
    e = dict(BRUTE["renders"][name])
    g = load_golden(f"brute_render_{name}.npz")
    rk, fb = rt_cases.make_kernel(e, _cameras(), hostsim)
    rk.set_use_bvh(False)
    if "px" not in g:
        rk.render()
        return fb.pixels, g["rgba"]
    px = g["px"]
    rk.ray_trace_pixels(px)
    return fb.pixels[px[:, 1], px[:, 0]], g["rgba"]


def _cameras():
    z = np.load(os.path.join(gio.GOLDEN, "cameras.npz"))
    return {k: z[k] for k in z.files}


def _bits_equal(got, want):
    return (np.ascontiguousarray(got).view(np.uint32) == np.ascontiguousarray(want).view(np.uint32)).all()


def _pixels(W, H, n=256, seed=5):
    """n distinct pixels (a pixel listed twice would accumulate twice in the oracle's framebuffer)."""
    rng = np.random.default_rng(seed)
    idx = rng.choice(W * H, n, replace=False)
    return np.stack([idx % W, idx // W], 1).astype(np.int32)


def _render_brute(name, manifest, cameras, hostsim, W=None, H=None, spp=None, px=None):
    e = rt_cases.golden_case(name, manifest)
    W, H, spp = W or e["W"], H or e["H"], spp or e["spp"]
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim, W=W, H=H, spp=spp)
    rk.set_use_bvh(False)
    S = rt_cases.oracle_scene(e)
    S.set_use_bvh(False)
    if px is None:
        rk.render()
        got = fb.pixels
        want, _ = S.render(cameras[e["camera"]], W, H, spp, e["bounces"])
    else:
        rk.ray_trace_pixels(px)
        got = fb.pixels[px[:, 1], px[:, 0]]
        want, _ = S.render(cameras[e["camera"]], W, H, spp, e["bounces"], pixels=px)
    return got, want


def _edge_rays(tris, n_per=4, seed=2):
    """Rays through points on triangle edges (shared edges give exact t ties)."""
    rng = np.random.default_rng(seed)
    t = tris.reshape(-1, 3, 3).astype(np.float64)
    pts = []
    for k in range(t.shape[0]):
        for _ in range(n_per):
            a, b = rng.choice(3, 2, replace=False)
            s = rng.random()
            pts.append(t[k, a] * (1 - s) + t[k, b] * s)
    pts = np.asarray(pts)
    o = pts + rng.normal(0, 1.0, pts.shape)
    d = pts - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], 1).astype(np.float32)


def _check_rays(hostsim):
    from oracle_bindings import OracleScene
    P = parsed_scene("cornell")
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles), rt_amd.Image(1, 1), None,
                             hostsim=hostsim)
    rk.set_use_bvh(False)
    S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices)
    S.set_use_bvh(False)
    rays = _edge_rays(P.triangles)
    got, want = rk.intersect(rays), S.intersect(rays)
    np.testing.assert_array_equal(got[:, :9], want[:, :9])
    return rays, got


# ---- the oracle's restatement of the loop, against the reference's answers
@pytest.mark.parametrize("name", CORNELL_RAYS)
def test_oracle_brute_rays_match_reference(name):
    from oracle_bindings import OracleScene
    entry = BRUTE["rays"][name]
    P = parsed_scene(entry["scene"])
    mats, mi, spheres = rt_cases.sphere_buffers(entry, P, P.materials.copy())
    S = OracleScene(P.triangles, mi, mats, P.emissive_triangle_indices, spheres=spheres)
    S.set_use_bvh(False)
    g = load_golden(f"brute_rays_{name}.npz")
    want = np.ascontiguousarray(g["hits"]).view(np.int32).reshape(-1, 11)
    np.testing.assert_array_equal(S.intersect(g["rays"])[:, :9], want[:, :9])


@pytest.mark.parametrize("name", CORNELL_RENDERS)
def test_oracle_brute_renders_match_reference(name):
    e = dict(BRUTE["renders"][name])
    g = load_golden(f"brute_render_{name}.npz")
    S = rt_cases.oracle_scene(e)
    S.set_use_bvh(False)
    got, _ = S.render(_cameras()[e["camera"]], e["W"], e["H"], e["spp"], e["bounces"], pixels=g.get("px"))
    assert _bits_equal(got, g["rgba"])


# ---- the product's device code compiled for the host (hostsim)
@pytest.mark.parametrize("name", CORNELL_RAYS)
def test_hostsim_brute_rays_match_reference(name):
    _check_ref_rays(name, hostsim=True)


@pytest.mark.parametrize("name", CORNELL_RENDERS)
def test_hostsim_brute_renders_match_reference(name):
    got, want = _ref_render(name, hostsim=True)
    assert _bits_equal(got, want)


@pytest.mark.parametrize("name", ["cfg1_cornell12", "cornell32_128"])
def test_hostsim_brute_frames_match_oracle(name, manifest, cameras):
    got, want = _render_brute(name, manifest, cameras, hostsim=True, W=64, H=64)
    assert (got.view(np.uint32) == want.view(np.uint32)).all()


def test_hostsim_brute_mis_pixels_match_oracle(manifest, cameras):
    got, want = _render_brute("mis_512", manifest, cameras, hostsim=True, spp=4, px=_pixels(512, 512, 128))
    assert (got.view(np.uint32) == want.view(np.uint32)).all()


def test_hostsim_brute_rays_and_ties():
    rays, got = _check_rays(hostsim=True)
    assert got[:, 0].sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", CORNELL_RAYS + ["dragon_tie_prone"])
def test_gpu_brute_rays_match_reference(name):
    _check_ref_rays(name, hostsim=False)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BRUTE["renders"]))
def test_gpu_brute_renders_match_reference(name):
    got, want = _ref_render(name, hostsim=False)
    assert _bits_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg1_cornell12", "cornell32_128"])
def test_gpu_brute_frames_match_oracle(name, manifest, cameras):
    got, want = _render_brute(name, manifest, cameras, hostsim=False)
    assert (got.view(np.uint32) == want.view(np.uint32)).all()


@pytest.mark.gpu
def test_gpu_brute_mis_and_rays_match_oracle(manifest, cameras):
    got, want = _render_brute("mis_512", manifest, cameras, hostsim=False, spp=4, px=_pixels(512, 512, 512))
    assert (got.view(np.uint32) == want.view(np.uint32)).all()
    _check_rays(hostsim=False)


@pytest.mark.gpu
def test_gpu_brute_dragon_pixels_match_oracle(cameras):
    """1 M triangles: the quad walk with the lowest-index tie rule, against the loop."""
    import scenes
    from oracle_bindings import OracleScene
    P = rt_amd.parse_obj(scenes.scene_path("dragon"))
    sky = scenes.make_sky("L")
    W, H = 1920, 1080
    rk = rt_amd.RenderKernel(W, H, 1, 8, rt_amd.Image(W, H), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky), None)
    rk.set_camera(rt_amd.Camera(cameras["dragon"][:16], cameras["dragon"][16]))
    rk.set_use_bvh(False)
    px = _pixels(W, H, 24)
    rk.ray_trace_pixels(px)
    got = rk.frame_buffer.pixels[px[:, 1], px[:, 0]]
    S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices, env=sky)
    S.set_use_bvh(False)
    want, _ = S.render(cameras["dragon"], W, H, 1, 8, pixels=px)
    assert (got.view(np.uint32) == want.view(np.uint32)).all()
