"""USE_BVH 0 (render_kernel.h:13): INTERSECT_SCENE as the brute-force loop
(render_kernel.cpp:453-483 — closest by strict `<` in buffer order, the
lowest index wins a tie). The reference's build fixes USE_BVH 1 in its header,
so this mode is checked against the oracle's restatement of the loop (parity
pinned to the reference's code only through that restatement). Host (hostsim)
and gfx950 (gpu marker) variants."""
from __future__ import annotations

import numpy as np
import pytest

import rt_cases
from conftest import parsed_scene

import rt_amd


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
