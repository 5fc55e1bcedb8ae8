"""The product's device code (rt_trace.h: explicit-stack octree walk,
libstdc++ heap-order emulation, glibc-exact libm) compiled for the host
(librt_hostsim.so) against the reference's golden renders. This runs the
kernel's algorithm in a GPU-less container; the same source is compiled for
gfx950 into librt_hip.so and checked on the GPU by test_gpu_parity.py."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import golden_io as gio
import rt_cases
from conftest import load_golden, parsed_scene

import rt_amd
from rt_amd import _capi


@pytest.mark.parametrize("name", rt_cases.CORNELL_CASES)
def test_hostsim_render_bit_exact(name, manifest, cameras):
    e = rt_cases.golden_case(name, manifest)
    got = rt_cases.run_case(e, cameras, hostsim=True)
    assert gio.compare_rgb(got, e["expected"])["bitwise_fraction"] == 1.0


@pytest.mark.parametrize("spec_cam", [0, 2])
def test_hostsim_camera_ahead_policies_bit_exact(spec_cam, manifest, cameras):
    """The next sample's camera ray traced ahead never (0) or only where the pixel's
    previous sample ended (2, rt_wave.h next_camera): which rays are cast changes, the
    answers do not."""
    for name in rt_cases.CORNELL_CASES[:2]:
        e = rt_cases.golden_case(name, manifest)
        got = rt_cases.run_case(e, cameras, hostsim=True, schedule={"spec_cam": spec_cam})
        assert gio.compare_rgb(got, e["expected"])["bitwise_fraction"] == 1.0, name


def test_schedule_is_not_read_from_the_environment(manifest, cameras, monkeypatch):
    """Product hygiene: the test stressor that sends every k-th query to the exact
    walk is a test-only C entry (rt_test_schedule), not an environment variable, so a stray
    RT_FORCE_FALLBACK (or any other old schedule knob) in a user's environment changes nothing:
    the fallback count with it set equals the count without; through rt_test_schedule the count
    rises and the frame stays bitwise."""
    e = rt_cases.golden_case(rt_cases.CORNELL_CASES[0], manifest)

    def fallbacks(schedule=None):
        rk, fb = rt_cases.make_kernel(e, cameras, hostsim=True)
        rk.set_stats(True)
        if schedule:
            rk.test_schedule(**schedule)
        rk.render()
        assert gio.compare_rgb(fb.pixels, e["expected"])["bitwise_fraction"] == 1.0
        return rk.stats()["fallback"]

    base = fallbacks()
    for k, v in (("RT_FORCE_FALLBACK", "3"), ("RT_STEP_BUDGET", "1"), ("RT_SPEC_CAM", "0"), ("RT_TAIL_PATHS", "0"),
                 ("RT_LANES", "2"), ("RT_HEAVY", "1"), ("RT_DRAIN_ROWS", "0")):
        monkeypatch.setenv(k, v)
    assert fallbacks() == base
    assert fallbacks({"force_fallback": 3}) > base
    rk, _ = rt_cases.make_kernel(e, cameras, hostsim=True)
    with pytest.raises(rt_amd.RtError):
        rk.test_schedule(no_such_knob=1)


def test_schedule_keys(manifest, cameras):
    """Every rt_test_schedule key the tests and tools use (include/rt_hip.h) is
    accepted, `reset` restores the product schedule, and the frame is the same either way (the
    hostsim backend ignores the GPU-only keys: lanes, tail kernel, fast lane)."""
    e = rt_cases.golden_case(rt_cases.CORNELL_CASES[0], manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=True)
    rk.test_schedule(lanes=2, tail_paths=1, tail_enter=1.5, tail_rows=0, drain_rows=1, heavy_calls=0, spec_cam=2,
                     tail_spec_cam=1, force_fallback=0, step_budget=64, fast_k=512, fast_spp=1.0)
    rk.render()
    assert gio.compare_rgb(fb.pixels, e["expected"])["bitwise_fraction"] == 1.0
    rk2, fb2 = rt_cases.make_kernel(e, cameras, hostsim=True)  # (a render writes over a fresh frame)
    rk2.test_schedule(fast_k=7)
    rk2.test_schedule(reset=1)
    rk2.render()
    assert gio.compare_rgb(fb2.pixels, e["expected"])["bitwise_fraction"] == 1.0


@pytest.mark.slow
@pytest.mark.parametrize("name", ["cfg2_dragon", "cfg4_dragon4k", "cfg5_sweep_m0_r0", "cfg5_sweep_m3_r3"])
def test_hostsim_dragon_bit_exact(name, manifest, cameras):
    e = rt_cases.golden_case(name, manifest)
    if e["px"].shape[0] > 256:
        e["px"], e["expected"] = e["px"][:256], e["expected"][:256]
    got = rt_cases.run_case(e, cameras, hostsim=True)
    assert gio.compare_rgb(got, e["expected"])["bitwise_fraction"] == 1.0


@pytest.mark.parametrize("keys", [
    [1, 1, 1, 1, 1, 1, 1, 1], [2, 1, 2, 1, 2, 1, 2, 1], [0.5, 0.5, 0.25], [3, 2, 1, 2, 3], [1, 2], [7],
    [1, 0, 1, 0, 0, 1, 1], [4, 4, 3, 3, 2, 2], [0, -1, 0, -1, 5, 5, 5, -1],
])
def test_heap_order_matches_std_priority_queue(keys):
    """Equal-t child ordering = libstdc++ std::priority_queue pop order (bvh.h:170-199)."""
    L = _capi.lib(hostsim=True)
    k = np.asarray(keys, np.float32)
    a, b = np.zeros(len(keys), np.int32), np.zeros(len(keys), np.int32)
    assert L.rt_hostsim_heap_order(_capi.ptr(k), len(keys), _capi.ptr(a), _capi.ptr(b)) == 0
    np.testing.assert_array_equal(a, b)


def test_heap_order_random_ties():
    L = _capi.lib(hostsim=True)
    rng = np.random.default_rng(3)
    for _ in range(3000):
        m = int(rng.integers(1, 9))
        k = rng.integers(0, 3, m).astype(np.float32)
        a, b = np.zeros(m, np.int32), np.zeros(m, np.int32)
        L.rt_hostsim_heap_order(_capi.ptr(k), m, _capi.ptr(a), _capi.ptr(b))
        assert (a == b).all(), (k, a, b)


def test_hostsim_reference_bvh_regression_rays():
    """source/tests.cpp:16-58 vectors through the device traversal."""
    P = parsed_scene("cornell")
    sky = rt_amd.Image.from_rgb(rt_cases.sky("S"))
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles), sky, None, hostsim=True)
    g = load_golden("bvhtests_cornell.npz")
    for part, hits in (("inter", True), ("miss", False)):
        rec = g[part]
        out = rk.intersect(np.concatenate([rec["o"], rec["d"]], axis=1))
        assert (out[:, 0] == int(hits)).all()
        if hits:
            assert np.all(np.abs(out[:, 3:6].view(np.float32) - rec["expect"]) <= 1e-5)
            np.testing.assert_array_equal(out[:, 1], rec["bvh"]["prim"])
            np.testing.assert_array_equal(out[:, 2].view(np.float32), rec["bvh"]["t"])


def sphere_scene():
    """cornell12 + two analytic spheres (main.cpp:20-30 add_sphere_to_scene):
    each sphere appends a material and a material index; its primitive index
    is the next id after the triangles. Both are non-emissive: an emissive
    sphere hit by the BRDF-sampled light ray makes the reference read
    m_triangle_buffer[sphere prim] out of bounds (render_kernel.cpp:690-700,
    undefined behaviour), so no parity exists to pin there."""
    P = parsed_scene("cornell12")
    n = P.triangles.shape[0]
    mats = np.concatenate([P.materials, rt_amd.make_materials([((0, 0, 0), (0.9, 0.2, 0.2), 1.0, 0.3),
                                                                ((0, 0, 0), (1, 1, 1), 0.0, 0.6)])])
    mi = np.concatenate([P.material_indices, np.array([mats.shape[0] - 2, mats.shape[0] - 1], np.int32)])
    sph = np.array([[0.3, 0.35, 0.1, 0.3, n], [-0.4, 0.25, -0.2, 0.2, n + 1]], np.float32)
    return P, mats, mi, sph


def test_hostsim_spheres_match_oracle(cameras):
    from oracle_bindings import OracleScene
    P, mats, mi, sph = sphere_scene()
    sky = rt_cases.sky("S")
    S = OracleScene(P.triangles, mi, mats, P.emissive_triangle_indices, env=sky, spheres=sph)
    want, _ = S.render(cameras["cornell"], 96, 96, 4, 4)
    fb = rt_amd.Image(96, 96)
    rk = rt_amd.RenderKernel(96, 96, 4, 4, fb, P.triangles, mats, P.emissive_triangle_indices, mi, sph,
                             rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky), None, hostsim=True)
    c = cameras["cornell"]
    rk.set_camera(rt_amd.Camera(c[:16], c[16]))
    rk.render()
    assert gio.compare_rgb(fb.pixels, want)["bitwise_fraction"] == 1.0


def test_hostsim_row_shards_reassemble(manifest, cameras):
    """rt_render_device row shards (y = off + j*stride) are bit-identical to
    the corresponding rows of the full render (pixels are independent)."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    full = e["expected"]
    for stride in (2, 3):
        for off in range(stride):
            rk, _ = rt_cases.make_kernel(e, cameras, hostsim=True)
            rows = len(range(off, e["H"], stride))
            shard = np.zeros((rows, e["W"], 4), np.float32)
            shard[..., 3] = 1.0
            rk.render_device(shard.ctypes.data, off, stride)
            np.testing.assert_array_equal(shard.view(np.uint32), full[off::stride].view(np.uint32))


def test_hostsim_stats_counters(manifest, cameras):
    e = rt_cases.golden_case("cfg1_cornell12", manifest)
    rk, _ = rt_cases.make_kernel(e, cameras, hostsim=True)
    rk.set_stats(True)
    rk.render()
    s = rk.stats()
    samples = e["W"] * e["H"] * e["spp"]
    assert s["rays"] >= samples and s["vol"] >= s["rays"] and s["tri"] > 0
    assert s["any_rays"] > 0 and s["any_vol"] >= s["any_rays"]
    assert s["mat"] > 0 and s["cdf"] > 0


@pytest.mark.parametrize("scene,cam", [("cornell", "cornell"), ("mis", "mis"), ("cornell12", "cornell")])
def test_hostsim_random_configs_match_oracle(scene, cam, cameras):
    """Seeded small configs incl. 0 and 1 bounces, 1-pixel-wide images and
    H < 25 (where the reference's progress print divides by zero)."""
    from oracle_bindings import OracleScene
    rng = np.random.default_rng(hash(scene) % 1000)
    P = parsed_scene(scene)
    S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices, env=rt_cases.sky("S"))
    for W, H, spp, nb in [(1, 1, 3, 0), (5, 3, 2, 1), (17, 9, 3, 2)] + [
            (int(rng.integers(1, 60)), int(rng.integers(1, 40)), int(rng.integers(1, 6)), int(rng.integers(0, 10)))
            for _ in range(3)]:
        want, _ = S.render(cameras[cam], W, H, spp, nb)
        fb = rt_amd.Image(W, H)
        rk = rt_amd.RenderKernel(W, H, spp, nb, fb, P.triangles, P.materials, P.emissive_triangle_indices,
                                 P.material_indices, None, rt_amd.BVH(P.triangles),
                                 rt_amd.Image.from_rgb(rt_cases.sky("S")), None, hostsim=True)
        c = cameras[cam]
        rk.set_camera(rt_amd.Camera(c[:16], c[16]))
        rk.render()
        assert gio.compare_rgb(fb.pixels, want)["bitwise_fraction"] == 1.0, (W, H, spp, nb)


@pytest.mark.parametrize("n", [0, 1, 2, 5])
def test_hostsim_tiny_scenes_match_oracle(n, cameras):
    """Empty scene (sky only), one and two triangles, five (one leaf split)."""
    got, want = rt_cases.render_tiny(n, cameras, hostsim=True)
    assert gio.compare_rgb(got, want)["bitwise_fraction"] == 1.0


@pytest.mark.parametrize("fixture", ["rays_dragon.npz", "brute_rays_dragon_tie_prone.npz"])
def test_fast_walk_settles_same_leaf_ties_like_the_octree_walk(fixture):
    """The search-BVH walk's answer (rt_fast.h fast_query_closest, the k_trace stage) on
    tie-prone rays (rays through triangle edges and vertices of the reference-pinned
    fixtures): every ray it settles, including two triangles hit at exactly the same t inside
    one octree leaf (the first in that leaf's list wins, bvh.h:150-161), gives the exact octree
    walk's (t, triangle); only ties across leaves (and failed chain checks) are left to the
    exact walk."""
    P = parsed_scene("dragon")
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(np.ones((8, 16, 3), np.float32)), None, hostsim=True)
    g = load_golden(fixture)
    rays = np.ascontiguousarray((g["rays"] if "rays" in g else g[list(g.keys())[0]])[:, :6], dtype=np.float32)
    n = rays.shape[0]
    t = np.zeros(n, np.float32)
    k = np.zeros(n, np.int32)
    L = _capi.lib(hostsim=True)
    assert L.rt_hostsim_fast_queries(rk.ctx, _capi.ptr(rays), n, _capi.ptr(t), _capi.ptr(k)) == 0
    ex = rk.intersect(rays)
    ok = t != -2.0
    want_t = np.where(ex[:, 0] == 1, ex[:, 2].view(np.float32), -1.0).astype(np.float32)
    np.testing.assert_array_equal(t[ok].view(np.uint32), want_t[ok].view(np.uint32))
    hit = ok & (ex[:, 0] == 1)
    np.testing.assert_array_equal(k[hit], ex[hit, 1])
    assert ok.mean() > 0.95, f"{(~ok).sum()} of {n} left to the exact walk"
