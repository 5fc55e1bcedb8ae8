"""GPU parity: the product library librt_hip.so (gfx950 kernel) through the
C ABI against (1) the golden renders the compiled reference produced and (2)
the pinned CPU restatement oracle on the same seeded inputs.

Tolerance (BASELINE.json north_star): per-channel L-inf <= 1e-4 on the
tone-mapped RGB, NaN == NaN. The kernel is built to be bit-exact, so the
bitwise-identical fraction is also asserted (>= 0.9999)."""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np
import pytest

import golden_io as gio
import rt_cases
from conftest import load_golden, parsed_scene

import rt_amd
from rt_amd import _capi

pytestmark = pytest.mark.gpu
TOL = 1e-4


def assert_parity(got, want, min_bitwise=0.9999):
    c = gio.compare_rgb(got, want)
    print("parity", c)
    assert c["nan_mismatch"] == 0, c
    assert c["linf"] <= TOL, c
    assert c["pixels_over_1e4"] == 0, c
    assert c["bitwise_fraction"] >= min_bitwise, c


@pytest.mark.parametrize("name", rt_cases.CORNELL_CASES + rt_cases.DRAGON_CASES)
def test_gpu_matches_reference_goldens(name, manifest, cameras):
    e = rt_cases.golden_case(name, manifest)
    got = rt_cases.run_case(e, cameras, hostsim=False)
    assert_parity(got, e["expected"])


def test_gpu_cfg2_full_frame_rows_match_oracle(manifest, cameras):
    """Cfg2 (dragon, 1920x1080x64spp x8) rendered as a whole frame on the
    GPU; every 60th row is re-rendered by the oracle and compared."""
    e = rt_cases.golden_case("cfg2_dragon", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False)
    rk.render()
    rows = np.arange(7, e["H"], 60)
    xs, ys = np.meshgrid(np.arange(e["W"]), rows)
    e["px"] = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    want = rt_cases.run_oracle(e, cameras)
    assert_parity(fb.pixels[rows].reshape(-1, 4), want)
    # and the golden pixels
    g = rt_cases.golden_case("cfg2_dragon", manifest)
    assert_parity(fb.pixels[g["px"][:, 1], g["px"][:, 0]], g["expected"])


def test_gpu_row_shards_bit_identical(manifest, cameras):
    """rt_render_device row shards == rows of the full frame, bit for bit
    (the multi-GPU partition). Device memory comes straight
    from the HIP runtime (no torch in this process)."""
    from hip_mem import DeviceBuffer
    e = rt_cases.golden_case("cornell32_128", manifest)
    for stride in (2, 3, 8):
        for off in range(stride):
            rk, _ = rt_cases.make_kernel(e, cameras, hostsim=False)
            rows = len(range(off, e["H"], stride))
            init = np.zeros((rows, e["W"], 4), np.float32)
            init[..., 3] = 1.0
            buf = DeviceBuffer(init.nbytes)
            buf.upload(init)
            rk.render_device(buf.ptr, off, stride, None)
            got = buf.download(init.shape, np.float32)
            np.testing.assert_array_equal(got.view(np.uint32), e["expected"][off::stride].view(np.uint32))


def test_gpu_reference_bvh_regression_rays():
    """source/tests.cpp:16-58 / include/bvh_tests.h through the gfx950 traversal."""
    P = parsed_scene("cornell")
    sky = rt_amd.Image.from_rgb(rt_cases.sky("S"))
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles), sky, None)
    g = load_golden("bvhtests_cornell.npz")
    for part, hits in (("inter", True), ("miss", False)):
        rec = g[part]
        out = rk.intersect(np.concatenate([rec["o"], rec["d"]], axis=1))
        assert (out[:, 0] == int(hits)).all()
        if hits:
            assert np.all(np.abs(out[:, 3:6].view(np.float32) - rec["expect"]) <= 1e-5)
            np.testing.assert_array_equal(out[:, 1], rec["bvh"]["prim"])
            np.testing.assert_array_equal(out[:, 2].view(np.float32), rec["bvh"]["t"])


def test_gpu_dragon_rays_match_reference():
    P = parsed_scene("dragon")
    sky = rt_amd.Image.from_rgb(rt_cases.sky("S"))
    rk = rt_amd.RenderKernel(4, 4, 1, 1, rt_amd.Image(4, 4), P.triangles, P.materials, P.emissive_triangle_indices,
                             P.material_indices, None, rt_amd.BVH(P.triangles), sky, None)
    g = load_golden("rays_dragon.npz")
    out = rk.intersect(g["rays"])
    h = g["hits"]
    np.testing.assert_array_equal(out[:, 0], h["found"])
    hit = h["found"] == 1
    np.testing.assert_array_equal(out[hit, 1], h["prim"][hit])
    np.testing.assert_array_equal(out[hit, 2].view(np.float32), h["t"][hit])
    np.testing.assert_array_equal(out[hit, 3:6].view(np.float32), h["p"][hit])
    np.testing.assert_array_equal(out[hit, 6:9].view(np.float32), h["n"][hit])


def test_gpu_spheres_match_oracle(cameras):
    from oracle_bindings import OracleScene
    from test_hostsim import sphere_scene
    P, mats, mi, sph = sphere_scene()
    sky = rt_cases.sky("S")
    S = OracleScene(P.triangles, mi, mats, P.emissive_triangle_indices, env=sky, spheres=sph)
    want, _ = S.render(cameras["cornell"], 96, 96, 4, 4)
    fb = rt_amd.Image(96, 96)
    rk = rt_amd.RenderKernel(96, 96, 4, 4, fb, P.triangles, mats, P.emissive_triangle_indices, mi, sph,
                             rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky), None)
    c = cameras["cornell"]
    rk.set_camera(rt_amd.Camera(c[:16], c[16]))
    rk.render()
    assert_parity(fb.pixels, want, min_bitwise=1.0)


def test_gpu_random_configs_match_oracle(cameras):
    """Seeded sweep of small configs (sizes, spp, bounce counts incl. 0/1 and
    the H<25 case that crashes the reference's progress print) vs the oracle."""
    from oracle_bindings import OracleScene
    rng = np.random.default_rng(11)
    for scene, sky_kind, cam in (("cornell", "S", "cornell"), ("mis", "S", "mis"), ("cornell12", "S", "cornell")):
        P = parsed_scene(scene)
        S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices,
                        env=rt_cases.sky(sky_kind))
        for _ in range(3):
            W, H = int(rng.integers(1, 90)), int(rng.integers(1, 70))
            spp, nb = int(rng.integers(1, 9)), int(rng.integers(0, 10))
            want, _ = S.render(cameras[cam], W, H, spp, nb)
            fb = rt_amd.Image(W, H)
            rk = rt_amd.RenderKernel(W, H, spp, nb, fb, P.triangles, P.materials, P.emissive_triangle_indices,
                                     P.material_indices, None, rt_amd.BVH(P.triangles),
                                     rt_amd.Image.from_rgb(rt_cases.sky(sky_kind)), None)
            c = cameras[cam]
            rk.set_camera(rt_amd.Camera(c[:16], c[16]))
            rk.render()
            assert_parity(fb.pixels, want, min_bitwise=1.0)


@pytest.mark.gpu
def test_gpu_many_materials_match_oracle(cameras):
    """A material table larger than the shading kernels stage in LDS (> 64
    entries: the global-memory path): the Cornell box with its 9 materials
    repeated 9 times and triangle t using copy t % 9, against the oracle on
    the same buffers (and so the same image as the plain box)."""
    from oracle_bindings import OracleScene
    P = parsed_scene("cornell")
    k = 9
    nm = len(P.materials)
    mats = np.tile(P.materials, (k, 1))
    mi = (P.material_indices + nm * (np.arange(len(P.material_indices)) % k)).astype(P.material_indices.dtype)
    assert len(mats) > 64
    sky = rt_cases.sky("S")
    S = OracleScene(P.triangles, mi, mats, P.emissive_triangle_indices, env=sky)
    W, H, spp, nb = 96, 72, 4, 5
    want, _ = S.render(cameras["cornell"], W, H, spp, nb)
    fb = rt_amd.Image(W, H)
    rk = rt_amd.RenderKernel(W, H, spp, nb, fb, P.triangles, mats, P.emissive_triangle_indices, mi, None,
                             rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky), None)
    c = cameras["cornell"]
    rk.set_camera(rt_amd.Camera(c[:16], c[16]))
    rk.render()
    assert_parity(fb.pixels, want, min_bitwise=1.0)


# ------------------------------------------------------------ device libm
_FN = {0: "expf", 2: "sinf", 3: "cosf", 4: "acosf", 5: "asinf"}


def _glibc():
    m = ctypes.CDLL(ctypes.util.find_library("m"))
    for n in ("expf", "sinf", "cosf", "acosf", "asinf"):
        getattr(m, n).restype = ctypes.c_float
        getattr(m, n).argtypes = [ctypes.c_float]
    for n in ("powf", "atan2f"):
        getattr(m, n).restype = ctypes.c_float
        getattr(m, n).argtypes = [ctypes.c_float, ctypes.c_float]
    return m


def _inputs(fn, rng, n):
    if fn == 0:
        x = rng.uniform(-104, 89, n)
    elif fn in (2, 3):
        x = np.concatenate([rng.uniform(0, 2 * np.pi, n // 2), rng.uniform(-1e4, 1e4, n - n // 2)])
    else:
        x = rng.uniform(-1, 1, n)
    x = x.astype(np.float32)
    special = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3.14159265, 1.5707964],
                       np.float32)
    return np.concatenate([special, x])


@pytest.mark.parametrize("fn", sorted(_FN))
def test_gpu_libm_unary_matches_glibc(fn):
    """rt_libm.h on gfx950 == this image's glibc 2.35 float libm, bit for bit."""
    m = _glibc()
    f = getattr(m, _FN[fn])
    x = _inputs(fn, np.random.default_rng(fn), 20000)
    out = np.zeros_like(x)
    assert _capi.lib().rt_device_libm(0, fn, _capi.ptr(x), None, _capi.ptr(out), x.shape[0]) == 0
    want = np.array([f(float(v)) for v in x], np.float32)
    same = (out.view(np.uint32) == want.view(np.uint32)) | (np.isnan(out) & np.isnan(want))
    assert same.all(), (x[~same][:5], out[~same][:5], want[~same][:5])


@pytest.mark.parametrize("fn", [1, 6])
def test_gpu_libm_binary_matches_glibc(fn):
    m = _glibc()
    rng = np.random.default_rng(100 + fn)
    n = 20000
    if fn == 1:  # powf at the exponents the path uses: 5 (fresnel) and 1/2.2 (gamma)
        x = rng.uniform(0, 1.0, n).astype(np.float32)
        y = np.where(rng.random(n) < 0.5, np.float32(5.0), np.float32(1.0) / np.float32(2.2)).astype(np.float32)
        f = m.powf
    else:
        x = rng.uniform(-1, 1, n).astype(np.float32)
        y = rng.uniform(-1, 1, n).astype(np.float32)
        f = m.atan2f
    out = np.zeros_like(x)
    assert _capi.lib().rt_device_libm(0, fn, _capi.ptr(x), _capi.ptr(y), _capi.ptr(out), n) == 0
    want = np.array([f(float(a), float(b)) for a, b in zip(x, y)], np.float32)
    same = (out.view(np.uint32) == want.view(np.uint32)) | (np.isnan(out) & np.isnan(want))
    assert same.all()


def test_gpu_ieee_div_sqrt_f64():
    """IEEE f32 division / sqrt with denormals, and the f64 GGX path, on device."""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-10, 10, 5000), rng.uniform(0, 1e-36, 1000)]).astype(np.float32)
    y = np.concatenate([rng.uniform(-10, 10, 5000), rng.uniform(1, 1e3, 1000)]).astype(np.float32)
    L = _capi.lib()
    out = np.zeros_like(x)
    assert L.rt_device_libm(0, 8, _capi.ptr(x), _capi.ptr(y), _capi.ptr(out), x.shape[0]) == 0
    np.testing.assert_array_equal(out.view(np.uint32), (x / y).astype(np.float32).view(np.uint32))
    ax = np.abs(x)
    assert L.rt_device_libm(0, 7, _capi.ptr(ax), None, _capi.ptr(out), x.shape[0]) == 0
    np.testing.assert_array_equal(out.view(np.uint32), np.sqrt(ax).view(np.uint32))
    assert L.rt_device_libm(0, 9, _capi.ptr(x), _capi.ptr(y), _capi.ptr(out), x.shape[0]) == 0
    want = (x.astype(np.float64) * 0.31830988618379067154 / y.astype(np.float64)).astype(np.float32)
    np.testing.assert_array_equal(out.view(np.uint32), want.view(np.uint32))


def test_gpu_slab_division_exact():
    """The slab quotient (float)((double)a * (1.0/(double)den)) on gfx950 ==
    IEEE f32 a/den (the reference's division, bounding_volume.h:113-114)."""
    from test_numerics import division_cases
    a, d = division_cases(400000)
    out = np.zeros_like(a)
    assert _capi.lib().rt_device_libm(0, 10, _capi.ptr(a), _capi.ptr(d), _capi.ptr(out), a.shape[0]) == 0
    want = (a / d).astype(np.float32)
    same = (out.view(np.uint32) == want.view(np.uint32)) | (np.isnan(out) & np.isnan(want))
    assert same.all(), (a[~same][:4], d[~same][:4])


def test_gpu_schedules_bit_identical():
    """The frame does not depend on the schedule: 1-4 wavefront lanes, the
    tail kernel on or off (1-8 paths per wave, entered at once or late), quad or
    row walks (rt_row.h) in the tail kernel and in k_trace, row
    shards split across lanes (framebuffer row pitch), k_trace's heavy class
    (off, every walk heavy, the default), the camera ray traced ahead or not and
    the fast lane all give the same bits as one lane without the tail kernel."""
    import scenes
    from hip_mem import DeviceBuffer
    P = rt_amd.parse_obj(scenes.scene_path("dragon_small"))
    sky = scenes.make_sky("L")
    W, H, spp, nb = 640, 480, 2, 8

    def render(lanes, tail, off=0, stride=1, heavy=6, enter=2.0, spec_cam=1, rows=1, drain=4, tail_cam=0, fast_k=0,
               fast_spp=2.25):
        rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                                 P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                                 rt_amd.Image.from_rgb(sky), None, device=0)
        rk.test_schedule(lanes=lanes, tail_paths=tail, heavy_calls=heavy, tail_enter=enter, spec_cam=spec_cam,
                         tail_rows=rows, drain_rows=drain, tail_spec_cam=tail_cam, fast_k=fast_k, fast_spp=fast_spp)
        rk.set_camera(rt_amd.Camera.preset("dragon"))
        rows = len(range(off, H, stride))
        init = np.zeros((rows, W, 4), np.float32)
        init[..., 3] = 1.0
        buf = DeviceBuffer(init.nbytes)
        buf.upload(init)
        rk.render_device(buf.ptr, off, stride, None)
        return buf.download(init.shape, np.float32)

    base = render(1, 0)
    assert np.isfinite(base[..., :3]).any()
    for lanes, tail in ((2, 4), (3, 4), (4, 8), (3, 0)):
        got = render(lanes, tail)
        np.testing.assert_array_equal(got.view(np.uint32), base.view(np.uint32), err_msg=f"lanes={lanes} tail={tail}")
    for off in (0, 1):
        got = render(3, 4, off, 2)
        np.testing.assert_array_equal(got.view(np.uint32), base[off::2].view(np.uint32), err_msg=f"shard {off}/2")
    for heavy in (0, 1):  # heavy class off / every path's rays in the heavy shards
        got = render(3, 4, heavy=heavy)
        np.testing.assert_array_equal(got.view(np.uint32), base.view(np.uint32), err_msg=f"heavy={heavy}")
    # the tail kernel entered at once (it takes nearly every path, its waves refilling from
    # the live list) with 1 and 2 paths per wave; the next camera ray not traced ahead
    for lanes, tail, enter in ((3, 1, 1000.0), (2, 2, 1000.0), (1, 2, 1000.0)):
        got = render(lanes, tail, enter=enter)
        np.testing.assert_array_equal(got.view(np.uint32), base.view(np.uint32),
                                      err_msg=f"lanes={lanes} tail={tail} enter={enter}")
    # camera rays traced ahead: never, only where the pixel's previous sample ended (2), and the
    # tail kernel's own mode
    for lanes, tail, spec_cam, tail_cam in ((1, 0, 0, 0), (3, 2, 0, 0), (1, 0, 2, 0), (3, 1, 2, 2), (3, 1, 1, 1),
                                            (3, 1, 1, 2)):
        got = render(lanes, tail, spec_cam=spec_cam, tail_cam=tail_cam)
        np.testing.assert_array_equal(got.view(np.uint32), base.view(np.uint32),
                                      err_msg=f"spec_cam={spec_cam} tail_cam={tail_cam} lanes={lanes}")
    # the walks by quads or by rows (rt_row.h) in the tail kernel (and a k_trace drain continuing
    # its quad walks as rows, or not; 1 walk at most, or 4)
    for rows, tail, enter, drain in ((0, 2, 2.0, 0), (1, 1, 1000.0, 1), (1, 1, 2.0, 4), (0, 4, 2.0, 0), (1, 0, 2.0, 4),
                                     (1, 0, 2.0, 1)):
        got = render(3, tail, enter=enter, rows=rows, drain=drain)
        np.testing.assert_array_equal(got.view(np.uint32), base.view(np.uint32),
                                      err_msg=f"rows={rows} tail={tail} drain={drain}")
    # the fast lane: the slowest paths of every lane handed to one tail kernel on a stream of its
    # own (a few, or most of the paths; early or late; with 1, 3 and 4 lanes; with and without the
    # lanes' own tail kernel), the rest still in the wavefront; and the product's default
    for lanes, tail, fast_k, fast_spp in ((1, 1, 64, 0.0), (3, 1, 768, 2.25), (4, 1, 4096, 0.5), (3, 0, 256, 1.0),
                                          (2, 2, 100000, 0.0), (0, -1, -1, -1.0)):
        got = render(lanes, tail, fast_k=fast_k, fast_spp=fast_spp)
        np.testing.assert_array_equal(got.view(np.uint32), base.view(np.uint32),
                                      err_msg=f"fast_k={fast_k} fast_spp={fast_spp} lanes={lanes} tail={tail}")


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 2, 5])
def test_gpu_tiny_scenes_match_oracle(n, cameras):
    """Empty scene (sky only), one and two triangles, five (one leaf split):
    the degenerate search-BVH and octree shapes through the gfx950 kernels."""
    got, want = rt_cases.render_tiny(n, cameras, hostsim=False)
    assert_parity(got, want, min_bitwise=1.0)


@pytest.mark.parametrize("tail", ["0", "5"])
@pytest.mark.parametrize("name,budget,every", [("mis_512", 1, 7), ("cornell32_128", 1, 7), ("cfg2_dragon", 8, 31)])
def test_gpu_parked_walks_small_launches(name, budget, every, tail, manifest, cameras):
    """Exact-walk hand-off under stress: every `every`-th query (by
    a hash of its ray, rt_test_schedule force_fallback) skips the quad walk for the exact
    octree walk, a step budget of 1 (8 on the dragon, whose walks take ~200
    steps: each park costs an iteration) parks those walks at node
    boundaries, and with the tail kernel off the last iterations run k_step on
    a live count of a few paths while fallbacks and parked walks are pending
    (with it on, k_tail walks them inline). Every pixel must still be written,
    bit for bit the reference's."""
    e = rt_cases.golden_case(name, manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False)
    rk.test_schedule(step_budget=budget, tail_paths=int(tail), force_fallback=every)
    rk.set_stats(True)
    if e.get("px") is None:
        rk.render()
        got = fb.pixels
    else:
        rk.ray_trace_pixels(e["px"])
        got = fb.pixels[e["px"][:, 1], e["px"][:, 0]]
    st = rk.stats()
    print(name, "fallbacks", st["fallback"], "in k_tail", st["tail_fallback"], "iterations", rk.last_iterations())
    assert st["fallback"] > 0
    assert_parity(got, e["expected"], min_bitwise=1.0)


def test_gpu_exact_handovers_are_rare(manifest, cameras):
    """The search-BVH walks' health in the product's timed kernels (not the stats variant):
    queries k_trace hands to the exact octree walk (rt_device_exact_handovers) stay at the
    ~1e-6-per-sample level of ties on the dragon (a walk that went wrong, e.g. a corrupted
    stack, still renders the reference's image through the exact walk, only slower: this is
    where it shows), and the counter does count: the force_fallback stressor raises it."""
    e = rt_cases.golden_case("cfg2_dragon", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False, W=480, H=270, spp=8)
    samples = 480 * 270 * 8
    rk.render()
    rk.exact_handovers(reset=True)
    rk.render()
    ho = rk.exact_handovers()
    print("hand-overs", ho, "per sample", ho / samples)
    assert ho <= 1e-4 * samples
    rk.test_schedule(force_fallback=64)
    rk.exact_handovers(reset=True)
    rk.render()
    forced = rk.exact_handovers(reset=True)
    print("forced hand-overs", forced)
    assert forced > 0.01 * samples


@pytest.mark.parametrize("name,off,stride", [("cfg3_dragon", 311, 400), ("cfg4_dragon4k", 1083, 1100)])
def test_gpu_full_rows_at_256spp_match_oracle(name, off, stride, manifest, cameras):
    """Cfg3 (1080p) and Cfg4 (4K) at their full 256 spp: whole image rows
    rendered as a row shard on the GPU (rt_render_device, rows off + j*stride)
    against the oracle on the same rows."""
    from hip_mem import DeviceBuffer
    e = rt_cases.golden_case(name, manifest)
    rk, _ = rt_cases.make_kernel(e, cameras, hostsim=False)
    rows = np.arange(off, e["H"], stride)
    init = np.zeros((rows.size, e["W"], 4), np.float32)
    init[..., 3] = 1.0
    buf = DeviceBuffer(init.nbytes)
    buf.upload(init)
    rk.render_device(buf.ptr, off, stride, None)
    got = buf.download(init.shape, np.float32)
    xs, ys = np.meshgrid(np.arange(e["W"]), rows)
    e["px"] = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    want = rt_cases.run_oracle(e, cameras)
    assert_parity(got.reshape(-1, 4), want, min_bitwise=1.0)


def test_gpu_cfg4_full_frame_rows_match_oracle(manifest, cameras):
    """Cfg4 (4K x 256 spp x 8, the 8-GPU config) rendered as one whole frame on the GPU
    (the 1-GPU leg of bench.py's strong_cfg4): four rows spread over the frame against
    the oracle, bitwise, and every golden pixel of the compiled reference."""
    e = rt_cases.golden_case("cfg4_dragon4k", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False)
    rk.render()
    rows = np.arange(137, e["H"], 540)
    xs, ys = np.meshgrid(np.arange(e["W"]), rows)
    o = dict(e)
    o["px"] = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    want = rt_cases.run_oracle(o, cameras)
    assert_parity(fb.pixels[rows].reshape(-1, 4), want, min_bitwise=1.0)
    assert_parity(fb.pixels[e["px"][:, 1], e["px"][:, 0]], e["expected"], min_bitwise=1.0)


@pytest.mark.parametrize("variant", ["cfg5_sweep_m0_r0", "cfg5_sweep_m3_r3"])
def test_gpu_cfg5_variant_row_matches_oracle(variant, manifest, cameras):
    """Two cfg5 sweep variants at their full 1024 spp (the smoothest dielectric and the
    roughest metal of the grid): a whole image row through the dragon, rendered as
    a row shard on the GPU, against the oracle with the variant's material table."""
    from hip_mem import DeviceBuffer
    e = rt_cases.golden_case(variant, manifest)
    rk, _ = rt_cases.make_kernel(e, cameras, hostsim=False)
    off, stride = 700, e["H"]  # (one row)
    init = np.zeros((1, e["W"], 4), np.float32)
    init[..., 3] = 1.0
    buf = DeviceBuffer(init.nbytes)
    buf.upload(init)
    rk.render_device(buf.ptr, off, stride, None)
    got = buf.download(init.shape, np.float32)
    o = dict(e)
    o["px"] = np.stack([np.arange(e["W"]), np.full(e["W"], off)], 1).astype(np.int32)
    want = rt_cases.run_oracle(o, cameras)
    assert_parity(got.reshape(-1, 4), want, min_bitwise=1.0)
