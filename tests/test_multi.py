"""One context over several devices (rt_create_multi: rows y -> device y mod N,
RCCL scatter / gather through the root, include/rt_hip.h) and the material
table pushed alone (rt_set_materials, the reference's by-reference
`std::vector<SimpleMaterial>&`, render_kernel.h:81-93).

CPU: the hostsim build shards the same way (one host thread per device, host
copies in place of RCCL), so the row mapping, the per-device error collection
and recovery are checked here against the reference's goldens. GPU: the
multi-device driver on one GPU through its loopback exchange (rt_create_multi_loopback,
a test-only entry: device copies in place of RCCL, which needs distinct GPUs) and the cfg5 material
sweep through one context, against the compiled reference's goldens. The RCCL
scatter / gather itself runs only on a node with two or more GPUs (bench.py
--gpus N, the driver's scaling runs)."""
from __future__ import annotations

import numpy as np
import pytest

import golden_io as gio
import rt_cases
from conftest import parsed_scene

import rt_amd


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("n", [2, 3, 5])
def test_hostsim_multi_device_frame_matches_golden(n, manifest, cameras):
    e = rt_cases.golden_case("cornell32_128", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=True, device=list(range(n)))
    assert rk.n_devices == n
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))


@pytest.mark.parametrize("n,off,stride", [(2, 0, 1), (3, 1, 2), (4, 2, 3)])
def test_hostsim_multi_device_shard_matches_golden(n, off, stride, manifest, cameras):
    """rt_render_device of a row shard on an N-device context: the shard's rows
    split again over the devices and come back in shard order."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    rk, _ = rt_cases.make_kernel(e, cameras, hostsim=True, device=list(range(n)))
    rows = len(range(off, e["H"], stride))
    shard = np.zeros((rows, e["W"], 4), np.float32)
    shard[..., 3] = 1.0
    rk.render_device(shard.ctypes.data, off, stride, None)  # hostsim: a host pointer
    np.testing.assert_array_equal(_bits(shard), _bits(e["expected"][off::stride]))


@pytest.mark.parametrize("bad", [1, 2])
def test_hostsim_multi_device_failure_surfaces_and_recovers(bad, manifest, cameras):
    """A device >= 1 failing inside a multi-device render (rt_test_fail_device, tests only):
    the render returns its error code with the device's message (collected in the
    device thread's own slot, raised once after the join), and the next render on
    the same context succeeds bit for bit."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=True, device=[0, 1, 2])
    rk.test_fail_device(bad)
    with pytest.raises(rt_amd.RtError) as ei:
        rk.render()
    assert f"({rt_amd.RT_ERR_STATE})" in str(ei.value) and f"device {bad}: injected failure" in str(ei.value)
    rk.test_fail_device(-1)
    fb.pixels[...] = rt_amd.Image(e["W"], e["H"]).pixels
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))


def test_create_multi_device_ids(monkeypatch):
    """rt_create_multi: a device listed twice or a negative id is RT_ERR_ARG (an
    environment variable cannot turn the check off: the loopback form is its own
    test-only entry); one listed device is a single-device context on that ordinal
    (nothing to shard, no RCCL)."""
    import ctypes
    from rt_amd._capi import lib
    L = lib(hostsim=True)
    h = ctypes.c_void_p()
    monkeypatch.setenv("RT_MULTI_LOOPBACK", "1")  # (the round-3 knob: no longer read)
    for ids in ([0, 0], [1, 2, 1], [-1, 0]):
        a = np.asarray(ids, np.int32)
        assert L.rt_create_multi(len(ids), a.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)) == rt_amd.RT_ERR_ARG
        assert not h.value
    a = np.asarray([3], np.int32)
    assert L.rt_create_multi(1, a.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)) == 0
    assert L.rt_device_count(h) == 1
    L.rt_destroy(h)
    a = np.asarray([-1, 0], np.int32)
    assert L.rt_create_multi_loopback(2, a.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)) == rt_amd.RT_ERR_ARG
    a = np.asarray([0, 0], np.int32)
    assert L.rt_create_multi_loopback(2, a.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)) == 0
    assert L.rt_device_count(h) == 2
    L.rt_destroy(h)


def test_hostsim_materials_edited_in_place(manifest, cameras):
    """Editing the bound material array between renders changes the next
    render exactly as a fresh kernel with the new table would."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    P = parsed_scene(e["scene"])
    mats = P.materials.copy()
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=True, materials=mats)
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))
    mats[1:, 8] = np.float32(0.75)  # metalness
    mats[1:, 9] = np.float32(0.2)   # roughness
    fb.pixels[...] = rt_amd.Image(e["W"], e["H"]).pixels
    rk.render()
    rk2, fb2 = rt_cases.make_kernel(e, cameras, hostsim=True, materials=mats.copy())
    rk2.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(fb2.pixels))
    assert not np.array_equal(_bits(fb.pixels), _bits(e["expected"]))


def test_set_materials_rejects_short_table(manifest, cameras):
    e = rt_cases.golden_case("cornell32_128", manifest)
    rk, _ = rt_cases.make_kernel(e, cameras, hostsim=True)
    with pytest.raises(rt_amd.RtError):
        rk.set_materials(parsed_scene(e["scene"]).materials[:1])


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_multi_context_one_device_is_single(manifest, cameras):
    """device=[0]: one listed device is a single-device context on it (no RCCL);
    frames and row shards bit-identical to the goldens."""
    from hip_mem import DeviceBuffer
    e = rt_cases.golden_case("cornell32_128", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False, device=[0])
    assert rk.n_devices == 1
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))
    for off, stride in ((0, 1), (1, 3)):
        rows = len(range(off, e["H"], stride))
        init = np.zeros((rows, e["W"], 4), np.float32)
        init[..., 3] = 1.0
        buf = DeviceBuffer(init.nbytes)
        buf.upload(init)
        rk.render_device(buf.ptr, off, stride, None)
        got = buf.download(init.shape, np.float32)
        np.testing.assert_array_equal(_bits(got), _bits(e["expected"][off::stride]))


@pytest.mark.gpu
def test_gpu_multi_device_driver_rccl_one_rank(manifest, cameras):
    """The RCCL path itself on one GPU (rt_test_create_multi_rccl([0]): a one-rank
    ncclCommInitAll clique): render_multi's pack, ncclScatter of the caller's framebuffer
    rows, the device's wavefront loop into its block, ncclGather back to the root and the
    un-permute (render_kernel.cpp:169-180, 189-211), bit-identical to the goldens for the
    Cornell frame and row shards, and to the single-device context for a dragon row shard."""
    from hip_mem import DeviceBuffer
    e = rt_cases.golden_case("cornell32_128", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False, device=[0], rccl_clique=True)
    assert rk.n_devices == 1
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))
    for off, stride in ((0, 1), (1, 3)):
        rows = len(range(off, e["H"], stride))
        init = np.zeros((rows, e["W"], 4), np.float32)
        init[..., 3] = 1.0
        buf = DeviceBuffer(init.nbytes)
        buf.upload(init)
        rk.render_device(buf.ptr, off, stride, None)
        got = buf.download(init.shape, np.float32)
        np.testing.assert_array_equal(_bits(got), _bits(e["expected"][off::stride]))
    c1 = rt_cases.golden_case("cfg1_cornell12", manifest)
    rk1, fb1 = rt_cases.make_kernel(c1, cameras, hostsim=False, device=[0], rccl_clique=True)
    rk1.render()
    np.testing.assert_array_equal(_bits(fb1.pixels), _bits(c1["expected"]))
    g = rt_cases.golden_case("cfg2_dragon", manifest)
    rkr, _ = rt_cases.make_kernel(g, cameras, hostsim=False, device=[0], spp=4, rccl_clique=True)
    rks, _ = rt_cases.make_kernel(g, cameras, hostsim=False, device=0, spp=4)
    outs = []
    for k in (rkr, rks):
        rows = len(range(3, g["H"], 5))
        init = np.zeros((rows, g["W"], 4), np.float32)
        buf = DeviceBuffer(init.nbytes)
        buf.upload(init)
        k.render_device(buf.ptr, 3, 5, None)
        outs.append(buf.download(init.shape, np.float32))
    np.testing.assert_array_equal(_bits(outs[0]), _bits(outs[1]))


@pytest.mark.gpu
@pytest.mark.parametrize("ids", [[0, 0], [0, 0, 0]])
def test_gpu_multi_device_driver_loopback(ids, manifest, cameras):
    """The multi-device driver on one GPU (rt_create_multi_loopback: the device list may name
    GPU 0 repeatedly; the shards are exchanged with device copies instead of RCCL):
    the row pack, one host thread and stream per device running its own wavefront
    loop, the block exchange and the un-permute, bit-identical to the goldens for
    frames, row shards and the dragon; then a device failure (rt_test_fail_device) surfaces
    and the context renders correctly again."""
    from hip_mem import DeviceBuffer
    e = rt_cases.golden_case("cornell32_128", manifest)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False, device=ids, loopback=True)
    assert rk.n_devices == len(ids)
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))
    for off, stride in ((0, 1), (1, 3)):
        rows = len(range(off, e["H"], stride))
        init = np.zeros((rows, e["W"], 4), np.float32)
        init[..., 3] = 1.0
        buf = DeviceBuffer(init.nbytes)
        buf.upload(init)
        rk.render_device(buf.ptr, off, stride, None)
        got = buf.download(init.shape, np.float32)
        np.testing.assert_array_equal(_bits(got), _bits(e["expected"][off::stride]))
    rk.test_fail_device(len(ids) - 1)
    fb.pixels[...] = rt_amd.Image(e["W"], e["H"]).pixels
    with pytest.raises(rt_amd.RtError) as ei:
        rk.render()
    assert f"device {len(ids) - 1}: injected failure" in str(ei.value)
    rk.test_fail_device(-1)
    fb.pixels[...] = rt_amd.Image(e["W"], e["H"]).pixels
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))
    # a dragon frame's row shard (cfg2 rows at 4 spp) against the single-device context
    g = rt_cases.golden_case("cfg2_dragon", manifest)
    rk2, _ = rt_cases.make_kernel(g, cameras, hostsim=False, device=ids, spp=4, loopback=True)
    rk1, _ = rt_cases.make_kernel(g, cameras, hostsim=False, device=0, spp=4)
    outs = []
    for k in (rk2, rk1):
        rows = len(range(3, g["H"], 5))
        init = np.zeros((rows, g["W"], 4), np.float32)
        buf = DeviceBuffer(init.nbytes)
        buf.upload(init)
        k.render_device(buf.ptr, 3, 5, None)
        outs.append(buf.download(init.shape, np.float32))
    np.testing.assert_array_equal(_bits(outs[0]), _bits(outs[1]))


@pytest.mark.gpu
def test_gpu_cfg5_sweep_one_context(manifest, cameras):
    """The 16 cfg5 material variants through ONE context (one octree / BVH
    build): the material table is edited in place between renders, and every
    variant's pixels match the compiled reference's goldens bit for bit."""
    first = rt_cases.golden_case("cfg5_sweep_m0_r0", manifest)
    P = parsed_scene(first["scene"])
    mats = P.materials.copy()
    rk, fb = rt_cases.make_kernel(first, cameras, hostsim=False, materials=mats)
    for m in range(4):
        for r in range(4):
            e = rt_cases.golden_case(f"cfg5_sweep_m{m}_r{r}", manifest)
            mats[...] = rt_cases.materials_for(e, P)
            fb.pixels[...] = rt_amd.Image(e["W"], e["H"]).pixels
            rk.ray_trace_pixels(e["px"])
            got = fb.pixels[e["px"][:, 1], e["px"][:, 0]]
            c = gio.compare_rgb(got, e["expected"])
            assert c["bitwise_fraction"] == 1.0, (m, r, c)


@pytest.mark.gpu
def test_gpu_materials_edit_between_async_renders(manifest, cameras):
    """render_device returns before its kernels finish (non-blocking lane streams); a
    material edit pushed right after must not reach the table the running frame reads:
    render_device, set_materials, render_device with no sync in between, then each
    frame against a synchronous render of its own table."""
    from hip_mem import DeviceBuffer
    g = rt_cases.golden_case("cfg2_dragon", manifest)
    P = parsed_scene(g["scene"])
    mats = P.materials.copy()
    rk, _ = rt_cases.make_kernel(g, cameras, hostsim=False, spp=4, materials=mats)
    mats2 = mats.copy()
    mats2[1, 8], mats2[1, 9] = np.float32(1.0), np.float32(0.05)  # the dragon: polished metal
    H, W = g["H"], g["W"]
    init = np.zeros((H, W, 4), np.float32)
    bufs = [DeviceBuffer(init.nbytes), DeviceBuffer(init.nbytes)]
    for b in bufs:
        b.upload(init)
    rk.render_device(bufs[0].ptr, 0, 1, None)
    mats[...] = mats2  # in place, as the reference's by-reference vector (render_kernel.h:81-93)
    rk.render_device(bufs[1].ptr, 0, 1, None)
    got = [b.download(init.shape, np.float32) for b in bufs]
    for m, frame in ((P.materials, got[0]), (mats2, got[1])):
        ref, _ = rt_cases.make_kernel(g, cameras, hostsim=False, spp=4, materials=m.copy())
        b = DeviceBuffer(init.nbytes)
        b.upload(init)
        ref.render_device(b.ptr, 0, 1, None)
        np.testing.assert_array_equal(_bits(frame), _bits(b.download(init.shape, np.float32)))
    assert not np.array_equal(_bits(got[0]), _bits(got[1]))


# ---------------------------------------------- the material sweep as replicas
def _variant_tables(P, n=4):
    """n Cook-Torrance variants of every material (metalness x roughness grid, cfg5-style)."""
    out = []
    for v in range(n):
        m = P.materials.copy()
        m[:, 8] = np.float32([0.0, 1.0 / 3.0, 2.0 / 3.0, 1.0][v % 4])
        m[:, 9] = np.float32([0.05, 0.25, 0.5, 1.0][(v // 4 + v) % 4])
        out.append(m)
    return out


@pytest.mark.parametrize("devices", [0, [0, 1], [0, 1, 2]])
def test_hostsim_render_variants_match_single_renders(devices, manifest, cameras):
    """rt_render_variants (variant v on device v mod N, no exchange): every variant's
    frame equals a render of a fresh context built with that table; the bound table
    is what the next plain render uses."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    P = parsed_scene(e["scene"])
    tabs = _variant_tables(P, 5)
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=True, device=devices, W=48, H=40)
    frames = rk.render_variants(tabs)
    for v, m in enumerate(tabs):
        ref, rfb = rt_cases.make_kernel(e, cameras, hostsim=True, W=48, H=40, materials=m.copy())
        ref.render()
        np.testing.assert_array_equal(_bits(frames[v]), _bits(rfb.pixels))
    # a row shard of every variant
    shards = rk.render_variants(tabs[:3], row_offset=1, row_stride=3)
    np.testing.assert_array_equal(_bits(shards), _bits(frames[:3, 1::3]))
    rk.render()  # the bound table again
    ref, rfb = rt_cases.make_kernel(e, cameras, hostsim=True, W=48, H=40)
    ref.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(rfb.pixels))


def test_render_variants_rejects_bad_arguments(manifest, cameras):
    e = rt_cases.golden_case("cornell32_128", manifest)
    P = parsed_scene(e["scene"])
    rk, _ = rt_cases.make_kernel(e, cameras, hostsim=True, W=16, H=16)
    with pytest.raises(rt_amd.RtError):
        rk.render_variants([P.materials[:1]])  # a material index out of range
    with pytest.raises(rt_amd.RtError):
        rk.render_variants([P.materials], row_offset=2, row_stride=2)


# golden pixels of every cfg5 variant on rows 1, 540, 1079 (sample_pixels' fixed set)
CFG5_ROWS = (1, 539)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [0, [0, 0]])
def test_gpu_cfg5_variants_replicas_match_goldens(devices, manifest, cameras):
    """BASELINE config 5 as replicas: the 16 material variants in one rt_render_variants
    call (rows 1, 540, 1079 of each 1920x1080x1024spp frame), against the compiled
    reference's goldens on every golden pixel of those rows, host and device outputs;
    [0, 0]: two replica devices on one GPU (rt_create_multi_loopback), variants alternating."""
    from hip_mem import DeviceBuffer
    cases = [rt_cases.golden_case(f"cfg5_sweep_m{m}_r{r}", manifest) for m in range(4) for r in range(4)]
    P = parsed_scene(cases[0]["scene"])
    tabs = [rt_cases.materials_for(e, P) for e in cases]
    rk, _ = rt_cases.make_kernel(cases[0], cameras, hostsim=False, device=devices,
                                 loopback=isinstance(devices, list))
    off, stride = CFG5_ROWS
    rows = list(range(off, cases[0]["H"], stride))
    frames = rk.render_variants(tabs, row_offset=off, row_stride=stride)
    checked = 0
    for v, e in enumerate(cases):
        for (x, y), want in zip(e["px"], e["expected"]):
            if y in rows:
                got = frames[v, rows.index(y), x]
                assert (got.view(np.uint32)[:3] == want.view(np.uint32)[:3]).all(), (v, x, y, got, want)
                checked += 1
    assert checked >= 16 * 5
    # device outputs: the same bits
    init = np.zeros((len(rows), cases[0]["W"], 4), np.float32)
    init[..., 3] = 1.0
    bufs = [DeviceBuffer(init.nbytes) for _ in tabs]
    for b in bufs:
        b.upload(init)
    rk.render_variants(tabs, device_ptrs=[b.ptr for b in bufs], row_offset=off, row_stride=stride)
    for v, b in enumerate(bufs):
        np.testing.assert_array_equal(_bits(b.download(init.shape, np.float32)), _bits(frames[v]))


def test_hostsim_render_variants_stats_cover_every_variant(manifest, cameras):
    """rt_get_stats after rt_render_variants holds every variant's counters (summed over
    variants and devices), not only the last variant's."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    P = parsed_scene(e["scene"])
    tabs = _variant_tables(P, 3)
    per = []
    for m in tabs:
        ref, _ = rt_cases.make_kernel(e, cameras, hostsim=True, W=24, H=20, materials=m.copy())
        ref.set_stats(True)
        ref.render()
        per.append(ref.stats())
    for devices in (0, [0, 1]):
        rk, _ = rt_cases.make_kernel(e, cameras, hostsim=True, device=devices, W=24, H=20)
        rk.set_stats(True)
        rk.render_variants(tabs)
        got = rk.stats()
        for k in ("rays", "any_rays", "steps", "mat"):
            assert got[k] == sum(s[k] for s in per), (devices, k, got[k], [s[k] for s in per])


@pytest.mark.gpu
def test_gpu_render_after_variants_keeps_bound_table(manifest, cameras):
    """render, rt_render_variants with tables LONGER than the bound one (more materials:
    the n_mats / LDS material staging paths), render again: the two plain renders are
    bitwise equal, and each variant equals a fresh context built with its table."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    P = parsed_scene(e["scene"])
    W, H = 48, 40
    rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False, W=W, H=H)
    rk.render()
    first = fb.pixels.copy()
    extra = np.repeat(P.materials[-1:], 70, axis=0)  # 70 unused materials: > the 64-entry LDS table
    tabs = [np.concatenate([m, extra]) for m in _variant_tables(P, 3)]
    frames = rk.render_variants(tabs)
    for v, m in enumerate(tabs):
        ref, rfb = rt_cases.make_kernel(e, cameras, hostsim=False, W=W, H=H, materials=m.copy())
        ref.render()
        np.testing.assert_array_equal(_bits(frames[v]), _bits(rfb.pixels))
    fb.pixels[...] = rt_amd.Image(W, H).pixels
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(first))
