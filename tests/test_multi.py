"""One context over several devices (rt_create_multi: rows y -> device y mod N,
RCCL scatter / gather through the root, include/rt_hip.h) and the material
table pushed alone (rt_set_materials, the reference's by-reference
`std::vector<SimpleMaterial>&`, render_kernel.h:81-93).

CPU: the hostsim build shards the same way (host copies in place of RCCL), so
the row mapping is checked here against the reference's goldens. GPU: the
product's RCCL path (a one-device clique on a one-GPU box, a two-rank clique
on one device where RCCL allows it) and the cfg5 material sweep through one
context, against the compiled reference's goldens."""
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
def test_gpu_multi_context_one_device_matches_single(manifest, cameras):
    """The RCCL path (pack, ncclScatter, render, ncclGather, un-permute) on a
    one-device clique: frames and row shards bit-identical to the goldens and
    to the single-device context."""
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
    g = rt_cases.golden_case("cfg2_dragon", manifest)
    rk, fb = rt_cases.make_kernel(g, cameras, hostsim=False, device=[0])
    rk.ray_trace_pixels(g["px"])
    got = fb.pixels[g["px"][:, 1], g["px"][:, 0]]
    assert gio.compare_rgb(got, g["expected"])["bitwise_fraction"] == 1.0


@pytest.mark.gpu
def test_gpu_multi_context_two_ranks_one_device(manifest, cameras):
    """A two-rank RCCL clique on device 0 twice (skipped where RCCL refuses two
    ranks on one GPU): the N=2 scatter / gather and un-permute on one box."""
    e = rt_cases.golden_case("cornell32_128", manifest)
    try:
        rk, fb = rt_cases.make_kernel(e, cameras, hostsim=False, device=[0, 0])
    except rt_amd.RtError as err:
        pytest.skip(f"RCCL: two ranks on one device refused ({err})")
    rk.render()
    np.testing.assert_array_equal(_bits(fb.pixels), _bits(e["expected"]))


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
