"""Render cases shared by the parity tests: the golden fixtures written by
the compiled reference (tools/gen_golden.py, tests/golden/manifest.json) and
helpers to run the same case through the product (gfx950), the hostsim build
of the product's device code, or the CPU restatement oracle."""
from __future__ import annotations

import numpy as np

import scenes
from conftest import load_golden, parsed_scene

import rt_amd

_sky = {}


def sky(kind: str) -> np.ndarray:
    if kind not in _sky:
        _sky[kind] = scenes.make_sky(kind)
    return _sky[kind]


def materials_for(entry: dict, P) -> np.ndarray:
    mats = P.materials.copy()
    mo = entry.get("mat_override")
    if mo:
        mats[mo["index"], 8] = np.float32(repr(mo["metalness"]))
        mats[mo["index"], 9] = np.float32(repr(mo["roughness"]))
    return mats


def sphere_buffers(entry: dict, P, mats: np.ndarray):
    """(materials, material_indices, spheres) with the entry's analytic spheres
    added the way main.cpp:20-30 add_sphere_to_scene does: each sphere's
    material appended to the materials, its material index to the material
    indices, primitive index = triangle count + k (gen_golden.py, ref_driver)."""
    sph = entry.get("spheres")
    if not sph:
        return mats, P.material_indices, None
    sph = np.asarray(sph, np.float32).reshape(-1, 12)
    n_tris = P.triangles.shape[0]
    new_mats = [mats]
    mi = [P.material_indices]
    spheres = np.zeros((sph.shape[0], 5), np.float32)
    for k, row in enumerate(sph):
        m = np.zeros((1, 10), np.float32)
        m[0, 0:3] = row[4:7]          # emission (alpha 1: Color(r, g, b))
        m[0, 3] = 1.0
        m[0, 4:7] = row[7:10]         # diffuse
        m[0, 7] = 1.0
        m[0, 8], m[0, 9] = row[10], row[11]
        mi.append(np.array([mats.shape[0] + k], np.int32))
        new_mats.append(m)
        spheres[k, :4] = row[:4]
        spheres[k, 4] = n_tris + k
    return np.concatenate(new_mats), np.concatenate(mi).astype(np.int32), spheres


def golden_case(name: str, manifest: dict) -> dict:
    e = dict(manifest["renders"][name])
    g = load_golden(f"render_{name}.npz")
    e["name"] = name
    e["expected"] = g["rgba"]
    e["px"] = g.get("px")
    return e


def make_kernel(entry: dict, cameras: dict, hostsim: bool, W=None, H=None, spp=None, bounces=None, fb=None,
                spheres=None, device=0, materials=None, loopback=False, rccl_clique=False):
    P = parsed_scene(entry["scene"])
    W = W or entry["W"]
    H = H or entry["H"]
    fb = fb if fb is not None else rt_amd.Image(W, H)
    c = cameras[entry["camera"]]
    mats = materials if materials is not None else materials_for(entry, P)
    mi = P.material_indices
    if spheres is None and entry.get("spheres"):
        mats, mi, spheres = sphere_buffers(entry, P, mats)
    rk = rt_amd.RenderKernel(W, H, spp or entry["spp"], bounces or entry["bounces"], fb, P.triangles,
                             mats, P.emissive_triangle_indices, mi, spheres,
                             rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky(entry["sky"])), None,
                             hostsim=hostsim, device=device, loopback=loopback, rccl_clique=rccl_clique)
    rk.set_camera(rt_amd.Camera(c[:16], c[16]))
    return rk, fb


def run_case(entry: dict, cameras: dict, hostsim: bool, schedule: dict | None = None) -> np.ndarray:
    """Returns the tone-mapped RGBA of the case (full frame or its pixel list); schedule:
    rt_test_schedule overrides (tests only)."""
    rk, fb = make_kernel(entry, cameras, hostsim)
    if schedule:
        rk.test_schedule(**schedule)
    if entry.get("px") is None:
        rk.render()
        return fb.pixels
    rk.ray_trace_pixels(entry["px"])
    px = entry["px"]
    return fb.pixels[px[:, 1], px[:, 0]]


def oracle_scene(entry: dict):
    from oracle_bindings import OracleScene
    P = parsed_scene(entry["scene"])
    mats, mi, spheres = sphere_buffers(entry, P, materials_for(entry, P))
    return OracleScene(P.triangles, mi, mats, P.emissive_triangle_indices, env=sky(entry["sky"]), spheres=spheres)


def run_oracle(entry: dict, cameras: dict, threads: int = 0) -> np.ndarray:
    S = oracle_scene(entry)
    res, _ = S.render(cameras[entry["camera"]], entry["W"], entry["H"], entry["spp"], entry["bounces"],
                      pixels=entry.get("px"), threads=threads)
    return res


CORNELL_CASES = ["cfg1_cornell12", "cornell32_128", "cornell32_64spp", "mis_512", "spheres_cornell32_128",
                 "spheres_cornell32_64spp"]
SPHERE_CASES = ["spheres_cornell32_128", "spheres_cornell32_64spp", "spheres_dragon"]
DRAGON_CASES = ["cfg2_dragon", "cfg3_dragon", "cfg4_dragon4k", "spheres_dragon"] + [
    f"cfg5_sweep_m{m}_r{r}" for m in range(4) for r in range(4)]


def tiny_scene(n: int):
    """The first n triangles of cornell12 (0: an empty scene, only the sky): the
    degenerate octree / search-BVH shapes (no root children, one leaf, a leaf that
    splits at the 4-triangle limit)."""
    from conftest import parsed_scene
    P = parsed_scene("cornell12")
    tris = P.triangles[:n].copy() if n else np.zeros((0, 9), np.float32)
    mi = P.material_indices[:n].copy()
    em = np.array([i for i in P.emissive_triangle_indices if i < n], np.int32)
    return tris, mi, P.materials, em


def render_tiny(n: int, cameras: dict, hostsim: bool, W=24, H=20, spp=2, nb=3):
    """(got, want): the tiny scene through the product (or hostsim) and the oracle."""
    from oracle_bindings import OracleScene
    tris, mi, mats, em = tiny_scene(n)
    env = sky("S")
    c = cameras["cornell"]
    want, _ = OracleScene(tris, mi, mats, em, env=env).render(c, W, H, spp, nb)
    fb = rt_amd.Image(W, H)
    rk = rt_amd.RenderKernel(W, H, spp, nb, fb, tris, mats, em, mi, None, rt_amd.BVH(tris),
                             rt_amd.Image.from_rgb(env), None, hostsim=hostsim)
    rk.set_camera(rt_amd.Camera(c[:16], c[16]))
    rk.render()
    return fb.pixels, want
