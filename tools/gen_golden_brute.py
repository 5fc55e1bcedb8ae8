"""Golden fixtures for USE_BVH 0 (render_kernel.h:13): INTERSECT_SCENE as the
brute-force loop, written by the REFERENCE itself (container only).

* Ray answers: `ref_driver brute` calls the public RenderKernel::intersect_scene
  (render_kernel.h:65, render_kernel.cpp:453-483) on ray lists: the reference's
  own Cornell regression rays (bvh_tests.h), tie-prone rays aimed at Cornell
  triangle edges (with and without main.cpp's sphere) and the 8192 dragon rays of
  rays_dragon.npz (a quarter aimed at vertices, a quarter at edge midpoints).
* Renders: `ref_driver_bruteO2` links the reference's render_kernel.cpp compiled
  unchanged with USE_BVH 0 (oracle/ref/render_kernel_brute.cpp), so
  ray_trace_pixel runs the brute-force loop for every query.

    make -C oracle/ref && python tools/gen_golden_brute.py

Writes tests/golden/brute_*.npz and tests/golden/brute_manifest.json (data only).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import golden_io as gio  # noqa: E402
import scenes  # noqa: E402
from gen_golden import SPH_DIFFUSE, SPH_DRAGON, SPH_MAIN, sphere_env  # noqa: E402

REF = os.path.join(gio.REPO, "oracle", "_ref", "ref_driverO2")
REF_BRUTE = os.path.join(gio.REPO, "oracle", "_ref", "ref_driver_bruteO2")
OUT = gio.GOLDEN

# (name, scene, sky, camera, W, H, spp, bounces, pixels or None for a full frame, spheres)
RENDERS = [
    ("cfg1_cornell12_64", "cornell12", "S", "cornell", 64, 64, 4, 3, None, None),
    ("cornell32_64", "cornell", "S", "cornell", 64, 64, 4, 3, None, None),
    ("cornell32_8spp", "cornell", "S", "cornell", 256, 256, 8, 8, 512, None),
    ("mis_512", "mis", "S", "mis", 512, 512, 4, 8, 256, None),
    ("spheres_cornell32_64", "cornell", "S", "cornell", 64, 64, 4, 3, None, [SPH_MAIN, SPH_DIFFUSE]),
    ("dragon_2spp", "dragon", "L", "dragon", 1920, 1080, 2, 8, 96, None),
    ("spheres_dragon_2spp", "dragon", "L", "dragon", 1920, 1080, 2, 8, 64, SPH_DRAGON),
]


def run(exe, *args, env=None):
    e = dict(os.environ)
    if env:
        e.update(env)
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, env=e)
    if r.returncode != 0:
        raise RuntimeError(f"{os.path.basename(exe)} {args} failed: {r.stderr}")
    return r.stderr


def edge_rays(tris: np.ndarray, n_per: int = 4, seed: int = 2) -> np.ndarray:
    """Rays through points on triangle edges (shared edges give exact t ties): the
    tie rule of the loop (strict `<` in buffer order) decides these."""
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


def brute_rays(tmp, obj, rays, spheres=None):
    p = os.path.join(tmp, "rays.bin")
    with open(p, "wb") as f:
        f.write(np.int32(rays.shape[0]).tobytes())
        f.write(np.ascontiguousarray(rays, np.float32).tobytes())
    env = {"RT_SPHERES": sphere_env(spheres)} if spheres else None
    run(REF, "brute", obj, p, os.path.join(tmp, "hits.bin"), env=env)
    return gio.read_hits(open(os.path.join(tmp, "hits.bin"), "rb").read(), rays.shape[0], 4)


def main():
    tmp = tempfile.mkdtemp()
    man = {"generator": "tools/gen_golden_brute.py", "reference": [REF, REF_BRUTE], "rays": {}, "renders": {}}

    # rays: Cornell regression vectors + edge rays (+ spheres), dragon tie-prone rays
    bt = np.load(os.path.join(OUT, "bvhtests_cornell.npz"))
    reg = np.concatenate([np.concatenate([bt[k]["o"], bt[k]["d"]], 1) for k in ("inter", "miss")]).astype(np.float32)
    run(REF, "parse", scenes.scene_path("cornell"), os.path.join(tmp, "p.bin"))
    ctris = gio.read_parse(os.path.join(tmp, "p.bin"))["tris"]
    cases = {
        "cornell_regression": ("cornell", reg, None),
        "cornell_edges": ("cornell", edge_rays(ctris), None),
        "cornell_edges_spheres": ("cornell", edge_rays(ctris, seed=3), [SPH_MAIN, SPH_DIFFUSE]),
        "dragon_tie_prone": ("dragon", np.load(os.path.join(OUT, "rays_dragon.npz"))["rays"], None),
    }
    for name, (sc, rays, sph) in cases.items():
        hits = brute_rays(tmp, scenes.scene_path(sc), rays, sph)
        np.savez_compressed(os.path.join(OUT, f"brute_rays_{name}.npz"), rays=rays, hits=hits)
        entry = {"scene": sc, "n": int(rays.shape[0]), "found": int(hits["found"].sum()),
                 "hits_sha256": gio.sha256(hits)}
        if sph:
            entry["spheres"] = np.asarray(sph, np.float32).reshape(-1, 12).tolist()
        man["rays"][name] = entry
        print(name, entry["n"], "found", entry["found"], flush=True)

    sky = {k: os.path.join(tmp, f"sky{k}.raw") for k in "SL"}
    for k, p in sky.items():
        scenes.write_sky_raw(p, k)
    for name, sc, sk, cam, W, H, spp, nb, npx, sph in RENDERS:
        obj = scenes.scene_path(sc)
        env = {"RT_SPHERES": sphere_env(sph)} if sph else {}
        entry = {"scene": sc, "sky": sk, "camera": cam, "W": W, "H": H, "spp": spp, "bounces": nb}
        if sph:
            entry["spheres"] = np.asarray(sph, np.float32).reshape(-1, 12).tolist()
        if npx is None:
            out = os.path.join(tmp, "fb.f32")
            log = run(REF_BRUTE, "render", obj, sky[sk], cam, W, H, spp, nb, out, env=env)
            fb = np.fromfile(out, dtype="<f4").reshape(H, W, 4)
            np.savez_compressed(os.path.join(OUT, f"brute_render_{name}.npz"), rgba=fb)
            entry["full_frame"] = True
            entry["rgba_sha256"] = gio.sha256(fb)
        else:
            px = gio.sample_pixels(W, H, npx, sum(map(ord, name)))
            gio.write_pixels(os.path.join(tmp, "px.bin"), px)
            log = run(REF_BRUTE, "pixels", obj, sky[sk], cam, W, H, spp, nb, os.path.join(tmp, "px.bin"),
                      os.path.join(tmp, "pc.bin"), env=env)
            rgba = gio.read_pixel_colors(os.path.join(tmp, "pc.bin"))
            np.savez_compressed(os.path.join(OUT, f"brute_render_{name}.npz"), px=px, rgba=rgba)
            entry["pixels"] = int(px.shape[0])
        entry["ref_log"] = log.strip().splitlines()[-1]
        man["renders"][name] = entry
        print(name, entry["ref_log"], flush=True)

    with open(os.path.join(OUT, "brute_manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
