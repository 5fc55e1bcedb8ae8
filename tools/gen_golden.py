"""Generate the golden fixtures in tests/golden/ by running the REFERENCE
(oracle/_ref/ref_driverO2, built from /root/reference by oracle/ref/Makefile).

Run in the container (the reference sources are not on the GPU box):
    make -C oracle/ref && python tools/gen_golden.py

Fixtures are data only: inputs, expected outputs and hashes of expected
outputs. Everything larger than a few hundred KB is stored as a SHA-256 plus
a sampled subset.
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

REF = os.path.join(gio.REPO, "oracle", "_ref", "ref_driverO2")
OUT = gio.GOLDEN

# analytic spheres (main.cpp:20-30 add_sphere_to_scene): 12 floats each,
# center xyz, radius, emission rgb, diffuse rgb, metalness, roughness. Non-emissive only: an
# emissive sphere makes the reference read the triangle buffer out of bounds (render_kernel.cpp:690-700).
SPH_MAIN = [0.3275, 0.7, 0.3725, 0.2, 0, 0, 0, 1.0, 0.71, 0.29, 1.0, 0.4]  # main.cpp:72 (commented out there)
SPH_DIFFUSE = [-0.35, 0.3, 0.1, 0.25, 0, 0, 0, 0.2, 0.6, 0.9, 0.0, 0.8]
SPH_DRAGON = [[2.6, 1.0, 1.4, 1.0, 0, 0, 0, 0.95, 0.95, 0.95, 1.0, 0.1],
              [-2.9, 0.8, 0.6, 0.8, 0, 0, 0, 0.8, 0.3, 0.2, 0.0, 0.6]]

# (name, scene, sky, camera, W, H, spp, bounces, pixels or None for full frame, mat override[, spheres])
RENDERS = [
    ("cfg1_cornell12", "cornell12", "S", "cornell", 256, 256, 4, 3, None, None),
    ("cornell32_128", "cornell", "S", "cornell", 128, 128, 4, 3, None, None),
    ("cornell32_64spp", "cornell", "S", "cornell", 512, 512, 64, 8, 1024, None),
    ("mis_512", "mis", "S", "mis", 512, 512, 16, 8, 2048, None),
    ("cfg2_dragon", "dragon", "L", "dragon", 1920, 1080, 64, 8, 4096, None),
    ("cfg3_dragon", "dragon", "L", "dragon", 1920, 1080, 256, 8, 1024, None),
    ("cfg4_dragon4k", "dragon", "L", "dragon", 3840, 2160, 256, 8, 1024, None),
] + [
    (f"cfg5_sweep_m{mi}_r{ri}", "dragon", "L", "dragon", 1920, 1080, 1024, 8, 48,
     (1, [0.0, 1.0 / 3.0, 2.0 / 3.0, 1.0][mi], [0.05, 0.25, 0.5, 1.0][ri]))
    for mi in range(4) for ri in range(4)
] + [
    ("spheres_cornell32_128", "cornell", "S", "cornell", 128, 128, 4, 3, None, None, [SPH_MAIN]),
    ("spheres_cornell32_64spp", "cornell", "S", "cornell", 256, 256, 64, 8, 1024, None, [SPH_MAIN, SPH_DIFFUSE]),
    ("spheres_dragon", "dragon", "L", "dragon", 1920, 1080, 64, 8, 1024, None, SPH_DRAGON),
]


def sphere_env(spheres):
    """RT_SPHERES for ref_driver: the float32 values as C99 hex floats (exact through strtof)."""
    f32 = np.asarray(spheres, np.float32).reshape(-1, 12)
    return ";".join(",".join(float(v).hex() for v in row) for row in f32)


def run(*args, env=None):
    e = dict(os.environ)
    if env:
        e.update(env)
    r = subprocess.run([REF, *map(str, args)], capture_output=True, text=True, env=e)
    if r.returncode != 0:
        raise RuntimeError(f"ref_driver {args} failed: {r.stderr}")
    return r.stderr


def main():
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp()
    manifest = {"generator": "tools/gen_golden.py", "reference": REF, "renders": {}, "scenes": {}}

    sky = {k: os.path.join(tmp, f"sky{k}.raw") for k in "SL"}
    for k, p in sky.items():
        scenes.write_sky_raw(p, k)
        run("cdf", p, p + ".cdf")
        b = np.fromfile(p + ".cdf", dtype="<f4", offset=8)
        W, H = scenes.SKY_SPECS[k][:2]
        lum, cdf = b[: W * H], b[W * H:]
        manifest[f"sky{k}"] = {"lum_sha256": gio.sha256(lum), "cdf_sha256": gio.sha256(cdf),
                               "cdf_last": float(cdf[-1])}
        if k == "S":
            np.savez_compressed(os.path.join(OUT, "skyS_cdf.npz"), lum=lum, cdf=cdf)

    # cameras (camera.cpp:3-8 presets)
    cams = {}
    for name in ["default", "cornell", "ganesha", "ite", "dragon", "mis"]:
        run("camera", name, os.path.join(tmp, "cam.bin"))
        m, fov = gio.read_camera(os.path.join(tmp, "cam.bin"))
        cams[name] = np.concatenate([m, [fov]]).astype(np.float32)
    np.savez(os.path.join(OUT, "cameras.npz"), **cams)

    # parse + octree dumps
    for sc in ["cornell12", "cornell", "mis", "dragon"]:
        obj = scenes.scene_path(sc)
        run("parse", obj, os.path.join(tmp, "p.bin"))
        P = gio.read_parse(os.path.join(tmp, "p.bin"))
        run("bvh", obj, os.path.join(tmp, "b.bin"))
        bvh = open(os.path.join(tmp, "b.bin"), "rb").read()
        info = {k: {"sha256": gio.sha256(v), "shape": list(v.shape)} for k, v in P.items()}
        info["octree_sha256"] = gio.sha256(np.frombuffer(bvh, np.uint8))
        info["octree_bytes"] = len(bvh)
        info["octree_stats"] = gio.parse_octree_dump(bvh)
        manifest["scenes"][sc] = info
        if sc != "dragon":
            np.savez_compressed(os.path.join(OUT, f"parse_{sc}.npz"), **P)
            np.savez_compressed(os.path.join(OUT, f"octree_{sc}.npz"), dump=np.frombuffer(bvh, np.uint8))
        print(sc, info["octree_stats"], flush=True)

    # reference's own BVH regression vectors (source/tests.cpp, include/bvh_tests.h)
    run("bvhtests", scenes.scene_path("cornell"), os.path.join(tmp, "t.bin"))
    b = open(os.path.join(tmp, "t.bin"), "rb").read()
    rec = np.dtype([("o", "<f4", 3), ("d", "<f4", 3), ("expect", "<f4", 3),
                    ("bvh", gio.read_hits(b"\0" * 44, 1).dtype), ("flat", gio.read_hits(b"\0" * 44, 1).dtype)])
    n1 = int(np.frombuffer(b, "<i4", 1, 0)[0])
    inter = np.frombuffer(b, rec, n1, 4)
    n2 = int(np.frombuffer(b, "<i4", 1, 4 + n1 * rec.itemsize)[0])
    miss = np.frombuffer(b, rec, n2, 8 + n1 * rec.itemsize)
    np.savez_compressed(os.path.join(OUT, "bvhtests_cornell.npz"), inter=inter, miss=miss)
    manifest["bvhtests"] = {"inter": n1, "miss": n2}

    # ray-cast goldens on the dragon stand-in (closest hit, incl. vertex/edge-aimed rays)
    rng = np.random.default_rng(7)
    P = gio.read_parse(os.path.join(tmp, "p.bin")) if False else None
    run("parse", scenes.scene_path("dragon"), os.path.join(tmp, "pd.bin"))
    P = gio.read_parse(os.path.join(tmp, "pd.bin"))
    tris = P["tris"].reshape(-1, 3, 3)
    n = 8192
    sel = rng.integers(0, tris.shape[0], n)
    w = rng.dirichlet([1, 1, 1], n).astype(np.float32)
    target = np.einsum("nk,nkc->nc", w, tris[sel])
    # a quarter aimed exactly at a vertex, a quarter at an edge midpoint (tie-prone)
    q = n // 4
    target[:q] = tris[sel[:q], 0]
    target[q:2 * q] = 0.5 * (tris[sel[q:2 * q], 0] + tris[sel[q:2 * q], 1])
    orig = rng.normal(size=(n, 3)).astype(np.float32) * np.float32(6.0) + np.float32([0, 3, 0])
    d = (target - orig).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    rays = np.concatenate([orig, d], axis=1).astype(np.float32)
    with open(os.path.join(tmp, "rays.bin"), "wb") as f:
        f.write(np.int32(n).tobytes())
        f.write(rays.tobytes())
    run("rays", scenes.scene_path("dragon"), os.path.join(tmp, "rays.bin"), os.path.join(tmp, "hits.bin"))
    hb = open(os.path.join(tmp, "hits.bin"), "rb").read()
    hits = gio.read_hits(hb, n, 4)
    np.savez_compressed(os.path.join(OUT, "rays_dragon.npz"), rays=rays, hits=hits)

    # renders
    for name, sc, sk, cam, W, H, spp, nb, npx, mo, *rest in RENDERS:
        obj = scenes.scene_path(sc)
        env = {"RT_MAT_OVERRIDE": f"{mo[0]}:{mo[1]!r}:{mo[2]!r}"} if mo else {}
        entry = {"scene": sc, "sky": sk, "camera": cam, "W": W, "H": H, "spp": spp, "bounces": nb}
        if mo:
            entry["mat_override"] = {"index": mo[0], "metalness": mo[1], "roughness": mo[2]}
        if rest:
            env["RT_SPHERES"] = sphere_env(rest[0])
            entry["spheres"] = np.asarray(rest[0], np.float32).reshape(-1, 12).tolist()
        if npx is None:
            out = os.path.join(tmp, "fb.f32")
            log = run("render", obj, sky[sk], cam, W, H, spp, nb, out, env=env)
            fb = np.fromfile(out, dtype="<f4").reshape(H, W, 4)
            np.savez_compressed(os.path.join(OUT, f"render_{name}.npz"), rgba=fb)
            entry["full_frame"] = True
            entry["rgba_sha256"] = gio.sha256(fb)
        else:
            seed = abs(hash(name)) % (2 ** 31) if False else sum(map(ord, name))
            px = gio.sample_pixels(W, H, npx, seed)
            gio.write_pixels(os.path.join(tmp, "px.bin"), px)
            log = run("pixels", obj, sky[sk], cam, W, H, spp, nb, os.path.join(tmp, "px.bin"),
                      os.path.join(tmp, "pc.bin"), env=env)
            rgba = gio.read_pixel_colors(os.path.join(tmp, "pc.bin"))
            np.savez_compressed(os.path.join(OUT, f"render_{name}.npz"), px=px, rgba=rgba)
            entry["pixels"] = int(px.shape[0])
        entry["ref_log"] = log.strip().splitlines()[-1]
        manifest["renders"][name] = entry
        print(name, entry["ref_log"], flush=True)

    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
