"""Golden fixtures for far ray origins, written by the REFERENCE
itself (container only).

* Ray answers: `ref_driver rays` calls the reference's BVH::intersect (bvh.h:127-209, the
  octree walk INTERSECT_SCENE runs) on rays aimed at uniform points of uniformly chosen
  triangles from distance D along random directions, or along directions within ~3 degrees
  of the triangle's plane (grazing): tools/far_probe.py far_rays, D = 1e2 ... 1e5 (plus two
  near distances per scene, which the search BVH itself answers).
* Renders: far telephoto cameras, built the way camera.cpp:3-8 builds the presets
  (Camera(fov, RotationX(rx) * Translation(...)), `ref_driver` camera spec "tele:..."), at
  1000x the distance of the Cornell and dragon presets with the field of view narrowed to
  frame the same scene: whole frames through the reference's RenderKernel::render.

    make -C oracle/ref && python tools/gen_golden_far.py

Writes tests/golden/far_rays_{cornell,dragon}.npz, far_render_*.npz and
tests/golden/far_manifest.json (data only).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import far_probe  # noqa: E402
import golden_io as gio  # noqa: E402
import scenes  # noqa: E402
from gen_golden_brute import run  # noqa: E402

REF = os.path.join(gio.REPO, "oracle", "_ref", "ref_driverO2")
OUT = gio.GOLDEN
N_PER = 512
DISTS = {"cornell": [1.0, 2.0, 1e2, 1e3, 1e4, 1e5], "dragon": [10.0, 20.0, 1e2, 1e3, 1e4, 1e5]}
# (name, scene, sky, camera spec, W, H, spp, bounces)
RENDERS = [
    ("cornell_tele", "cornell", "S", "tele:0.0475:0:0:1:3500", 64, 64, 2, 3),
    ("dragon_tele", "dragon", "L", "tele:0.045:-45:0:-1:10500", 160, 90, 4, 8),
]


def ref_rays(tmp, obj, rays):
    p = os.path.join(tmp, "rays.bin")
    with open(p, "wb") as f:
        f.write(np.int32(rays.shape[0]).tobytes())
        f.write(np.ascontiguousarray(rays, np.float32).tobytes())
    run(REF, "rays", obj, p, os.path.join(tmp, "hits.bin"))
    return gio.read_hits(open(os.path.join(tmp, "hits.bin"), "rb").read(), rays.shape[0], 4)


def main():
    tmp = tempfile.mkdtemp()
    man = {"generator": "tools/gen_golden_far.py", "reference": REF, "rays": {}, "renders": {}}
    for sc, dists in DISTS.items():
        obj = scenes.scene_path(sc)
        run(REF, "parse", obj, os.path.join(tmp, "p.bin"))
        tris = gio.read_parse(os.path.join(tmp, "p.bin"))["tris"].reshape(-1, 9)
        rays, dist, mode = [], [], []
        for mi, m in enumerate(("random", "grazing")):
            for D in dists:
                rng = np.random.default_rng([11, int(D), mi, len(sc)])
                rays.append(far_probe.far_rays(tris, D, N_PER, m, rng))
                dist += [D] * N_PER
                mode += [mi] * N_PER
        rays = np.concatenate(rays)
        hits = ref_rays(tmp, obj, rays)
        np.savez_compressed(os.path.join(OUT, f"far_rays_{sc}.npz"), rays=rays, hits=hits,
                            dist=np.asarray(dist, np.float32), mode=np.asarray(mode, np.int8))
        man["rays"][sc] = {"n": int(rays.shape[0]), "per_set": N_PER, "distances": dists,
                           "modes": ["random", "grazing"], "found": int(hits["found"].sum()),
                           "hits_sha256": gio.sha256(hits)}
        print(sc, man["rays"][sc], flush=True)

    sky = {k: os.path.join(tmp, f"sky{k}.raw") for k in "SL"}
    for k, p in sky.items():
        scenes.write_sky_raw(p, k)
    for name, sc, sk, cam, W, H, spp, nb in RENDERS:
        run(REF, "camera", cam, os.path.join(tmp, "cam.bin"))
        cam17 = np.fromfile(os.path.join(tmp, "cam.bin"), dtype="<f4")
        out = os.path.join(tmp, "fb.f32")
        log = run(REF, "render", scenes.scene_path(sc), sky[sk], cam, W, H, spp, nb, out)
        fb = np.fromfile(out, dtype="<f4").reshape(H, W, 4)
        np.savez_compressed(os.path.join(OUT, f"far_render_{name}.npz"), rgba=fb, camera=cam17)
        man["renders"][name] = {"scene": sc, "sky": sk, "camera": cam, "W": W, "H": H, "spp": spp, "bounces": nb,
                                "rgba_sha256": gio.sha256(fb), "ref_log": log.strip().splitlines()[-1]}
        print(name, man["renders"][name]["ref_log"], flush=True)
    with open(os.path.join(OUT, "far_manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
