"""Diagnostic: closest-hit throughput of the gfx950 traversal on the dragon
stand-in for a batch of rays (camera rays and random rays), via rt_intersect
(one thread per ray, full grid) — isolates traversal speed from the
wavefront machinery."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools")]
import rt_amd  # noqa: E402
import scenes  # noqa: E402

P = rt_amd.parse_obj(scenes.scene_path("dragon"))
rk = rt_amd.RenderKernel(16, 16, 1, 1, rt_amd.Image(16, 16), P.triangles, P.materials, P.emissive_triangle_indices,
                         P.material_indices, None, rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(scenes.make_sky("S")),
                         None)
rng = np.random.default_rng(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
cam = rt_amd.Camera.preset("dragon").view_matrix
o = cam[:3, 3]
# camera-like rays toward the object, and uniformly random rays from points near it
tgt = np.stack([rng.uniform(-2, 2, n), rng.uniform(0, 3, n), rng.uniform(-2, 2, n)], 1)
d = tgt - o
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays_cam = np.concatenate([np.broadcast_to(o, (n, 3)), d], 1).astype(np.float32)
org = np.stack([rng.uniform(-3, 3, n), rng.uniform(0.01, 4, n), rng.uniform(-3, 3, n)], 1)
dd = rng.normal(size=(n, 3))
dd /= np.linalg.norm(dd, axis=1, keepdims=True)
rays_rnd = np.concatenate([org, dd], 1).astype(np.float32)
# the same random rays sorted by direction octant, then origin cell (coherence probe)
octant = (dd[:, 0] > 0) * 4 + (dd[:, 1] > 0) * 2 + (dd[:, 2] > 0)
cell = np.floor((org - org.min(0)) / 0.25).astype(np.int64)
key = octant * (1 << 30) + cell[:, 0] * (1 << 20) + cell[:, 1] * (1 << 10) + cell[:, 2]
rays_srt = rays_rnd[np.argsort(key, kind="stable")]
for name, rays in (("camera", rays_cam), ("random", rays_rnd), ("random_sorted", rays_srt)):
    for rep in range(2):
        out = rk.intersect(rays)
        ms = rk.last_kernel_ms()
        print(f"{name}: {n} rays {ms:.2f} ms -> {n / ms / 1e3:.1f} Mrays/s, hit {out[:, 0].mean():.3f}", flush=True)
