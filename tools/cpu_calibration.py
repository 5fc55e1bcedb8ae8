"""CPU calibration: the compiled reference (oracle/_ref/ref_driverO2, built
from /root/reference by oracle/ref/Makefile; container only) and the pinned CPU port
(oracle/cpu_oracle.cpp, bench.py's cpu_baseline) render the same cfg2 pixel subset on the
same host threads; their outputs must agree bit for bit and the ratio calibrates bench.py's
`cpu_baseline` (kind "port") against the reference itself.

  python tools/cpu_calibration.py [--row-step 10] [--col-step 16] [--spp 8] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--row-step", type=int, default=10)
    ap.add_argument("--col-step", type=int, default=16)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05_cpu_calibration.json"))
    args = ap.parse_args()
    import bench
    import golden_io as gio
    import scenes
    from oracle_bindings import OracleScene

    scene, sky_kind, cam, W, H, spp, nb, desc = bench.CONFIGS["cfg2"]
    spp = args.spp
    P, sky, cam17 = bench.build_inputs("cfg2")
    rows = np.arange(args.row_step // 2, H, args.row_step)
    cols = np.arange(args.col_step // 2, W, args.col_step)
    xs, ys = np.meshgrid(cols, rows)
    px = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    n = px.shape[0]
    ref = os.path.join(REPO, "oracle", "_ref", "ref_driverO2")
    tmp = tempfile.mkdtemp()
    sky_raw = os.path.join(tmp, "sky.raw")
    scenes.write_sky_raw(sky_raw, sky_kind)
    gio.write_pixels(os.path.join(tmp, "px.bin"), px)
    env = dict(os.environ, OMP_NUM_THREADS=str(args.threads))
    t0 = time.perf_counter()
    r = subprocess.run([ref, "pixels", scenes.scene_path(scene), sky_raw, cam, str(W), str(H), str(spp), str(nb),
                        os.path.join(tmp, "px.bin"), os.path.join(tmp, "pc.bin")], capture_output=True, text=True, env=env)
    wall = time.perf_counter() - t0
    if r.returncode:
        raise SystemExit(r.stderr)
    line = [x for x in r.stderr.splitlines() if x.startswith("REF_PIXELS_SECONDS")][-1]
    ref_sec = float(line.split()[1])
    ref_rgba = gio.read_pixel_colors(os.path.join(tmp, "pc.bin"))
    S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices, env=sky)
    port, port_sec = S.render(cam17, W, H, spp, nb, pixels=px, threads=args.threads, counters=False)
    par = gio.compare_rgb(port, ref_rgba)
    samples = n * spp
    out = {"what": "cfg2 scene (dragon stand-in, SKY-L), the same pixel subset rendered by the compiled reference "
                   "(RenderKernel::ray_trace_pixel, OpenMP dynamic) and by the CPU port (oracle/cpu_oracle.cpp), "
                   "same host threads, this container",
           "pixels": int(n), "subset": f"every {args.row_step}th row x every {args.col_step}th column",
           "spp": spp, "bounces": nb, "threads": args.threads, "cpu_model": bench.cpu_model(),
           "reference": {"seconds": round(ref_sec, 3), "msamples_per_s": round(samples / ref_sec / 1e6, 4),
                         "wall_s_incl_scene_build": round(wall, 2)},
           "port": {"seconds": round(port_sec, 3), "msamples_per_s": round(samples / port_sec / 1e6, 4)},
           "port_over_reference": round(ref_sec / port_sec, 3), "parity": par}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
