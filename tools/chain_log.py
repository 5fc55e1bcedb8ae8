"""Per-sample RNG draw counts of a shard's pixels (analysis input for tools/chain_model.py).

Renders every --every-th pixel of rank r's rows (y % world == r) of a config with the
CPU restatement (oracle_render_log; analysis only, nothing here is measured) and saves
draws[n_px][spp] (uint16) with the pixel list. A sample's draw count is 2 + D * (its
shaded bounces), D fixed per scene, so the log is the pixel's whole sample chain.

  python tools/chain_log.py --config cfg4 --world 8 --rank 0 --every 32 --out /tmp/chain_cfg4.npz
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--every", type=int, default=32)
    ap.add_argument("--out", default="/tmp/chain_cfg4.npz")
    args = ap.parse_args()
    import bench
    from oracle_bindings import OracleScene, _p, lib

    _, _, _, W, H, spp, nb, _ = bench.CONFIGS[args.config]
    P, sky, cam17 = bench.build_inputs(args.config)
    S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices, env=sky)
    rows = np.arange(args.rank, H, args.world)
    xs, ys = np.meshgrid(np.arange(W), rows)
    px = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)[:: args.every].copy()
    fb = np.zeros((H, W, 4), np.float32)
    log = np.zeros((px.shape[0], spp), np.uint16)
    L = lib()
    L.oracle_render_log.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float] + [ctypes.c_int] * 4 + \
        [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    cam = np.ascontiguousarray(cam17[:16], np.float32)
    t0 = time.time()
    L.oracle_render_log(S.h, _p(cam), float(np.float32(cam17[16])), W, H, spp, nb, _p(px), px.shape[0], _p(fb), _p(log))
    print(f"{px.shape[0]} px x {spp} spp in {time.time() - t0:.1f} s", flush=True)
    np.savez_compressed(args.out, draws=log, px=px, W=W, H=H, spp=spp, bounces=nb, world=args.world,
                        rank=args.rank, every=args.every)
    d = log.astype(np.int64)
    print("draw counts:", dict(zip(*np.unique(d, return_counts=True))))


if __name__ == "__main__":
    main()
