"""Readers for the binary dumps written by oracle/ref/ref_driver.cpp and the
shared fixture layout under tests/golden/.

Kept free of any GPU / product imports so tests, the fixture generator and
bench.py can all use it.
"""
from __future__ import annotations

import hashlib
import os
import struct

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def sha256(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def read_parse(path: str) -> dict:
    """ref_driver 'parse' dump -> dict(tris [N,9] f32, mat_idx [N] i32, mats [M,10] f32, emissive [E] i32)."""
    b = open(path, "rb").read()
    o = 0

    def i32():
        nonlocal o
        v = struct.unpack_from("<i", b, o)[0]
        o += 4
        return v

    def arr(dtype, n):
        nonlocal o
        a = np.frombuffer(b, dtype=dtype, count=n, offset=o).copy()
        o += a.nbytes
        return a

    n = i32()
    tris = arr("<f4", n * 9).reshape(n, 9)
    m = i32()
    mat_idx = arr("<i4", m)
    k = i32()
    mats = arr("<f4", k * 10).reshape(k, 10)
    e = i32()
    emissive = arr("<i4", e)
    return {"tris": tris, "mat_idx": mat_idx, "mats": mats, "emissive": emissive}


def parse_octree_dump(b: bytes) -> dict:
    """Pre-order octree dump (ref_driver 'bvh' / oracle_bvh_dump / rt_bvh_dump) -> summary stats."""
    o = 0
    nodes = leaves = empty = internal = maxleaf = maxdepth = 0
    stack = [0]
    while o < len(b):
        depth = stack.pop()
        leaf, nt = struct.unpack_from("<ii", b, o)
        o += 8 + 4 * nt + 4 * (6 + 14)
        nodes += 1
        maxdepth = max(maxdepth, depth)
        if leaf:
            leaves += 1
            empty += nt == 0
            maxleaf = max(maxleaf, nt)
        else:
            internal += 1
            stack.extend([depth + 1] * 8)
    return dict(nodes=nodes, internal=internal, leaves=leaves, empty_leaves=empty, max_leaf=maxleaf,
                max_depth=maxdepth)


def read_hits(buf: bytes, n: int, offset: int = 0) -> np.ndarray:
    """n x {found i32, prim i32, t, p[3], n[3], u, v} -> structured array."""
    dt = np.dtype([("found", "<i4"), ("prim", "<i4"), ("t", "<f4"), ("p", "<f4", 3), ("n", "<f4", 3),
                   ("u", "<f4"), ("v", "<f4")])
    return np.frombuffer(buf, dtype=dt, count=n, offset=offset).copy()


def read_camera(path: str):
    a = np.fromfile(path, dtype="<f4")
    return a[:16].copy(), float(a[16])


def write_pixels(path: str, px: np.ndarray) -> None:
    px = np.ascontiguousarray(px, dtype="<i4")
    with open(path, "wb") as f:
        f.write(struct.pack("<i", px.shape[0]))
        f.write(px.tobytes())


def read_pixel_colors(path: str) -> np.ndarray:
    b = open(path, "rb").read()
    n = struct.unpack_from("<i", b, 0)[0]
    return np.frombuffer(b, dtype="<f4", count=n * 4, offset=4).reshape(n, 4).copy()


def sample_pixels(W: int, H: int, n: int, seed: int) -> np.ndarray:
    """Unique, stratified pixel sample incl. corners and the x=0 / y=0 lines
    (where the reference's seed 31+x*y*spp collides)."""
    rng = np.random.default_rng(seed)
    fixed = [(0, 0), (W - 1, 0), (0, H - 1), (W - 1, H - 1), (0, H // 2), (W // 2, 0), (1, 1), (W // 2, H // 2)]
    g = int(np.ceil(np.sqrt(max(n - len(fixed), 1))))
    xs = ((np.arange(g) + 0.5) * W / g).astype(int)
    ys = ((np.arange(g) + 0.5) * H / g).astype(int)
    gx, gy = np.meshgrid(xs, ys)
    jit = rng.integers(-W // (3 * g) - 1, W // (3 * g) + 2, size=gx.shape)
    jjt = rng.integers(-H // (3 * g) - 1, H // (3 * g) + 2, size=gy.shape)
    cand = np.stack([np.clip(gx + jit, 0, W - 1).ravel(), np.clip(gy + jjt, 0, H - 1).ravel()], axis=1)
    allpx = np.concatenate([np.array(fixed), cand])
    _, idx = np.unique(allpx[:, 1] * W + allpx[:, 0], return_index=True)
    out = allpx[np.sort(idx)][:n]
    return out.astype(np.int32)


def compare_rgb(a: np.ndarray, b: np.ndarray) -> dict:
    """Per-channel L-inf on RGB with NaN == NaN; also bitwise-identical fraction."""
    a = np.asarray(a, dtype=np.float32)[..., :3]
    b = np.asarray(b, dtype=np.float32)[..., :3]
    na, nb = np.isnan(a), np.isnan(b)
    nan_mismatch = int(np.count_nonzero(na != nb))
    both = ~(na | nb)
    diff = np.zeros_like(a)
    diff[both] = np.abs(a[both] - b[both])
    linf = float(diff.max()) if diff.size else 0.0
    if nan_mismatch:
        linf = float("inf")
    px_over = int(np.count_nonzero((diff > 1e-4).any(axis=-1) | (na != nb).any(axis=-1)))
    bitwise = np.all((a.view(np.uint32) == b.view(np.uint32)) | (na & nb), axis=-1)
    return dict(linf=linf, pixels_over_1e4=px_over, nan_mismatch=nan_mismatch,
                bitwise_fraction=float(np.mean(bitwise)) if bitwise.size else 1.0)
