"""Synthetic scene inputs shared by tests, bench and the fixture generator.

Everything here is deterministic (numpy float32 arithmetic, fixed formulas)
so the same bytes are produced in this container and on the GPU box:

* ``make_sky(kind)``       — the SKY-S / SKY-L equirect env maps of SURVEY.md
  §8(d) (the reference HDR ``evening_road_01_puresky_2k.hdr`` is absent).
  Stored exactly as ``Utils::read_image_float`` would leave an HDR in memory
  (reference source/utils.cpp:100-124): row-major RGB, row 0 = the bottom
  row of the picture (flipY), alpha forced to 0 by the consumer.
* ``write_cornell12(path)`` — ``cornell_pbr.obj`` without the shortBox /
  tallBox faces (12 triangles, 2 emissive): BASELINE config 1.
* ``write_dragon_standin(path)`` — procedural 1,000,002-triangle stand-in
  for the absent ``pbrt_dragon.obj``: displaced UV sphere
  (500 x 1000 quads, each split into two triangles) on ``Material.001`` plus
  a ground quad on ``Material.002``, materials from the reference's
  ``pbrt_dragon.mtl``. Vertices are written ``%.6f`` so the file is
  bit-reproducible.
"""
from __future__ import annotations

import os
import shutil
import struct

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")

SKY_SPECS = {
    # kind: (W, H, sun_x0, sun_y0, sun_size)
    "S": (512, 256, 300, 200, 10),
    "L": (2048, 1024, 1200, 800, 24),
}


def make_sky(kind: str = "S") -> np.ndarray:
    """Return float32 array [H, W, 3] (row y = Image row y)."""
    W, H, sx, sy, n = SKY_SPECS[kind]
    y = np.arange(H, dtype=np.float32)[:, None]
    s = (y / np.float32(H)) * np.ones((1, W), dtype=np.float32)
    img = np.empty((H, W, 3), dtype=np.float32)
    img[..., 0] = np.float32(0.3) + np.float32(0.5) * s
    img[..., 1] = np.float32(0.4) + np.float32(0.4) * s
    img[..., 2] = np.float32(0.6) + np.float32(0.4) * s
    img[sy:sy + n, sx:sx + n, :] = np.array([200.0, 180.0, 150.0], dtype=np.float32)
    return img


def write_sky_raw(path: str, kind: str = "S") -> str:
    img = make_sky(kind)
    H, W, _ = img.shape
    with open(path, "wb") as f:
        f.write(struct.pack("<ii", W, H))
        f.write(np.ascontiguousarray(img, dtype="<f4").tobytes())
    return path


def write_cornell12(path: str) -> str:
    src = os.path.join(SCENES, "cornell_pbr.obj")
    out, keep = [], True
    with open(src) as f:
        for line in f:
            if line.startswith("usemtl"):
                keep = line.split()[1] not in ("shortBox.001", "tallBox.001")
            if line.startswith("f ") and not keep:
                continue
            out.append(line)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        f.writelines(out)
    mtl = os.path.join(d, "cornell_pbr.mtl")
    if not os.path.exists(mtl):
        shutil.copy(os.path.join(SCENES, "cornell_pbr.mtl"), mtl)
    return path


def dragon_vertices(n_theta: int = 500, n_phi: int = 1000) -> np.ndarray:
    th = (np.pi * np.arange(n_theta + 1) / n_theta)[:, None]
    ph = (2.0 * np.pi * np.arange(n_phi) / n_phi)[None, :]
    r = 1.5 * (1.0 + 0.08 * np.sin(9.0 * th) * np.cos(13.0 * ph) + 0.03 * np.sin(41.0 * ph + 7.0 * th))
    x = r * np.sin(th) * np.cos(ph)
    y = 1.6 + 0.8 * r * np.cos(th) * np.ones_like(ph)
    z = r * np.sin(th) * np.sin(ph)
    return np.stack([x, y, z], axis=-1).reshape(-1, 3)


def dragon_faces(n_theta: int = 500, n_phi: int = 1000) -> np.ndarray:
    i = np.arange(n_theta)[:, None]
    j = np.arange(n_phi)[None, :]
    jn = (j + 1) % n_phi
    v00 = i * n_phi + j
    v01 = i * n_phi + jn
    v10 = (i + 1) * n_phi + j
    v11 = (i + 1) * n_phi + jn
    # winding chosen so cross(b-a, c-a) points away from the centre
    t1 = np.stack([v00, v11, v10], axis=-1).reshape(-1, 3)
    t2 = np.stack([v00, v01, v11], axis=-1).reshape(-1, 3)
    f = np.empty((t1.shape[0] * 2, 3), dtype=np.int64)
    f[0::2] = t1
    f[1::2] = t2
    return f


def write_dragon_standin(path: str, n_theta: int = 500, n_phi: int = 1000) -> str:
    if os.path.exists(path):
        return path
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    mtl = os.path.join(d, "pbrt_dragon.mtl")
    if not os.path.exists(mtl):
        shutil.copy(os.path.join(SCENES, "pbrt_dragon.mtl"), mtl)
    v = dragon_vertices(n_theta, n_phi)
    f = dragon_faces(n_theta, n_phi) + 1
    nv = v.shape[0]
    ground_v = np.array([[-20.0, 0.0, -20.0], [-20.0, 0.0, 20.0], [20.0, 0.0, 20.0], [20.0, 0.0, -20.0]])
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as fh:
        fh.write("# procedural stand-in for pbrt_dragon.obj (tools/scenes.py)\nmtllib pbrt_dragon.mtl\n")
        fh.write("o dragon_standin\n")
        fh.write("".join("v %.6f %.6f %.6f\n" % tuple(p) for p in v))
        fh.write("usemtl Material.001\n")
        fh.write("".join("f %d %d %d\n" % tuple(t) for t in f))
        fh.write("o ground\n")
        fh.write("".join("v %.6f %.6f %.6f\n" % tuple(p) for p in ground_v))
        fh.write("usemtl Material.002\n")
        fh.write("f %d %d %d\n" % (nv + 1, nv + 2, nv + 3))
        fh.write("f %d %d %d\n" % (nv + 1, nv + 3, nv + 4))
    os.replace(tmp, path)
    return path


def build_dir() -> str:
    d = os.path.join(REPO, "build", "scenes")
    os.makedirs(d, exist_ok=True)
    return d


def scene_path(name: str) -> str:
    """Materialise a named scene under build/scenes and return its OBJ path."""
    d = build_dir()
    if name == "cornell12":
        p = os.path.join(d, "cornell12.obj")
        return p if os.path.exists(p) else write_cornell12(p)
    if name == "cornell":
        return os.path.join(SCENES, "cornell_pbr.obj")
    if name == "mis":
        return os.path.join(SCENES, "MIS.obj")
    if name == "dragon":
        return write_dragon_standin(os.path.join(d, "dragon_standin.obj"))
    if name == "dragon_small":  # 20k-triangle variant for quick tests
        return write_dragon_standin(os.path.join(d, "dragon_small.obj"), 50, 200)
    raise KeyError(name)
