"""Golden fixtures for the image input / output stages (container only: runs
the reference's own code, oracle/_ref/io_driver, built by oracle/ref/Makefile
from /root/reference/source/image_io.cpp and the vendored stb_image 2.28).

Writes tests/golden/imageio.npz:
  hdr_<name>        the .hdr file bytes (synthetic: flat, RLE, non-RLE scanline
                    in RLE mode, header variants, exponent edge cases)
  hdr_<name>_out    what Utils::read_image_float returns for it ([h, w, 4] f32)
  png_in            a float RGBA image with out-of-range, NaN and inf values
  png_out           the RGBA8 pixels of the reference's write_image_png file
                    (decoded with PIL), in file row order (flipY applied)

  python tools/gen_imageio_golden.py
"""
from __future__ import annotations

import io
import os
import struct
import subprocess
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(REPO, "oracle", "_ref", "io_driver")


def rgbe_of(rgb: np.ndarray) -> np.ndarray:
    """float RGB -> RGBE bytes (the usual encoder; any bytes are valid input)."""
    m = rgb.max(axis=-1)
    out = np.zeros(rgb.shape[:-1] + (4,), np.uint8)
    ok = m > 1e-32
    e = np.zeros_like(m, dtype=np.int32)
    mant, ex = np.frexp(m[ok])
    e[ok] = ex
    scale = np.zeros_like(m)
    scale[ok] = mant * 256.0 / m[ok]
    out[..., :3] = np.clip(rgb * scale[..., None], 0, 255).astype(np.uint8)
    out[..., 3] = np.where(ok, e + 128, 0).astype(np.uint8)
    return out


def rle_line(chan: np.ndarray) -> bytes:
    """Radiance RLE of one channel of one scanline (runs of >= 3 equal bytes)."""
    out = bytearray()
    i, n = 0, len(chan)
    while i < n:
        j = i
        while j < n and j - i < 127 and chan[j] == chan[i]:
            j += 1
        if j - i >= 3:
            out += bytes([128 + (j - i), chan[i]])
            i = j
            continue
        k = i
        while k < n and k - i < 128:
            if k + 2 < n and chan[k] == chan[k + 1] == chan[k + 2]:
                break
            k += 1
        out += bytes([k - i]) + bytes(chan[i:k])
        i = k
    return bytes(out)


def hdr_file(rgbe: np.ndarray, mode: str, head: str = "#?RADIANCE", extra: str = "") -> bytes:
    h, w, _ = rgbe.shape
    b = f"{head}\n# synthetic\n{extra}FORMAT=32-bit_rle_rgbe\n\n-Y {h} +X {w}\n".encode()
    if mode == "flat":
        return b + rgbe.tobytes()
    if mode == "rle":
        for y in range(h):
            b += bytes([2, 2, w >> 8, w & 255])
            for c in range(4):
                b += rle_line(rgbe[y, :, c])
        return b
    raise ValueError(mode)


def run(*args):
    subprocess.run([DRIVER, *args], check=True)


def main():
    from PIL import Image as PILImage
    rng = np.random.default_rng(11)
    cases = {}
    # smooth sky with a sun block (runs), width 64
    y, x = np.mgrid[0:16, 0:64].astype(np.float64)
    sky = np.stack([0.3 + 0.5 * y / 16, 0.4 + 0.4 * y / 16, 0.6 + 0.4 * y / 16], -1)
    sky[4:7, 30:40] = (200.0, 180.0, 150.0)
    cases["rle64"] = (hdr_file(rgbe_of(sky), "rle"), )
    # random bytes incl. exponent 0 / 1 / 255, flat storage (width < 8)
    raw = rng.integers(0, 256, (3, 5, 4), dtype=np.uint8)
    raw[0, 0, 3] = 0
    raw[0, 1, 3] = 1
    raw[0, 2, 3] = 255
    cases["flat5"] = (hdr_file(raw, "flat", head="#?RGBE", extra="EXPOSURE=1.0\n"),)
    # width >= 8 but stored flat: the first scanline does not start with (2, 2)
    raw2 = rng.integers(0, 256, (4, 16, 4), dtype=np.uint8)
    raw2[0, 0, 0] = 7
    cases["flat16"] = (hdr_file(raw2, "flat"),)
    # RLE whose 3rd scanline is not run-length encoded (stb_image restarts the flat loop at pixel 1)
    raw3 = rgbe_of(rng.uniform(0, 4, (5, 12, 3)))
    b = hdr_file(raw3[:2], "rle").replace(b"-Y 2 +X 12", b"-Y 5 +X 12")
    b += bytes([9, 9, 9, 130]) + rng.integers(0, 256, 12 * 5 * 4, dtype=np.uint8).tobytes()
    cases["rle_then_flat"] = (b,)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name, (data,) in cases.items():
            fi, fo = os.path.join(td, name + ".hdr"), os.path.join(td, name + ".bin")
            open(fi, "wb").write(data)
            run("hdr", fi, fo)
            blob = open(fo, "rb").read()
            w, h = struct.unpack("ii", blob[:8])
            out["hdr_" + name] = np.frombuffer(data, np.uint8)
            out["hdr_" + name + "_out"] = np.frombuffer(blob[8:], np.float32).reshape(h, w, 4)
        # PNG
        img = rng.uniform(-0.5, 1.5, (23, 37, 4)).astype(np.float32)
        img[..., 3] = 2.5
        img[0, 0, 0] = np.nan
        img[0, 1, 1] = np.inf
        img[0, 2, 2] = -np.inf
        img[1, 0, :3] = (1.0, 0.0, 254.9 / 255)
        img[1, 1, :3] = (0.999999, 1e-9, -0.0)
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.png")
        open(fi, "wb").write(struct.pack("ii", 37, 23) + img.tobytes())
        run("png", fi, fo)
        out["png_in"] = img
        out["png_out"] = np.asarray(PILImage.open(io.BytesIO(open(fo, "rb").read())).convert("RGBA"))
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "imageio.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
