"""Image input / output stages against fixtures made by the reference's own
code (tools/gen_imageio_golden.py: oracle/_ref/io_driver = image_io.cpp +
vendored stb_image 2.28): Utils::read_image_float on Radiance .hdr files
(utils.cpp:100-124) and write_image_png (image_io.cpp:165-182). Host only."""
from __future__ import annotations

import io
import os

import numpy as np
import pytest

import rt_amd

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "imageio.npz"))
HDR = sorted(k[4:] for k in G.files if k.startswith("hdr_") and not k.endswith("_out"))


@pytest.mark.parametrize("name", HDR)
def test_read_hdr_bit_exact(name, tmp_path):
    p = tmp_path / f"{name}.hdr"
    p.write_bytes(G["hdr_" + name].tobytes())
    img = rt_amd.read_image_float(str(p))
    want = G["hdr_" + name + "_out"]
    assert img.pixels.shape == want.shape
    assert (img.pixels.view(np.uint32) == want.view(np.uint32)).all()


def test_read_hdr_no_flip(tmp_path):
    p = tmp_path / "a.hdr"
    p.write_bytes(G["hdr_rle64"].tobytes())
    a = rt_amd.read_image_float(str(p), flipY=False).pixels
    assert (a[::-1].view(np.uint32) == G["hdr_rle64_out"].view(np.uint32)).all()


def test_read_hdr_errors(tmp_path):
    bad = tmp_path / "bad.hdr"
    bad.write_bytes(b"#?RADIANCE\nFORMAT=32-bit_rle_xyze\n\n-Y 1 +X 1\n\0\0\0\0")
    with pytest.raises(rt_amd.RtError):
        rt_amd.read_image_float(str(bad))
    with pytest.raises(rt_amd.RtError):
        rt_amd.read_image_float(str(tmp_path / "missing.hdr"))


def test_rgba8_conversion_matches_reference():
    """x * 255, clamp (NaN passes), float -> uchar as x86-64 g++ converts."""
    img = rt_amd.Image(37, 23, pixels=G["png_in"])
    got = rt_amd.image_to_rgba8(img)
    want = G["png_out"][::-1]  # the file holds the rows flipped
    assert (got == want).all()


def test_write_png_decodes_to_reference_pixels(tmp_path):
    from PIL import Image as PILImage
    img = rt_amd.Image(37, 23, pixels=G["png_in"])
    p = tmp_path / "out.png"
    assert rt_amd.write_image_png(img, str(p))
    got = np.asarray(PILImage.open(io.BytesIO(p.read_bytes())).convert("RGBA"))
    assert (got == G["png_out"]).all()
    assert not rt_amd.write_image_png(rt_amd.Image(0, 0), str(tmp_path / "empty.png"))


def test_env_from_hdr_renders_like_from_array(tmp_path):
    """A decoded .hdr feeds the env CDF exactly like the in-memory image."""
    p = tmp_path / "sky.hdr"
    p.write_bytes(G["hdr_rle64"].tobytes())
    img = rt_amd.read_image_float(str(p))
    cdf = rt_amd.compute_env_map_cdf(img)
    assert cdf.shape == (64 * 16,) and np.all(np.diff(cdf) >= 0) and cdf[-1] > 0
