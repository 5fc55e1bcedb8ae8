"""Host ingest on worker threads: the chunked OBJ parse and
the top-down parallel octree build must give the reference's results exactly —
the parse goldens and octree dumps written by the compiled reference (its own
utils.cpp / bvh.h), the first error in file order, and, for the 1 M-triangle
dragon, the reference's octree dump hash (tests/golden/manifest.json)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import golden_io as gio
import scenes
from conftest import load_golden

import rt_amd


@pytest.fixture
def chunked():
    """rt_test_obj_parallel_min: chunked(True) sends every file through the chunked parse, even
    small ones; chunked(False) restores the default size threshold (also at the test's end)."""
    L_ = rt_amd.lib()

    def set_(on: bool):
        L_.rt_test_obj_parallel_min(0 if on else -1)
    yield set_
    set_(False)


@pytest.mark.parametrize("scene", ["cornell12", "cornell", "mis"])
def test_chunked_parse_matches_reference(scene, chunked):
    chunked(True)  # the chunked path even on small files
    P = rt_amd.parse_obj(scenes.scene_path(scene))
    g = load_golden(f"parse_{scene}.npz")
    np.testing.assert_array_equal(P.triangles.reshape(-1).view(np.uint32), g["tris"].reshape(-1).view(np.uint32))
    np.testing.assert_array_equal(P.material_indices, g["mat_idx"])
    np.testing.assert_array_equal(P.materials.reshape(-1).view(np.uint32), g["mats"].reshape(-1).view(np.uint32))
    np.testing.assert_array_equal(P.emissive_triangle_indices, g["emissive"])


def _obj(tmp_path, lines):
    p = tmp_path / "t.obj"
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def _err(path):
    try:
        rt_amd.parse_obj(path)
        return None
    except rt_amd.RtError as e:
        return str(e)  # (the return code and the message)


def _grid(n):
    out = []
    for i in range(n):
        out += [f"v {i} 0 0", f"v {i} 1 0", f"v {i} 0 1", f"f -3 -2 -1", f"f {3 * i + 1} {3 * i + 2} {3 * i + 3} {3 * i + 1}"]
    return out


@pytest.mark.parametrize("case", ["index_then_vertex", "vertex_then_index", "polygon", "ok", "index_then_parse_same_chunk",
                                  "polygon_with_bad_index", "index_then_mtllib", "mtllib_then_index", "short_face"])
def test_chunked_parse_first_error_in_file_order(case, tmp_path, chunked):
    lines = _grid(400)
    if case == "index_then_vertex":
        lines[100] = "f 1 2 99999"
        lines[1500] = "v 1 2"
    elif case == "vertex_then_index":
        lines[100] = "v 1 2"
        lines[1500] = "f 1 2 99999"
    elif case == "polygon":
        lines[700] = "f 1 2 3 4 5"
    elif case == "index_then_parse_same_chunk":  # (the parse error's chunk skipped its index checks)
        lines[100] = "f 1 2 99999"
        lines[104] = "v 1 2"
    elif case == "polygon_with_bad_index":  # load_obj_serial checks the index range before the vertex count
        lines[700] = "f 1 2 3 99999 5"
    elif case == "index_then_mtllib":
        lines[100] = "f 1 2 99999"
        lines[1500] = "mtllib no_such_library.mtl"
    elif case == "mtllib_then_index":
        lines[100] = "mtllib no_such_library.mtl"
        lines[1500] = "f 1 2 99999"
    elif case == "short_face":
        lines[900] = "f 1 2"
    path = _obj(tmp_path, lines)
    serial = _err(path)
    chunked(True)
    got = _err(path)
    assert got == serial
    if case == "ok":
        assert serial is None
        chunked(False)
        a = rt_amd.parse_obj(path)
        chunked(True)
        b = rt_amd.parse_obj(path)
        np.testing.assert_array_equal(a.triangles, b.triangles)
    else:
        assert serial is not None


@pytest.mark.slow
def test_parallel_octree_dragon_matches_reference(manifest):
    """1,000,002 triangles: above the parallel builder's threshold."""
    P = rt_amd.parse_obj(scenes.scene_path("dragon"))
    dump = rt_amd.octree_dump(P.triangles)
    assert hashlib.sha256(dump).hexdigest() == manifest["scenes"]["dragon"]["octree_sha256"]
