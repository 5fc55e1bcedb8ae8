"""Shared pytest setup: the `gpu` marker, import paths, scene fixtures."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the gfx950 product library)")
    config.addinivalue_line("markers", "slow: minutes of CPU work (dragon stand-in scene)")


import golden_io as gio  # noqa: E402
import scenes  # noqa: E402


@pytest.fixture(scope="session")
def manifest():
    import json
    with open(os.path.join(gio.GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def cameras():
    z = np.load(os.path.join(gio.GOLDEN, "cameras.npz"))
    return {k: z[k] for k in z.files}


_parsed = {}


def parsed_scene(name: str):
    """ParsedOBJ of a named scene through the product's own OBJ loader."""
    if name not in _parsed:
        import rt_amd
        _parsed[name] = rt_amd.parse_obj(scenes.scene_path(name))
    return _parsed[name]


def load_golden(name: str):
    z = np.load(os.path.join(gio.GOLDEN, name))
    return {k: z[k] for k in z.files}
