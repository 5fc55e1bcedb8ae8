"""The sample-chain model (tools/chain_sim.c; analysis only): with one runner per
pixel it must reproduce the chain itself (a pixel finishes after the sum of its samples'
bounces), speculation must never finish a pixel later, and a pixel whose samples all take
the predicted bounce count finishes in ~spp / K steps with K runners."""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def _lib(tmp_path):
    so = str(tmp_path / "libchain_sim.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", os.path.join(REPO, "tools", "chain_sim.c"), "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.chain_sim.restype = ctypes.c_long
    L.chain_sim.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                                     ctypes.c_void_p]
    L.lattice_sim.restype = ctypes.c_long
    L.lattice_sim.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                                       ctypes.c_void_p]
    return L


def _window(L, b, k, pred_mode=0):
    n, spp = b.shape
    hist = np.zeros(4096, np.int32)
    fin = np.zeros(n, np.int32)
    work = np.zeros(1, np.int64)
    L.chain_sim(b.ctypes.data, n, spp, 1, k, 0, 1, pred_mode, hist.ctypes.data, 4096, fin.ctypes.data, work.ctypes.data)
    return fin, int(work[0])


def _lattice(L, b, r, t0):
    n, spp = b.shape
    hist = np.zeros(4096, np.int32)
    fin = np.zeros(n, np.int32)
    work = np.zeros(1, np.int64)
    L.lattice_sim(b.ctypes.data, n, spp, r, t0, 8, hist.ctypes.data, 4096, fin.ctypes.data, work.ctypes.data)
    return fin


def test_chain_model(tmp_path):
    L = _lib(tmp_path)
    rng = np.random.default_rng(3)
    b = rng.choice(np.arange(1, 9), size=(64, 32), p=[0.7, 0.1, 0.05, 0.05, 0.03, 0.03, 0.02, 0.02]).astype(np.uint16)
    chain = b.astype(np.int64).sum(1)
    fin1, work1 = _window(L, b, 1)
    np.testing.assert_array_equal(fin1, chain)  # one runner: the chain itself
    assert work1 == chain.sum()
    for k in (2, 4):
        for pm in (0, 1):
            fin, work = _window(L, b, k, pm)
            assert (fin <= chain).all() and work >= chain.sum()
    for r in (1, 4, 16):
        fin = _lattice(L, b, r, 5)
        assert (fin <= chain).all()
    # all samples one bounce: K runners, ~spp / K steps
    ones = np.ones((4, 32), np.uint16)
    fin4, _ = _window(L, ones, 4)
    assert (fin4 <= 32 // 4 + 1).all()
