"""Host-side numerics checks of the arithmetic identities the kernel relies
on (the same checks run on gfx950 in test_gpu_parity.py)."""
from __future__ import annotations

import numpy as np


def division_cases(n: int, seed: int = 1):
    """(a, den) float32 pairs: random magnitudes over the whole exponent
    range, slab-like values, exact quotients, denormals, near-overflow."""
    rng = np.random.default_rng(seed)
    k = n // 4
    a1 = (rng.standard_normal(k) * 2.0 ** rng.integers(-140, 120, k)).astype(np.float32)
    d1 = (rng.standard_normal(k) * 2.0 ** rng.integers(-140, 120, k)).astype(np.float32)
    a2 = rng.uniform(-50, 50, k).astype(np.float32)                     # (d_near - numer)
    d2 = rng.uniform(-1, 1, k).astype(np.float32)                       # n . dir
    m = rng.integers(1, 2 ** 24, k).astype(np.float32)
    d3 = rng.integers(1, 2 ** 12, k).astype(np.float32)
    a3 = (m * d3).astype(np.float32)                                    # exact quotients
    bits = rng.integers(0, 2 ** 32, k, dtype=np.uint64).astype(np.uint32)
    a4 = bits.view(np.float32)
    d4 = rng.integers(0, 2 ** 32, k, dtype=np.uint64).astype(np.uint32).view(np.float32)
    special_a = np.array([0.0, -0.0, 1.0, 1e-45, 3e38, -3e38, 1e-38, 7.0, 1.0, 2.0], np.float32)
    special_d = np.array([1.0, 3.0, 1e-45, 1e-45, 1e-3, 7e-3, 3.0, 1.5e-45, -3e38, 3.4e38], np.float32)
    a = np.concatenate([a1, a2, a3, a4, special_a])
    d = np.concatenate([d1, d2, d3, d4, special_d])
    ok = np.isfinite(a) & np.isfinite(d) & (d != 0)
    return np.ascontiguousarray(a[ok]), np.ascontiguousarray(d[ok])


def test_slab_division_identity_host():
    """float(double(a) * (1/double(d))) is the correctly rounded a/d for
    finite floats (rt_trace.h slab_div); numpy's float32 divide is IEEE."""
    a, d = division_cases(2_000_000)
    with np.errstate(all="ignore"):
        got = (a.astype(np.float64) * (1.0 / d.astype(np.float64))).astype(np.float32)
        want = a / d
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), (a[~same][:4], d[~same][:4], got[~same][:4], want[~same][:4])


REPO = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


def _native(name):
    import os
    p = os.path.join(REPO, "build", name)
    if not os.path.exists(p):
        import subprocess
        subprocess.run(["make", "-C", REPO, f"build/{name}"], check=True, capture_output=True)
    return p


def test_cdf_fence_search_matches_reference_loop():
    """The counting env-CDF search (rt_trace.h fence_count) returns the
    reference's binary-search result (render_kernel.cpp:532-567) on flat runs,
    ties, out-of-range, +-inf and NaN values, and the host refuses fence
    tables for NaN / decreasing CDFs (tests/native/cdf_check.cpp)."""
    import subprocess
    r = subprocess.run([_native("cdf_check")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


def test_libm_restatement_sampled():
    """rt_libm.h against this host's glibc 2.35 on every 4099th float input
    (the exhaustive run is tests/native/libm_check.cpp with stride 1)."""
    import subprocess
    r = subprocess.run([_native("libm_check"), "4099"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
