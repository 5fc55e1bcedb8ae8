"""The CPU build of the render path under ASan + UBSan: `make
build/san_asan/driver` links the hostsim backend, the C ABI, host ingest and the
CPU oracle with -fsanitize=address,undefined, and tests/native/sanitize_driver.cpp
drives single / multi-device renders, failure injection, the material sweep,
ingest, pixels and intersect, each checked bitwise against the oracle. Any
sanitizer report fails the run (halt_on_error). The TSan twin (`make sanitize`)
is slower to build; its log is committed under profiles/r04_sanitize_tsan.log."""
from __future__ import annotations

import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_asan_ubsan_driver_clean():
    subprocess.run(["make", "-C", REPO, "-s", "build/san_asan/driver"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="4")
    r = subprocess.run([os.path.join(REPO, "build", "san_asan", "driver"), os.path.join(REPO, "scenes"), "asan"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "asan: 0 failure(s)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
