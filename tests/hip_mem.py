"""Minimal device-memory helper over the HIP runtime (ctypes), for GPU
tests that exercise the device-pointer entry points without torch."""
from __future__ import annotations

import ctypes

import numpy as np

_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        _hip.hipFree.argtypes = [ctypes.c_void_p]
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipDeviceSynchronize.argtypes = []
    return _hip


class DeviceBuffer:
    H2D, D2H = 1, 2

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        assert hip().hipMalloc(ctypes.byref(p), nbytes) == 0
        self.ptr, self.nbytes = p.value, nbytes

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        assert hip().hipMemcpy(self.ptr, a.ctypes.data, a.nbytes, self.H2D) == 0

    def download(self, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype)
        assert hip().hipDeviceSynchronize() == 0
        assert hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, self.D2H) == 0
        return out

    def __del__(self):
        if getattr(self, "ptr", None):
            hip().hipFree(self.ptr)
            self.ptr = None
