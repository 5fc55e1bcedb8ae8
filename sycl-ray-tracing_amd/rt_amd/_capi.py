"""ctypes bindings for the C ABI in include/rt_hip.h.

``lib()`` loads the product library ``lib/librt_hip.so`` (gfx950 kernels).
There is no CPU fallback: creating a context without a HIP device raises.
``lib(hostsim=True)`` loads ``lib/librt_hostsim.so`` — the same device code
compiled for the host — which only the CPU test-suite uses to validate the
kernel algorithm in a GPU-less container.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_DIR, "lib")
PRODUCT = os.environ.get("RT_HIP_LIB") or os.path.join(LIB_DIR, "librt_hip.so")  # (override: debug builds)
HOSTSIM = os.environ.get("RT_HOSTSIM_LIB") or os.path.join(LIB_DIR, "librt_hostsim.so")  # (override: study builds)

# every symbol declared in include/rt_hip.h (tests check the export table)
EXPORTS = [
    "rt_create", "rt_destroy", "rt_last_error", "rt_version", "rt_build_id", "rt_set_scene", "rt_build_bvh",
    "rt_set_bvh_preorder", "rt_bvh_dump", "rt_bvh_info", "rt_set_env", "rt_set_camera", "rt_render",
    "rt_render_device", "rt_render_pixels", "rt_intersect", "rt_set_stats", "rt_get_stats", "rt_last_kernel_ms",
    "rt_mesh_load", "rt_mesh_counts", "rt_mesh_copy", "rt_mesh_free", "rt_camera_preset", "rt_env_luminance_cdf",
    "rt_octree_dump", "rt_read_hdr", "rt_write_png", "rt_image_to_rgba8",
    "rt_set_intersect_mode", "rt_create_multi", "rt_device_count", "rt_set_materials", "rt_render_variants",
    "rt_create_multi_loopback", "rt_test_create_multi_rccl", "rt_test_fail_device", "rt_test_schedule", "rt_test_walk_log",
    "rt_test_walk_log_read", "rt_test_obj_parallel_min",
]

# return codes (include/rt_hip.h)
RT_OK, RT_ERR_ARG, RT_ERR_HIP, RT_ERR_STATE, RT_ERR_IO, RT_ERR_NODEV = 0, -1, -2, -3, -4, -5

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float

_SIGS = {
    "rt_create": (I, [I, ctypes.POINTER(P)]),
    "rt_create_multi": (I, [I, P, ctypes.POINTER(P)]),
    "rt_create_multi_loopback": (I, [I, P, ctypes.POINTER(P)]),
    "rt_test_create_multi_rccl": (I, [I, P, ctypes.POINTER(P)]),
    "rt_test_fail_device": (I, [P, I]),
    "rt_test_schedule": (I, [P, ctypes.c_char_p, ctypes.c_double]),
    "rt_test_walk_log": (I, [P, I, I, I]),
    "rt_test_walk_log_read": (L, [P, P, L]),
    "rt_test_obj_parallel_min": (I, [L]),
    "rt_device_count": (I, [P]),
    "rt_set_materials": (I, [P, P, I]),
    "rt_destroy": (None, [P]),
    "rt_last_error": (ctypes.c_char_p, [P]),
    "rt_version": (I, []),
    "rt_build_id": (ctypes.c_char_p, []),
    "rt_set_scene": (I, [P, P, I, P, I, P, I, P, I, P, I]),
    "rt_build_bvh": (I, [P, I, I]),
    "rt_set_bvh_preorder": (I, [P, P, L]),
    "rt_bvh_dump": (L, [P, P, L]),
    "rt_bvh_info": (I, [P, P]),
    "rt_set_env": (I, [P, P, I, I, I, P]),
    "rt_set_camera": (I, [P, P, F]),
    "rt_render": (I, [P, I, I, I, I, P]),
    "rt_render_device": (I, [P, I, I, I, I, P, I, I, P]),
    "rt_render_pixels": (I, [P, I, I, I, I, P, I, P]),
    "rt_render_variants": (I, [P, I, I, I, I, I, P, I, I, I, P, P]),
    "rt_intersect": (I, [P, P, I, P]),
    "rt_set_stats": (I, [P, I]),
    "rt_set_intersect_mode": (I, [P, I]),
    "rt_get_stats": (I, [P, P, I]),
    "rt_last_kernel_ms": (ctypes.c_double, [P]),
    "rt_mesh_load": (I, [ctypes.c_char_p, ctypes.POINTER(P)]),
    "rt_mesh_counts": (I, [P, P, P, P]),
    "rt_mesh_copy": (I, [P, P, P, P, P]),
    "rt_mesh_free": (None, [P]),
    "rt_camera_preset": (I, [ctypes.c_char_p, P, P]),
    "rt_env_luminance_cdf": (I, [P, I, I, I, P, P]),
    "rt_octree_dump": (L, [P, I, I, I, P, L]),
    "rt_read_hdr": (I, [ctypes.c_char_p, I, P, P, P]),
    "rt_write_png": (I, [ctypes.c_char_p, P, I, I, I]),
    "rt_image_to_rgba8": (I, [P, L, P]),
    # product-only extras
    "rt_device_libm": (I, [I, I, P, P, P, I]),
    "rt_device_last_kernel_ms": (ctypes.c_double, [P]),
    "rt_device_kernel_timing": (I, [P, I, P, P]),
    "rt_device_set_lanes": (I, [P, I]),
    "rt_device_last_iterations": (I, [P]),
    "rt_device_exact_handovers": (I, [P, P, I]),
    "rt_device_queries": (I, [P, I, P, I, I, P, P, P]),
    # hostsim-only extra
    "rt_hostsim_heap_order": (I, [P, I, P, P]),
    "rt_hostsim_fast_queries": (I, [P, P, I, P, P]),
}

STAT_NAMES = ["rays", "vol", "tri", "leaf", "mat", "env", "cdf", "heap_slow", "any_rays", "any_vol", "any_tri",
              "any_leaf", "verify", "fallback", "quad_visits", "wave_slots", "refills", "drain_slots", "drain_visits",
              "steps"]

_libs: dict = {}


class RtError(RuntimeError):
    pass


def lib(hostsim: bool = False):
    path = HOSTSIM if hostsim else PRODUCT
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RtError(f"{path} is not built: run `make` (or __graft_entry__.build()) first")
    L_ = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L_, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _libs[path] = L_
    return L_


def check(L_, rc: int, ctx=None, what: str = ""):
    if rc != 0:
        msg = L_.rt_last_error(ctx)
        raise RtError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


def ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)
