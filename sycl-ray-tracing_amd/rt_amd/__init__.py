"""rt_amd — Python mirror of the reference host API over librt_hip.so.

Names, argument meaning and mutation semantics follow the reference
(TomClabault/SYCL-ray-tracing @ 2024-08-07) so tests read like its own:

  Camera / presets     include/camera.h:10-40, source/camera.cpp:3-8
  Image                include/image.h:25-178  (RGBA float32, black = (0,0,0,1))
  parse_obj            source/utils.cpp:16-98  -> ParsedOBJ (include/parsed_obj.h)
  compute_env_map_cdf  source/utils.cpp:126-142
  read_image_float     source/utils.cpp:100-124  (Radiance .hdr, stb_image 2.28 decode, flipY)
  write_image_png      source/image_io.cpp:165-182
  BVH                  include/bvh.h:211-280, source/bvh.cpp:19-37
  RenderKernel         include/render_kernel.h:21-96
     render()            mutates the image buffer in place (render_kernel.cpp:189-211)
     ray_trace_pixel()   one pixel (render_kernel.cpp:75-181)

All compute runs in the native library (C++ host preparation + gfx950 HIP
kernels); this module only moves numpy buffers across the C ABI.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from ._capi import (RT_ERR_ARG, RT_ERR_HIP, RT_ERR_IO, RT_ERR_NODEV, RT_ERR_STATE, RT_OK,  # noqa: F401
                    RtError, check, lib, ptr)

__all__ = ["Camera", "Image", "ParsedOBJ", "parse_obj", "compute_env_map_cdf", "luminance_of_pixels", "BVH",
           "RenderKernel", "RtError", "octree_dump", "make_materials", "read_image_float", "write_image_png",
           "image_to_rgba8"]


# ------------------------------------------------------------------ camera
class Camera:
    """view_matrix: 4x4 float32 row-major (Transform::m); fov_dist (camera.h:38-40)."""

    PRESETS = ("default", "cornell", "ganesha", "ite", "dragon", "mis")

    def __init__(self, view_matrix=None, fov_dist=None):
        if view_matrix is None:
            c = Camera.preset("default")
            view_matrix, fov_dist = c.view_matrix, c.fov_dist
        self.view_matrix = np.ascontiguousarray(view_matrix, dtype=np.float32).reshape(4, 4)
        self.fov_dist = float(np.float32(fov_dist))

    @staticmethod
    def preset(name: str) -> "Camera":
        v = np.zeros(16, dtype=np.float32)
        f = ctypes.c_float()
        check(lib(), lib().rt_camera_preset(name.encode(), ptr(v), ctypes.byref(f)), None, f"camera preset {name}")
        return Camera(v, f.value)

    def as17(self) -> np.ndarray:
        return np.concatenate([self.view_matrix.ravel(), [np.float32(self.fov_dist)]]).astype(np.float32)


# ------------------------------------------------------------------- image
class Image:
    """Image(w, h[, color]) — pixels is a [h, w, 4] float32 array (RGBA)."""

    def __init__(self, width: int, height: int, color=(0.0, 0.0, 0.0, 1.0), pixels=None):
        if pixels is not None:
            self.pixels = np.ascontiguousarray(pixels, dtype=np.float32).reshape(height, width, 4)
        else:
            self.pixels = np.empty((height, width, 4), dtype=np.float32)
            self.pixels[...] = np.asarray(color, dtype=np.float32)
        self.width, self.height = width, height

    @staticmethod
    def from_rgb(rgb: np.ndarray, alpha: float = 0.0) -> "Image":
        """Like Utils::read_image_float (utils.cpp:100-124): alpha forced to 0."""
        h, w = rgb.shape[:2]
        px = np.empty((h, w, 4), dtype=np.float32)
        px[..., :3] = rgb[..., :3]
        px[..., 3] = alpha
        return Image(w, h, pixels=px)

    def data(self) -> np.ndarray:
        return self.pixels


def luminance_of_pixels(img: Image) -> np.ndarray:
    lum = np.empty(img.width * img.height, dtype=np.float32)
    cdf = np.empty_like(lum)
    check(lib(), lib().rt_env_luminance_cdf(ptr(img.pixels), img.width, img.height, 4, ptr(lum), ptr(cdf)))
    return lum


def compute_env_map_cdf(img: Image) -> np.ndarray:
    lum = np.empty(img.width * img.height, dtype=np.float32)
    cdf = np.empty_like(lum)
    check(lib(), lib().rt_env_luminance_cdf(ptr(img.pixels), img.width, img.height, 4, ptr(lum), ptr(cdf)))
    return cdf


def read_image_float(filepath: str, flipY: bool = True) -> Image:
    """Utils::read_image_float (utils.cpp:100-124) for Radiance .hdr files:
    RGB decoded like stb_image 2.28, alpha 0, rows flipped when flipY."""
    L_ = lib()
    w, h = ctypes.c_int(), ctypes.c_int()
    check(L_, L_.rt_read_hdr(filepath.encode(), int(flipY), ctypes.byref(w), ctypes.byref(h), None), None,
          f"read_image_float({filepath})")
    img = Image(w.value, h.value)
    check(L_, L_.rt_read_hdr(filepath.encode(), int(flipY), ctypes.byref(w), ctypes.byref(h), ptr(img.pixels)), None,
          f"read_image_float({filepath})")
    return img


def image_to_rgba8(img: Image) -> np.ndarray:
    """write_image_png's 8-bit conversion (image_io.cpp:170-177), no flip: [h, w, 4] uint8."""
    out = np.empty((img.height, img.width, 4), dtype=np.uint8)
    check(lib(), lib().rt_image_to_rgba8(ptr(img.pixels), img.width * img.height, ptr(out)), None, "image_to_rgba8")
    return out


def write_image_png(image: Image, filename: str, flipY: bool = True) -> bool:
    """write_image_png (image_io.cpp:165-182): False for an empty image."""
    if image.width * image.height == 0:
        return False
    check(lib(), lib().rt_write_png(filename.encode(), ptr(image.pixels), image.width, image.height, int(flipY)), None,
          f"write_image_png({filename})")
    return True


# --------------------------------------------------------------------- OBJ
@dataclass
class ParsedOBJ:
    triangles: np.ndarray                  # [N, 9] float32
    materials: np.ndarray                  # [M, 10] float32
    emissive_triangle_indices: np.ndarray  # [E] int32
    material_indices: np.ndarray           # [N] int32
    spheres: np.ndarray = field(default_factory=lambda: np.zeros((0, 5), np.float32))


def parse_obj(path: str) -> ParsedOBJ:
    L_ = lib()
    m = ctypes.c_void_p()
    check(L_, L_.rt_mesh_load(path.encode(), ctypes.byref(m)), None, f"parse_obj({path})")
    try:
        nt, nm, ne = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        L_.rt_mesh_counts(m, ctypes.byref(nt), ctypes.byref(nm), ctypes.byref(ne))
        tris = np.empty((nt.value, 9), np.float32)
        mi = np.empty(nt.value, np.int32)
        mats = np.empty((nm.value, 10), np.float32)
        em = np.empty(ne.value, np.int32)
        L_.rt_mesh_copy(m, ptr(tris), ptr(mi), ptr(mats), ptr(em))
    finally:
        L_.rt_mesh_free(m)
    return ParsedOBJ(tris, mats, em, mi)


def make_materials(rows) -> np.ndarray:
    """rows of (emission rgb, diffuse rgb, metalness, roughness) -> [M,10] SimpleMaterial buffer."""
    out = []
    for e, d, metal, rough in rows:
        out.append([*e, 1.0, *d, 1.0, metal, rough])
    return np.asarray(out, dtype=np.float32)


def octree_dump(triangles: np.ndarray, max_depth: int = 32, leaf_max: int = 8) -> bytes:
    tris = np.ascontiguousarray(triangles, dtype=np.float32).reshape(-1, 9)
    L_ = lib()
    n = L_.rt_octree_dump(ptr(tris), tris.shape[0], max_depth, leaf_max, None, 0)
    buf = ctypes.create_string_buffer(n)
    L_.rt_octree_dump(ptr(tris), tris.shape[0], max_depth, leaf_max, buf, n)
    return buf.raw


class BVH:
    """BVH(triangles, max_depth=32, leaf_max_obj_count=8) (bvh.cpp:19-37).

    The octree itself is built natively when a RenderKernel binds it. Pass
    ``preorder=`` (a pre-order walk of a reference BVH::_root) to bind an
    externally built tree instead."""

    def __init__(self, triangles, max_depth: int = 32, leaf_max_obj_count: int = 8, preorder: bytes | None = None):
        self.triangles = triangles
        self.max_depth = max_depth
        self.leaf_max_obj_count = leaf_max_obj_count
        self.preorder = preorder


# -------------------------------------------------------------- RenderKernel
class RenderKernel:
    """RenderKernel(width, height, render_samples, max_bounces, image_buffer,
    triangles, materials, emissive_triangle_indices, materials_indices,
    analytic_spheres, bvh, skysphere, env_map_cdf) — render_kernel.h:24-46.

    device: a HIP ordinal, or a sequence of them for one context over several
    GPUs (rt_create_multi: rows sharded over the devices, RCCL scatter/gather
    through the first). Like the reference, which keeps a reference to the
    material vector (render_kernel.h:81-93), a render picks up in-place edits
    of `materials_buffer` (rt_set_materials: no BVH rebuild); the triangles,
    BVH and sky are bound at construction."""

    def __init__(self, width, height, render_samples, max_bounces, image_buffer: Image, triangle_buffer,
                 materials_buffer, emissive_triangle_indices_buffer, materials_indices_buffer, analytic_spheres_buffer,
                 bvh: BVH, skysphere: Image, env_map_cdf, device=0, hostsim: bool = False, loopback: bool = False,
                 rccl_clique: bool = False):
        self.L = lib(hostsim)
        self.width, self.height = int(width), int(height)
        self.render_samples, self.max_bounces = int(render_samples), int(max_bounces)
        self.frame_buffer = image_buffer
        h = ctypes.c_void_p()
        if isinstance(device, (list, tuple)):
            # loopback (tests / rehearsals only): the list may repeat a GPU, shards move by device copies
            ids = np.ascontiguousarray(device, dtype=np.int32)
            # rccl_clique (tests only): the RCCL driver even for one device (rt_test_create_multi_rccl)
            create = (self.L.rt_create_multi_loopback if loopback else
                      self.L.rt_test_create_multi_rccl if rccl_clique else self.L.rt_create_multi)
            check(self.L, create(ids.shape[0], ptr(ids), ctypes.byref(h)), None, "rt_create_multi")
        else:
            check(self.L, self.L.rt_create(int(device), ctypes.byref(h)), None, "rt_create")
        self.ctx = h
        self.n_devices = int(self.L.rt_device_count(self.ctx))
        tris = np.ascontiguousarray(triangle_buffer, dtype=np.float32).reshape(-1, 9)
        mats = np.ascontiguousarray(materials_buffer, dtype=np.float32).reshape(-1, 10)
        self.materials_buffer = materials_buffer if isinstance(materials_buffer, np.ndarray) else mats
        self._mats_sent = mats.copy()
        em = np.ascontiguousarray(emissive_triangle_indices_buffer, dtype=np.int32)
        mi = np.ascontiguousarray(materials_indices_buffer, dtype=np.int32)
        sph = np.ascontiguousarray(analytic_spheres_buffer if analytic_spheres_buffer is not None else np.zeros((0, 5)),
                                   dtype=np.float32).reshape(-1, 5)
        check(self.L, self.L.rt_set_scene(self.ctx, ptr(tris), tris.shape[0], ptr(mi), mi.shape[0], ptr(mats),
                                          mats.shape[0], ptr(em), em.shape[0], ptr(sph), sph.shape[0]), self.ctx,
              "rt_set_scene")
        if bvh.preorder is not None:
            buf = ctypes.create_string_buffer(bvh.preorder, len(bvh.preorder))
            check(self.L, self.L.rt_set_bvh_preorder(self.ctx, buf, len(bvh.preorder)), self.ctx, "rt_set_bvh_preorder")
        else:
            check(self.L, self.L.rt_build_bvh(self.ctx, bvh.max_depth, bvh.leaf_max_obj_count), self.ctx,
                  "rt_build_bvh")
        cdf = None if env_map_cdf is None else np.ascontiguousarray(env_map_cdf, dtype=np.float32)
        check(self.L, self.L.rt_set_env(self.ctx, ptr(skysphere.pixels), skysphere.width, skysphere.height, 4,
                                        ptr(cdf)), self.ctx, "rt_set_env")
        self.set_camera(Camera())

    def __del__(self):
        if getattr(self, "ctx", None):
            self.L.rt_destroy(self.ctx)
            self.ctx = None

    def set_camera(self, camera: Camera):
        self.camera = camera
        check(self.L, self.L.rt_set_camera(self.ctx, ptr(camera.view_matrix), camera.fov_dist), self.ctx,
              "rt_set_camera")

    def _sync_materials(self):
        """Push the material table again if the caller edited it in place."""
        m = np.ascontiguousarray(self.materials_buffer, dtype=np.float32).reshape(-1, 10)
        if m.shape != self._mats_sent.shape or not np.array_equal(m.view(np.uint32), self._mats_sent.view(np.uint32)):
            self.set_materials(m)

    def set_materials(self, materials):
        """rt_set_materials: a new material table for the bound scene (the cfg5 sweep)."""
        m = np.ascontiguousarray(materials, dtype=np.float32).reshape(-1, 10)
        check(self.L, self.L.rt_set_materials(self.ctx, ptr(m), m.shape[0]), self.ctx, "rt_set_materials")
        self._mats_sent = m.copy()

    def render(self):
        self._sync_materials()
        fb = self.frame_buffer.pixels
        assert fb.flags.c_contiguous and fb.dtype == np.float32 and fb.shape == (self.height, self.width, 4)
        check(self.L, self.L.rt_render(self.ctx, self.width, self.height, self.render_samples, self.max_bounces,
                                       ptr(fb)), self.ctx, "rt_render")

    def render_device(self, d_fb: int, row_offset: int = 0, row_stride: int = 1, stream: int | None = None):
        """Render into a device buffer (e.g. a torch tensor's data_ptr()); no host copies."""
        self._sync_materials()
        check(self.L, self.L.rt_render_device(self.ctx, self.width, self.height, self.render_samples,
                                              self.max_bounces, ctypes.c_void_p(d_fb), row_offset, row_stride,
                                              ctypes.c_void_p(stream) if stream else None), self.ctx,
              "rt_render_device")

    def render_variants(self, materials, frames=None, device_ptrs=None, row_offset: int = 0, row_stride: int = 1):
        """rt_render_variants: the material sweep as replicas. `materials` is
        [n_variants, n_materials, 10] (or a list of [n_materials, 10] tables); variant v
        renders rows row_offset + j*row_stride of its own frame on device v mod N of the
        context, no exchange between devices. Output into `frames` (host float32
        [n_variants, rows, W, 4], read-modify-written like render()), or into
        `device_ptrs[v]` (device buffers of rows*W*4 floats, each on device v mod N).
        Returns `frames` (host mode). The bound material table is untouched."""
        tabs = np.ascontiguousarray(np.stack([np.asarray(m, np.float32).reshape(-1, 10) for m in materials]),
                                    dtype=np.float32)
        n_var, n_mats = tabs.shape[0], tabs.shape[1]
        rows = len(range(row_offset, self.height, row_stride))
        self._sync_materials()
        if device_ptrs is not None:
            assert len(device_ptrs) == n_var
            arr = (ctypes.c_void_p * n_var)(*[ctypes.c_void_p(int(p)) for p in device_ptrs])
            fb_p, d_p = None, ctypes.cast(arr, ctypes.c_void_p)
        else:
            if frames is None:
                frames = np.zeros((n_var, rows, self.width, 4), np.float32)
                frames[..., 3] = 1.0  # (Image's default alpha, as Image(w, h))
            assert frames.flags.c_contiguous and frames.dtype == np.float32 and frames.shape == (n_var, rows,
                                                                                                  self.width, 4)
            fb_p, d_p = ptr(frames), None
        check(self.L, self.L.rt_render_variants(self.ctx, self.width, self.height, self.render_samples,
                                                self.max_bounces, n_var, ptr(tabs), n_mats, row_offset, row_stride,
                                                fb_p, d_p), self.ctx, "rt_render_variants")
        return frames

    def ray_trace_pixels(self, xy) -> None:
        self._sync_materials()
        xy = np.ascontiguousarray(xy, dtype=np.int32).reshape(-1, 2)
        fb = self.frame_buffer.pixels
        rgba = np.ascontiguousarray(fb[xy[:, 1], xy[:, 0]])
        check(self.L, self.L.rt_render_pixels(self.ctx, self.width, self.height, self.render_samples,
                                              self.max_bounces, ptr(xy), xy.shape[0], ptr(rgba)), self.ctx,
              "rt_render_pixels")
        fb[xy[:, 1], xy[:, 0]] = rgba

    def ray_trace_pixel(self, x: int, y: int) -> None:
        self.ray_trace_pixels(np.array([[x, y]], dtype=np.int32))

    def intersect(self, rays) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        out = np.zeros((rays.shape[0], 11), dtype=np.int32)
        check(self.L, self.L.rt_intersect(self.ctx, ptr(rays), rays.shape[0], ptr(out)), self.ctx, "rt_intersect")
        return out

    def set_use_bvh(self, use_bvh: bool = True):
        """USE_BVH (render_kernel.h:13): False switches INTERSECT_SCENE to the
        brute-force intersect_scene loop (render_kernel.cpp:453-483)."""
        check(self.L, self.L.rt_set_intersect_mode(self.ctx, 1 if use_bvh else 0), self.ctx, "rt_set_intersect_mode")

    def test_fail_device(self, device: int = -1):
        """Tests only (rt_test_fail_device): later multi-device renders fail `device` (-1: off)."""
        check(self.L, self.L.rt_test_fail_device(self.ctx, int(device)), self.ctx, "rt_test_fail_device")

    def test_schedule(self, **params):
        """Tests and measurement tools only (rt_test_schedule): override wavefront-schedule
        parameters of the later renders, e.g. test_schedule(lanes=2, tail_paths=0,
        force_fallback=7); reset=1 restores the product's schedule. No parameter changes
        a result."""
        for k, v in params.items():
            check(self.L, self.L.rt_test_schedule(self.ctx, k.encode(), float(v)), self.ctx, "rt_test_schedule")

    def test_walk_log(self, min_calls: int, capacity: int = 1 << 20, sample_every: int = 1):
        """Tests and diagnostics only (rt_test_walk_log): stats renders record every walk of at
        least min_calls quad_visit calls (0: off), or every sample_every-th by a hash."""
        check(self.L, self.L.rt_test_walk_log(self.ctx, int(min_calls), int(sample_every), int(capacity)), self.ctx,
              "rt_test_walk_log")
        self._wlog_cap = int(capacity)

    def walk_log(self) -> tuple[np.ndarray, int]:
        """The last stats render's walk records as a structured array, and how many walks
        qualified (include/rt_hip.h rt_test_walk_log)."""
        cap = getattr(self, "_wlog_cap", 0)
        raw = np.zeros((max(cap, 1), 12), np.float32)
        total = int(self.L.rt_test_walk_log_read(self.ctx, ptr(raw), cap))
        if total < 0:
            check(self.L, total, self.ctx, "rt_test_walk_log_read")
        raw = raw[:min(total, cap)]
        iv = raw.view(np.int32)
        dt = np.dtype([("o", np.float32, 3), ("kind", np.int32), ("where", np.int32), ("d", np.float32, 3),
                       ("calls", np.int32), ("t", np.float32), ("tri", np.int32), ("iter", np.int32), ("slot", np.int32)])
        out = np.zeros(raw.shape[0], dt)
        out["o"], out["kind"], out["where"] = raw[:, 0:3], iv[:, 3] & 0xff, iv[:, 3] >> 8
        out["d"], out["calls"], out["t"] = raw[:, 4:7], iv[:, 7], raw[:, 8]
        out["tri"], out["iter"], out["slot"] = iv[:, 9], iv[:, 10], iv[:, 11]
        return out, total

    def set_stats(self, on):
        """True / 1: counters of the next renders; 2: the same with unpaired occlusion walks
        (the box tests a walk must make: same answers); False / 0: off."""
        self.L.rt_set_stats(self.ctx, int(on) if not isinstance(on, bool) else (1 if on else 0))

    def stats(self) -> dict:
        """Counters of the last render (rt_set_stats(True) first), by name."""
        from ._capi import STAT_NAMES
        n = len(STAT_NAMES)
        out = np.zeros(2 * n, dtype=np.uint64)
        self.L.rt_get_stats(self.ctx, ptr(out), 2 * n)
        d = {k: int(v) for k, v in zip(STAT_NAMES, out[:n])}
        d.update({"tail_" + k: int(v) for k, v in zip(STAT_NAMES, out[n:])})  # the tail kernel's share
        return d

    def kernel_timing(self, enable: int = -1):
        """Per-kernel-class GPU time (HIP events around every launch) since
        timing was last enabled: {class: (total_ms, launches)} for the
        query kernel (k_trace), the path step (k_step, with the exact-walk
        roles) and "other" (the tail kernel k_tail), summed over the
        context's devices. enable=1/0
        turns timing on/off and resets the totals; -1 only reads."""
        ms = np.zeros(3, dtype=np.float64)
        n = np.zeros(3, dtype=np.int64)
        check(self.L, self.L.rt_device_kernel_timing(self.ctx, enable, ptr(ms), ptr(n)), self.ctx, "kernel_timing")
        return {k: (float(a), int(b)) for k, a, b in zip(("trace", "step", "other"), ms, n)}

    def set_lanes(self, lanes: int):
        """Wavefront lanes (streams) per render on every device (1: launches serialized; 0: auto,
        4 for launches of at most 1.5 M pixels, else 3)."""
        check(self.L, self.L.rt_device_set_lanes(self.ctx, int(lanes)), self.ctx, "rt_device_set_lanes")

    def last_iterations(self) -> int:
        return int(self.L.rt_device_last_iterations(self.ctx))

    def exact_handovers(self, reset: bool = False) -> int:
        """Queries the search-BVH walks handed to the exact octree walk in every render since
        the last reset (GPU build; waits for the device): ~2e-6 per sample on cfg2."""
        import ctypes
        v = ctypes.c_ulonglong(0)
        check(self.L, self.L.rt_device_exact_handovers(self.ctx, ctypes.byref(v), 1 if reset else 0), self.ctx,
              "rt_device_exact_handovers")
        return int(v.value)

    def last_kernel_ms(self) -> float:
        return float(self.L.rt_last_kernel_ms(self.ctx))

    def device_last_kernel_ms(self) -> float:
        return float(self.L.rt_device_last_kernel_ms(self.ctx))

    def bvh_info(self) -> dict:
        info = np.zeros(5, dtype=np.int64)
        check(self.L, self.L.rt_bvh_info(self.ctx, ptr(info)), self.ctx, "rt_bvh_info")
        return dict(octree_nodes=int(info[0]), gpu_records=int(info[1]), triangles=int(info[2]),
                    max_depth=int(info[3]), gpu_bytes=int(info[4]))

    def bvh_dump(self) -> bytes:
        n = self.L.rt_bvh_dump(self.ctx, None, 0)
        buf = ctypes.create_string_buffer(n)
        self.L.rt_bvh_dump(self.ctx, buf, n)
        return buf.raw
