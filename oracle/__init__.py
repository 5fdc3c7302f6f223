"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- ctypes over oracle/liboracle.so.

PARITY UNPINNED: a clean-room restatement of the reference traversal
(vr_oracle.c cites the reference file:line per function); the reference
itself ships no golden vectors and may not be run here.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, as the checker -- never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_float, c_int, c_int32, c_size_t, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

STORE_VCS, STORE_HASHTABLE = 0, 1
ALGO_LONGESTAXIS, ALGO_ORIGINAL = 0, 1
EMPTY = 1 << 30


class OrCamera(ctypes.Structure):
    _fields_ = [("origin", c_float * 3), ("lower_left", c_float * 3), ("horizontal", c_float * 3),
                ("vertical", c_float * 3), ("forward", c_float * 3)]


class OrLighting(ctypes.Structure):
    _fields_ = [("light_dir", c_float * 3), ("light_color", c_float * 3), ("light_pos", c_float * 3),
                ("use_point_light", c_int32), ("use_shadows", c_int32)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.or_camera_make.argtypes = [POINTER(c_float), POINTER(c_float), POINTER(c_float), c_float, c_float,
                                     POINTER(OrCamera)]
        L.or_camera_make.restype = None
        L.or_lighting_default.argtypes = [POINTER(OrLighting)]
        L.or_lighting_default.restype = None
        L.or_scene_build.argtypes = [c_int, POINTER(c_int32), POINTER(c_uint32), c_size_t, POINTER(c_void_p)]
        L.or_scene_build.restype = c_int
        L.or_scene_free.argtypes = [c_void_p]
        L.or_scene_free.restype = None
        for n in ("or_scene_diameter", "or_scene_region_count"):
            getattr(L, n).argtypes = [c_void_p]
            getattr(L, n).restype = c_uint32
        L.or_scene_min_coord.argtypes = [c_void_p]
        L.or_scene_min_coord.restype = c_int32
        L.or_scene_lookup.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32]
        L.or_scene_lookup.restype = c_uint32
        L.or_scene_cuckoo_table.argtypes = [c_void_p, c_uint32, c_uint32, POINTER(c_int)]
        L.or_scene_cuckoo_table.restype = c_int
        L.or_hash1.argtypes = [c_int32, c_uint32]
        L.or_hash1.restype = c_int32
        L.or_hash2.argtypes = [c_int32, c_uint32]
        L.or_hash2.restype = c_int32
        L.or_cluster_id.argtypes = [c_uint32, c_uint32, c_uint32]
        L.or_cluster_id.restype = c_uint32
        L.or_generate_3d_point.argtypes = [c_uint32, c_uint32, c_uint32]
        L.or_generate_3d_point.restype = c_uint32
        L.or_render.argtypes = [c_void_p, c_int, POINTER(OrCamera), POINTER(OrLighting), POINTER(c_float), c_uint32,
                                c_uint32, c_uint32, c_uint32, c_uint32, POINTER(c_uint32), POINTER(c_uint64), c_int]
        L.or_render.restype = c_int
        L.or_render_pixels.argtypes = [c_void_p, c_int, POINTER(OrCamera), POINTER(OrLighting), POINTER(c_float),
                                       c_uint32, c_uint32, c_uint32, POINTER(c_uint32), POINTER(c_uint32), c_size_t,
                                       POINTER(c_uint32), POINTER(c_uint64)]
        L.or_render_pixels.restype = c_int
        L.or_pixel_stats.argtypes = [c_void_p, c_int, POINTER(OrCamera), POINTER(OrLighting), POINTER(c_float),
                                     c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, POINTER(c_uint64), c_int]
        L.or_pixel_stats.restype = c_int
        L.or_set_iter_budget.argtypes = [c_uint64]
        L.or_set_iter_budget.restype = None
        L.or_cycle_selftest.argtypes = [c_uint32, c_uint32, c_uint32]
        L.or_cycle_selftest.restype = ctypes.c_int64
        _lib = L
    return _lib


NO_BUDGET = (1 << 64) - 1


def set_iter_budget(budget: int = NO_BUDGET) -> None:
    """Diagnostic iteration budget of every later render (process-global; see vr_oracle.h)."""
    lib().or_set_iter_budget(int(budget))


def _f3(v):
    return (c_float * 3)(*[float(x) for x in v])


def camera(eye, look_at, up, fov, aspect) -> OrCamera:
    c = OrCamera()
    lib().or_camera_make(_f3(eye), _f3(look_at), _f3(up), float(fov), float(aspect), ctypes.byref(c))
    return c


def reference_camera(width: int, height: int) -> OrCamera:
    """Main.cu:197-199."""
    aspect = float(np.float32(width) / np.float32(height))
    return camera((6.0, 2.0, 6.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 60.0, aspect)


def lighting(use_shadows=True, use_point_light=False, light_position=(10.0, 10.0, -10.0)) -> OrLighting:
    lit = OrLighting()
    lib().or_lighting_default(ctypes.byref(lit))
    lit.use_shadows = int(bool(use_shadows))
    lit.use_point_light = int(bool(use_point_light))
    for i in range(3):
        lit.light_pos[i] = float(light_position[i])
    return lit


class Scene:
    def __init__(self, xyz: np.ndarray, rgb: np.ndarray, store: int):
        xyz = np.ascontiguousarray(xyz, dtype=np.int32).reshape(-1, 3)
        rgb = np.ascontiguousarray(rgb, dtype=np.uint32).reshape(-1)
        h = c_void_p()
        rc = lib().or_scene_build(int(store), xyz.ctypes.data_as(POINTER(c_int32)),
                                  rgb.ctypes.data_as(POINTER(c_uint32)), rgb.shape[0], ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"or_scene_build failed: {rc}")
        self.h = h
        self.store = store

    @property
    def diameter(self) -> int:
        return lib().or_scene_diameter(self.h)

    @property
    def min_coord(self) -> int:
        return lib().or_scene_min_coord(self.h)

    @property
    def region_count(self) -> int:
        return lib().or_scene_region_count(self.h)

    def lookup(self, region, local) -> int:
        return lib().or_scene_lookup(self.h, *[int(v) for v in region], *[int(v) for v in local])

    def cuckoo_table(self, region_index: int, key: int):
        """(table 1 or 2 the key sits in -- 0 absent --, the region's table was rehashed)."""
        rh = c_int()
        t = lib().or_scene_cuckoo_table(self.h, int(region_index), int(key) & 0xFFFFFFFF, ctypes.byref(rh))
        if t < 0:
            raise ValueError("not a hashtable region")
        return t, bool(rh.value)

    def render(self, algo: int, cam: OrCamera, lit: OrLighting, width: int, height: int, scale: int,
               translation=(0.0, 0.0, 0.0), row_begin: int = 0, row_end: int | None = None, nthreads: int = 0):
        """-> (uint32[rows*width] packed pixels, algorithmic bytes)."""
        row_end = height if row_end is None else row_end
        out = np.zeros((row_end - row_begin) * width, dtype=np.uint32)
        nbytes = c_uint64()
        rc = lib().or_render(self.h, int(algo), ctypes.byref(cam), ctypes.byref(lit), _f3(translation), int(scale),
                             int(width), int(height), int(row_begin), int(row_end),
                             out.ctypes.data_as(POINTER(c_uint32)), ctypes.byref(nbytes), int(nthreads))
        if rc != 0:
            raise RuntimeError(f"or_render failed: {rc}")
        return out, nbytes.value

    def render_pixels(self, algo: int, cam: OrCamera, lit: OrLighting, width: int, height: int, scale: int,
                      px, py, translation=(0.0, 0.0, 0.0)):
        px = np.ascontiguousarray(px, dtype=np.uint32)
        py = np.ascontiguousarray(py, dtype=np.uint32)
        out = np.zeros(px.shape[0], dtype=np.uint32)
        b = np.zeros(px.shape[0], dtype=np.uint64)
        rc = lib().or_render_pixels(self.h, int(algo), ctypes.byref(cam), ctypes.byref(lit), _f3(translation),
                                    int(scale), int(width), int(height), px.ctypes.data_as(POINTER(c_uint32)),
                                    py.ctypes.data_as(POINTER(c_uint32)), px.shape[0],
                                    out.ctypes.data_as(POINTER(c_uint32)), b.ctypes.data_as(POINTER(c_uint64)))
        if rc != 0:
            raise RuntimeError(f"or_render_pixels failed: {rc}")
        return out, b

    def pixel_stats(self, algo: int, cam: OrCamera, lit: OrLighting, width: int, height: int, scale: int,
                    translation=(0.0, 0.0, 0.0), row_begin: int = 0, row_end: int | None = None, nthreads: int = 0):
        """-> uint64[rows, width, 2, 9]: per-pixel (primary, shadow) x (region reads, existence
        checks, cluster skips, lookups, probes, hits, iterations, existence checks outside the
        region, aliased ones among them)."""
        row_end = height if row_end is None else row_end
        st = np.zeros(((row_end - row_begin), width, 2, 9), dtype=np.uint64)
        rc = lib().or_pixel_stats(self.h, int(algo), ctypes.byref(cam), ctypes.byref(lit), _f3(translation),
                                  int(scale), int(width), int(height), int(row_begin), int(row_end),
                                  st.ctypes.data_as(POINTER(c_uint64)), int(nthreads))
        if rc != 0:
            raise RuntimeError(f"or_pixel_stats failed: {rc}")
        return st

    def close(self):
        if self.h:
            lib().or_scene_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def hash1(key: int, offset: int) -> int:
    return lib().or_hash1(ctypes.c_int32(key & 0xFFFFFFFF).value, offset)


def hash2(key: int, prime: int) -> int:
    return lib().or_hash2(ctypes.c_int32(key & 0xFFFFFFFF).value, prime)
