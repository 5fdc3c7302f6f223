"""ctypes binding of libvr.so (include/vr.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C voxelraymarcher_amd/csrc``).  There is no fallback: if the library
is missing or fails to load, every entry point raises.

``torch`` is imported before the library is opened so that libvr.so binds to
the HIP runtime torch already loaded (same SONAME ``libamdhip64.so.7``):
device pointers and streams from torch are then valid in libvr.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_size_t, c_uint8, c_uint32,
                    c_uint64, c_void_p)

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# VR_LIBRARY selects another in-tree build of the same ABI (A/B tuning runs).
LIB_PATH = os.environ.get("VR_LIBRARY") or os.path.join(HERE, "libvr.so")

VR_OK = 0
ERRORS = {-1: "VR_E_INVALID", -2: "VR_E_HIP", -3: "VR_E_NOMEM", -4: "VR_E_IO", -5: "VR_E_BUILD", -6: "VR_E_PARSE"}

VR_STORE_VCS, VR_STORE_HASHTABLE = 0, 1
VR_ALGO_LONGESTAXIS, VR_ALGO_ORIGINAL = 0, 1


class VrCamera(ctypes.Structure):
    _fields_ = [("origin", c_float * 3), ("lower_left", c_float * 3), ("horizontal", c_float * 3),
                ("vertical", c_float * 3), ("forward", c_float * 3)]


class VrLighting(ctypes.Structure):
    _fields_ = [("light_dir", c_float * 3), ("light_color", c_float * 3), ("light_pos", c_float * 3),
                ("use_point_light", c_int32), ("use_shadows", c_int32)]


class VrSceneInfo(ctypes.Structure):
    _fields_ = [("diameter", c_uint32), ("min_coord", c_int32), ("region_count", c_uint32), ("store", c_uint32),
                ("voxel_count", c_uint64), ("device_bytes", c_uint64), ("device", c_int32)]


class VrSynthParams(ctypes.Structure):
    _fields_ = [("n", c_uint32), ("p_region", c_double), ("p_cluster", c_double), ("p_voxel", c_double),
                ("seed", c_uint64)]


VR_KERNEL_AUTO, VR_KERNEL_TILE, VR_KERNEL_TILE_REWALK = 0, 1, 3
VR_SCHEDULE_AUTO, VR_SCHEDULE_GRID, VR_SCHEDULE_HEAVIEST_FIRST = 0, 1, 2
VR_OCCUPANCY_AUTO, VR_OCCUPANCY_LONE, VR_OCCUPANCY_IN_FLIGHT = 0, 1, 2


class VrRenderOpts(ctypes.Structure):
    """vr_render_opts (versioned by its leading struct_size; VR_RENDER_OPTS_MIN_SIZE = 48)."""
    _fields_ = [("struct_size", c_uint32), ("kernel", c_uint32), ("row_begin", c_uint32), ("row_end", c_uint32),
                ("band_rows", c_uint32), ("rank", c_uint32), ("nranks", c_uint32), ("defer_cap", c_uint32),
                ("bytes_dev", c_void_p), ("schedule", c_uint32), ("reserved", c_uint32), ("stats_dev", c_void_p),
                ("occupancy", c_uint32), ("tile_cols", c_uint32), ("deal_stride", c_uint32), ("reserved2", c_uint32)]


VR_RENDER_OPTS_MIN_SIZE = 48


class VrError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {ERRORS.get(code, code)}: {msg}")
        self.code = code


# name -> (restype, argtypes); every symbol include/vr.h declares.
SIGNATURES = {
    "vr_camera_make": (c_int, [POINTER(c_float), POINTER(c_float), POINTER(c_float), c_float, c_float,
                               POINTER(VrCamera)]),
    "vr_lighting_default": (c_int, [POINTER(VrLighting)]),
    "vr_lighting_set_direction": (c_int, [POINTER(VrLighting), POINTER(c_float)]),
    "vr_png_write": (c_int, [c_char_p, c_void_p, c_uint32, c_uint32, c_int, c_int]),
    "vr_png_encode": (c_int, [c_void_p, c_uint32, c_uint32, c_int, c_int, c_int, c_void_p, c_size_t, POINTER(c_size_t)]),
    "vr_scene_create": (c_int, [c_int, c_int, POINTER(c_int32), POINTER(c_uint32), c_size_t, POINTER(c_void_p)]),
    "vr_scene_create_ex": (c_int, [c_int, c_int, c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p, POINTER(c_void_p)]),
    "vr_scene_digest": (c_int, [c_void_p, POINTER(c_uint64)]),
    "vr_scene_load_vox": (c_int, [c_int, c_int, c_char_p, POINTER(c_void_p)]),
    "vr_scene_get_info": (c_int, [c_void_p, POINTER(VrSceneInfo)]),
    "vr_scene_destroy": (None, [c_void_p]),
    "vr_render": (c_int, [c_void_p, c_int, POINTER(VrCamera), POINTER(VrLighting), POINTER(c_float), c_uint32,
                          c_uint32, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p]),
    "vr_render_bands": (c_int, [c_void_p, c_int, POINTER(VrCamera), POINTER(VrLighting), POINTER(c_float),
                                c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p]),
    "vr_band_buffer_words": (c_uint64, [c_uint32, c_uint32, c_uint32, c_uint32]),
    "vr_render_tiles": (c_int, [c_void_p, c_int, POINTER(VrCamera), POINTER(VrLighting), POINTER(c_float),
                                c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_void_p,
                                c_void_p]),
    "vr_tile_buffer_words": (c_uint64, [c_uint32, c_uint32, c_uint32, c_uint32, c_uint32]),
    "vr_deal_stride_default": (c_uint32, [c_uint32]),
    "vr_forget_orders": (c_int, [c_int]),
    "vr_debug_skip_next_crawl": (c_int, [c_int]),
    "vr_assemble_tiles": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_uint32,
                                  c_uint32, c_void_p]),
    "vr_render_ex": (c_int, [c_void_p, c_int, POINTER(VrCamera), POINTER(VrLighting), POINTER(c_float), c_uint32,
                             c_uint32, c_uint32, POINTER(VrRenderOpts), c_void_p, c_void_p]),
    "vr_render_opts_init": (c_int, [POINTER(VrRenderOpts)]),
    "vr_render_count": (c_int, [c_void_p, c_int, POINTER(VrCamera), POINTER(VrLighting), POINTER(c_float),
                                c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p]),
    "vr_pack_rgb8": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    "vr_synth_generate": (c_int, [POINTER(VrSynthParams), POINTER(c_int32), POINTER(c_uint32), c_size_t,
                                  POINTER(c_size_t)]),
    "vr_vox_read": (c_int, [c_char_p, POINTER(c_int32), POINTER(c_uint32), c_size_t, POINTER(c_size_t)]),
    "vr_vox_write": (c_int, [c_char_p, POINTER(c_int32), POINTER(c_uint32), c_size_t]),
    "vr_vxb_read": (c_int, [c_char_p, POINTER(c_int32), POINTER(c_uint32), c_size_t, POINTER(c_size_t)]),
    "vr_vxb_write": (c_int, [c_char_p, POINTER(c_int32), POINTER(c_uint32), c_size_t]),
    "vr_scene_file_read": (c_int, [c_char_p, POINTER(c_int32), POINTER(c_uint32), c_size_t, POINTER(c_size_t)]),
    "vr_last_error": (c_char_p, []),
    "vr_version": (c_char_p, []),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Open libvr.so (once); raises if it is missing -- there is no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                              "(make -C voxelraymarcher_amd/csrc)")
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int, where: str) -> None:
    if rc != VR_OK:
        raise VrError(rc, where, lib().vr_last_error().decode(errors="replace"))


def f3(v) -> ctypes.Array:
    return (c_float * 3)(*[float(x) for x in v])


__all__ = ["lib", "check", "VrCamera", "VrLighting", "VrRenderOpts", "VR_RENDER_OPTS_MIN_SIZE", "VR_KERNEL_AUTO",
           "VR_KERNEL_TILE", "VR_KERNEL_TILE_REWALK", "VR_SCHEDULE_AUTO", "VR_SCHEDULE_GRID",
           "VR_SCHEDULE_HEAVIEST_FIRST", "VR_OCCUPANCY_AUTO", "VR_OCCUPANCY_LONE", "VR_OCCUPANCY_IN_FLIGHT",
           "VrSceneInfo", "VrSynthParams", "VrError", "SIGNATURES",
           "VR_STORE_VCS", "VR_STORE_HASHTABLE", "VR_ALGO_LONGESTAXIS", "VR_ALGO_ORIGINAL", "f3", "LIB_PATH",
           "c_uint8"]
