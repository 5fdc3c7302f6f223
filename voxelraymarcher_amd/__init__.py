"""voxelraymarcher_amd -- MI355X-native voxel ray-march renderer.

Drop-in for the hot path of lukeduball/VoxelRaymarcher: the per-pixel ray
march (original 3-axis DDA and longest-axis jump) over the VoxelClusterStore
and CuckooHashTable lookups, as hand-written HIP for gfx950 behind the C ABI
in include/vr.h (libvr.so).  This package is the Python host mirror used by
the tests and the benchmark; the C++ host mirror is include/vr.hpp and the
CLI is bin/VoxelRaymarcher.
"""
from ._capi import LIB_PATH, VrError, lib
from .output import FrameWriter, ImageWriter, encode_png, write_png
from .renderer import (CONFIGS, Build, Camera, DeviceScene, Kernel, Occupancy, PreparedRender, RayMarchAlgorithm,
                       RenderConfig,
                       Schedule, StorageType, VoxelSceneCPU, VoxelSceneInfo, assemble_tiles_device, band_buffer_words,
                       create_scene, deal_stride_default, debug_skip_next_crawl, forget_orders, pack_rgb8, parse_algorithm, parse_storage,
                       read_voxel_file, render_bands, render_count, render_ex, render_tiles, run_raymarching_kernel,
                       setup_constant_values, synth_scene, tile_buffer_words, write_binary_scene, write_voxel_file)

__all__ = ["LIB_PATH", "VrError", "lib", "FrameWriter", "ImageWriter", "encode_png", "write_png", "CONFIGS", "Build",
           "Camera", "DeviceScene", "Kernel", "Occupancy", "PreparedRender", "RayMarchAlgorithm", "RenderConfig", "Schedule",
           "StorageType", "VoxelSceneCPU", "VoxelSceneInfo", "assemble_tiles_device", "band_buffer_words",
           "create_scene", "deal_stride_default", "debug_skip_next_crawl", "forget_orders", "pack_rgb8", "parse_algorithm", "parse_storage",
           "read_voxel_file", "render_bands", "render_count", "render_ex", "render_tiles", "run_raymarching_kernel",
           "setup_constant_values", "synth_scene", "tile_buffer_words", "write_binary_scene", "write_voxel_file"]
