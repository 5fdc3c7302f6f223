"""Host-side interface of the renderer, mirroring the reference's host names.

  StorageType            geometry/VoxelFunctions.cuh:37
  Camera                 renderer/camera/Camera.cuh:11-29
  VoxelSceneInfo         renderer/VoxelSceneInfo.cuh:5-15
  VoxelSceneCPU          geometry/VoxelSceneCPU.cuh:13-131 (insertVoxel, generateVoxelScene)
  read_voxel_file        geometry/VoxelFile.cuh:9-35
  setup_constant_values  main/Main.cu:26-42
  run_raymarching_kernel main/Main.cu:105-163

All compute goes through libvr.so (HIP, gfx950).  Device buffers are torch
tensors (plumbing only); frames are uint32 tensors of packed 0x00RRGGBB words.
"""
from __future__ import annotations

import ctypes
import enum
from ctypes import c_int32, c_size_t, c_uint32, c_void_p
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _capi
from ._capi import check, f3, lib


class StorageType(enum.IntEnum):
    VOXEL_CLUSTER_STORE = _capi.VR_STORE_VCS
    HASH_TABLE = _capi.VR_STORE_HASHTABLE


class RayMarchAlgorithm(enum.IntEnum):
    LONGEST_AXIS = _capi.VR_ALGO_LONGESTAXIS
    ORIGINAL = _capi.VR_ALGO_ORIGINAL


def parse_storage(name: str) -> StorageType:
    """processStorageTypeCmdArg (Main.cu:45-55): 'hashtable' else VCS."""
    return StorageType.HASH_TABLE if name == "hashtable" else StorageType.VOXEL_CLUSTER_STORE


def parse_algorithm(name: str) -> RayMarchAlgorithm:
    """processAlgorithmCmdArg (Main.cu:58-68): 'original' else longest axis."""
    return RayMarchAlgorithm.ORIGINAL if name == "original" else RayMarchAlgorithm.LONGEST_AXIS


class Camera:
    """Camera(o, lookAt, globalUp, fieldOfView, aspectRatio) (Camera.cuh:11-23), built on the host."""

    def __init__(self, origin, look_at, global_up, field_of_view: float, aspect_ratio: float):
        self.raw = _capi.VrCamera()
        check(lib().vr_camera_make(f3(origin), f3(look_at), f3(global_up), float(field_of_view),
                                   float(aspect_ratio), ctypes.byref(self.raw)), "Camera")

    @classmethod
    def reference(cls, width: int, height: int) -> "Camera":
        """The hard-coded camera of Main.cu:197-199."""
        aspect = float(np.float32(width) / np.float32(height))
        return cls((6.0, 2.0, 6.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 60.0, aspect)

    def as_floats(self) -> np.ndarray:
        r = self.raw
        return np.array([list(r.origin), list(r.lower_left), list(r.horizontal), list(r.vertical),
                         list(r.forward)], dtype=np.float32)


def setup_constant_values(use_shadows: bool = True, use_point_light: bool = False,
                          light_position=(10.0, 10.0, -10.0), light_direction=None,
                          light_color=(1.0, 1.0, 1.0)) -> _capi.VrLighting:
    """setupConstantValues (Main.cu:26-42) -> the lighting block. The defaults are
    the reference's; `light_direction` (un-normalised, default (1,1,1)) goes through
    makeUnitVector exactly as Main.cu:28 does it."""
    lit = _capi.VrLighting()
    check(lib().vr_lighting_default(ctypes.byref(lit)), "setupConstantValues")
    if light_direction is not None:
        d = (ctypes.c_float * 3)(*[float(c) for c in light_direction])
        check(lib().vr_lighting_set_direction(ctypes.byref(lit), d), "light direction")
    lit.use_shadows = int(bool(use_shadows))
    lit.use_point_light = int(bool(use_point_light))
    for i in range(3):
        lit.light_pos[i] = float(light_position[i])
        lit.light_color[i] = float(light_color[i])
    return lit


@dataclass
class VoxelSceneInfo:
    """VoxelSceneInfo(location, scale) (VoxelSceneInfo.cuh:5-15)."""
    translation: tuple = (0.0, 0.0, 0.0)
    scale: int = 1


class DeviceScene:
    """One immutable scene resident in HBM (owns the vr_scene handle)."""

    def __init__(self, handle: c_void_p):
        self._h = handle

    @property
    def handle(self) -> c_void_p:
        if not self._h:
            raise ValueError("scene destroyed")
        return self._h

    def info(self) -> dict:
        i = _capi.VrSceneInfo()
        check(lib().vr_scene_get_info(self.handle, ctypes.byref(i)), "vr_scene_get_info")
        return {"diameter": i.diameter, "min_coord": i.min_coord, "region_count": i.region_count,
                "store": StorageType(i.store), "voxel_count": i.voxel_count, "device_bytes": i.device_bytes,
                "device": i.device}

    def digest(self) -> tuple:
        """FNV-1a of (region table, VCS masks, VCS colours, cuckoo meta, cuckoo slots)."""
        d = (ctypes.c_uint64 * 5)()
        check(lib().vr_scene_digest(self.handle, d), "vr_scene_digest")
        return tuple(int(x) for x in d)

    def close(self) -> None:
        if self._h:
            lib().vr_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Build(enum.IntEnum):
    """vr_build: where the scene image is built (both give identical images)."""
    AUTO = 0
    DEVICE = 1
    HOST = 2


def _build_stream(stream) -> c_void_p:
    return c_void_p(None) if stream is None else c_void_p(stream.cuda_stream)


def create_scene(xyz, rgb, store: StorageType, device: int = 0, build: Build = Build.AUTO, stream=None) -> DeviceScene:
    """generateVoxelScene(storageType) over the voxels (VoxelSceneCPU.cuh:49-93).
    xyz/rgb: numpy arrays, or torch tensors already on the GPU (int32 [n,3] / [n])."""
    h = c_void_p()
    if hasattr(xyz, "is_cuda") and xyz.is_cuda:
        import torch
        xyz = xyz.to(torch.int32).contiguous().reshape(-1, 3)
        rgb = rgb.to(torch.int32).contiguous().reshape(-1)
        if xyz.shape[0] != rgb.shape[0]:
            raise ValueError("xyz and rgb lengths differ")
        check(lib().vr_scene_create_ex(int(device), int(store), c_void_p(xyz.data_ptr()), c_void_p(rgb.data_ptr()),
                                       rgb.shape[0], 1, int(build), _build_stream(stream), ctypes.byref(h)),
              "generateVoxelScene")
        return DeviceScene(h)
    xyz = np.ascontiguousarray(xyz, dtype=np.int32).reshape(-1, 3)
    rgb = np.ascontiguousarray(rgb, dtype=np.uint32).reshape(-1)
    if xyz.shape[0] != rgb.shape[0]:
        raise ValueError("xyz and rgb lengths differ")
    check(lib().vr_scene_create_ex(int(device), int(store), xyz.ctypes.data_as(ctypes.c_void_p),
                                   rgb.ctypes.data_as(ctypes.c_void_p), rgb.shape[0], 0, int(build),
                                   _build_stream(stream), ctypes.byref(h)),
          "generateVoxelScene")
    return DeviceScene(h)


class VoxelSceneCPU:
    """Host-side voxel accumulator (VoxelSceneCPU.cuh:13-46)."""

    def __init__(self):
        self._xyz: list = []
        self._rgb: list = []

    def insert_voxel(self, x: int, y: int, z: int, color: int) -> None:
        self._xyz.append((int(x), int(y), int(z)))
        self._rgb.append(int(color) & 0xFFFFFFFF)

    insertVoxel = insert_voxel

    def extend(self, xyz: np.ndarray, rgb: np.ndarray) -> None:
        self._xyz.extend(map(tuple, np.asarray(xyz, dtype=np.int64).reshape(-1, 3).tolist()))
        self._rgb.extend(np.asarray(rgb, dtype=np.uint64).reshape(-1).tolist())

    def arrays(self):
        return (np.array(self._xyz, dtype=np.int32).reshape(-1, 3), np.array(self._rgb, dtype=np.uint32))

    def generate_voxel_scene(self, storage_type: StorageType, device: int = 0) -> DeviceScene:
        xyz, rgb = self.arrays()
        return create_scene(xyz, rgb, storage_type, device)

    generateVoxelScene = generate_voxel_scene


def _read_scene_file(fn: str, path: str):
    n = c_size_t()
    check(getattr(lib(), fn)(path.encode(), None, None, 0, ctypes.byref(n)), fn)
    xyz = np.zeros((max(n.value, 1), 3), dtype=np.int32)
    rgb = np.zeros(max(n.value, 1), dtype=np.uint32)
    check(getattr(lib(), fn)(path.encode(), xyz.ctypes.data_as(ctypes.POINTER(c_int32)),
                             rgb.ctypes.data_as(ctypes.POINTER(c_uint32)), n.value, ctypes.byref(n)), fn)
    return xyz[: n.value].copy(), rgb[: n.value].copy()


def read_voxel_file(path: str):
    """VoxelFile::readVoxelFile (VoxelFile.cuh:9-35) -> (xyz int32[n,3], rgb uint32[n]).
    Reads the .vox CSV (parsed in parallel, same rules) or, detected by its magic,
    the .vxb binary sidecar."""
    return _read_scene_file("vr_scene_file_read", path)


def write_voxel_file(path: str, xyz: np.ndarray, rgb: np.ndarray) -> None:
    xyz = np.ascontiguousarray(xyz, dtype=np.int32).reshape(-1, 3)
    rgb = np.ascontiguousarray(rgb, dtype=np.uint32).reshape(-1)
    check(lib().vr_vox_write(path.encode(), xyz.ctypes.data_as(ctypes.POINTER(c_int32)),
                             rgb.ctypes.data_as(ctypes.POINTER(c_uint32)), rgb.shape[0]), "write_voxel_file")


def write_binary_scene(path: str, xyz: np.ndarray, rgb: np.ndarray) -> None:
    """The .vxb binary sidecar (vr_vxb_write): the same voxels, loaded without parsing."""
    xyz = np.ascontiguousarray(xyz, dtype=np.int32).reshape(-1, 3)
    rgb = np.ascontiguousarray(rgb, dtype=np.uint32).reshape(-1)
    check(lib().vr_vxb_write(path.encode(), xyz.ctypes.data_as(ctypes.POINTER(c_int32)),
                             rgb.ctypes.data_as(ctypes.POINTER(c_uint32)), rgb.shape[0]), "write_binary_scene")


def synth_scene(n: int, p_region: float, p_cluster: float, p_voxel: float, seed: int):
    """Synthetic counter-hash grid -> (xyz int32[n,3], rgb uint32[n])."""
    p = _capi.VrSynthParams(int(n), float(p_region), float(p_cluster), float(p_voxel), int(seed))
    cnt = c_size_t()
    check(lib().vr_synth_generate(ctypes.byref(p), None, None, 0, ctypes.byref(cnt)), "vr_synth_generate")
    xyz = np.zeros((max(cnt.value, 1), 3), dtype=np.int32)
    rgb = np.zeros(max(cnt.value, 1), dtype=np.uint32)
    check(lib().vr_synth_generate(ctypes.byref(p), xyz.ctypes.data_as(ctypes.POINTER(c_int32)),
                                  rgb.ctypes.data_as(ctypes.POINTER(c_uint32)), cnt.value, ctypes.byref(cnt)),
          "vr_synth_generate")
    return xyz[: cnt.value].copy(), rgb[: cnt.value].copy()


def _stream_ptr(stream) -> c_void_p:
    if stream is None:
        stream = torch.cuda.current_stream()
    return c_void_p(stream.cuda_stream)


def _require_u32(out: torch.Tensor, words: int) -> None:
    if not out.is_cuda or out.dtype != torch.int32 and out.dtype != torch.uint32:
        raise TypeError("out must be a CUDA int32/uint32 tensor")
    if not out.is_contiguous() or out.numel() < words:
        raise ValueError(f"out must be contiguous with >= {words} elements")


class Kernel(enum.IntEnum):
    """vr_kernel: which HIP implementation renders (identical pixels)."""
    AUTO = _capi.VR_KERNEL_AUTO
    TILE = _capi.VR_KERNEL_TILE
    TILE_REWALK = _capi.VR_KERNEL_TILE_REWALK


class Schedule(enum.IntEnum):
    """vr_schedule: the tile pass's work order (identical pixels).  AUTO: heaviest tile
    groups first when the device's previous launch was on the same stream or has finished
    (a lone frame's latency), grid order while another stream's launch runs (frames in flight)."""
    AUTO = _capi.VR_SCHEDULE_AUTO
    GRID = _capi.VR_SCHEDULE_GRID
    HEAVIEST_FIRST = _capi.VR_SCHEDULE_HEAVIEST_FIRST


class Occupancy(enum.IntEnum):
    """vr_occupancy: the tile pass's occupancy variant (identical pixels).  AUTO: the in-flight
    variant while another stream's launch runs -- where one is built (vr_march.hip
    VR_ORIG_WAVES_HI / VR_LONG_WAVES_HI; round 6 measured every walk fastest in flight with its
    lone kernel, so by default IN_FLIGHT launches that kernel)."""
    AUTO = _capi.VR_OCCUPANCY_AUTO
    LONE = _capi.VR_OCCUPANCY_LONE
    IN_FLIGHT = _capi.VR_OCCUPANCY_IN_FLIGHT


def render_ex(scene: DeviceScene, algorithm: RayMarchAlgorithm, camera: Camera, lighting: _capi.VrLighting,
              info: VoxelSceneInfo, width: int, height: int, out: torch.Tensor, row_begin: int = 0,
              row_end: int | None = None, band_rows: int = 0, rank: int = 0, nranks: int = 1,
              counter: torch.Tensor | None = None, kernel: Kernel = Kernel.AUTO, stream=None,
              defer_cap: int = 0, schedule: Schedule = Schedule.AUTO,
              stats: torch.Tensor | None = None, occupancy: Occupancy = Occupancy.AUTO,
              tile_cols: int = 0, deal_stride: int = 0) -> torch.Tensor:
    """vr_render_ex: rows [row_begin,row_end), bands of band_rows (0 = one band) dealt to nranks ranks.
    defer_cap: capacity of the crawl pass's deferral list (0 = default; small values force its overflow path).
    schedule: the tile pass's work order (Schedule); occupancy: its occupancy variant (Occupancy).
    stats (with counter): CUDA int64[2], caller-zeroed: [0] crawl iterations fast-forwarded in closed form,
    [1] the existence-read bytes credited for them (part of counter's count, never loaded).
    tile_cols > 0: the 2-D tile deal (block j of band b -> rank (j + deal_stride * b) % nranks;
    tile_buffer_words per rank)."""
    row_end = height if row_end is None else row_end
    rows = row_end - row_begin
    if tile_cols:
        words = tile_buffer_words(width, rows, band_rows or max(1, rows), tile_cols, nranks)
    else:
        words = band_buffer_words(width, rows, band_rows or max(1, rows), nranks)
    _require_u32(out, words)
    for name, t in (("counter", counter), ("stats", stats)):
        if t is not None and (not t.is_cuda or t.dtype != torch.int64):
            raise TypeError(f"{name} must be a CUDA int64 tensor")
    if stats is not None and (counter is None or stats.numel() < 2 or not stats.is_contiguous()):
        raise ValueError("stats needs a counter and 2 contiguous int64 elements")
    opts = _capi.VrRenderOpts()
    check(lib().vr_render_opts_init(ctypes.byref(opts)), "vr_render_opts_init")
    opts.kernel, opts.row_begin, opts.row_end = int(kernel), int(row_begin), int(row_end)
    opts.band_rows, opts.rank, opts.nranks = int(band_rows), int(rank), int(nranks)
    opts.bytes_dev = c_void_p(counter.data_ptr()) if counter is not None else None
    opts.defer_cap, opts.schedule = int(defer_cap), int(schedule)
    opts.stats_dev = c_void_p(stats.data_ptr()) if stats is not None else None
    opts.occupancy, opts.tile_cols, opts.deal_stride = int(occupancy), int(tile_cols), int(deal_stride)
    check(lib().vr_render_ex(scene.handle, int(algorithm), ctypes.byref(camera.raw), ctypes.byref(lighting),
                             f3(info.translation), int(info.scale), int(width), int(height), ctypes.byref(opts),
                             c_void_p(out.data_ptr()), _stream_ptr(stream)), "vr_render_ex")
    return out


class PreparedRender:
    """One view's launch with its arguments made once (render_ex's options, without counter
    or stats): calling it enqueues vr_render_ex into `out` on `stream` (a torch stream, or
    None for the current one).  For a frame loop's per-frame host path: render_ex rebuilds
    the options and re-checks the buffer on every call (~20 us of Python per frame, which a
    20-frame timed loop pays up front while the GPU waits for its first frame;
    profiles/r06/driver_probe2.py).  The camera and lighting structs are passed by reference,
    so changing `camera.raw` in place re-aims the next call; out's size is checked once per
    buffer.  `vr_stream_arg`: BandGather hands its slot stream over instead of entering a
    torch stream context."""
    vr_stream_arg = True

    def __init__(self, scene: DeviceScene, algorithm: RayMarchAlgorithm, camera: Camera,
                 lighting: _capi.VrLighting, info: VoxelSceneInfo, width: int, height: int, row_begin: int = 0,
                 row_end: int | None = None, band_rows: int = 0, rank: int = 0, nranks: int = 1,
                 kernel: Kernel = Kernel.AUTO, schedule: Schedule = Schedule.AUTO,
                 occupancy: Occupancy = Occupancy.AUTO, tile_cols: int = 0, deal_stride: int = 0):
        row_end = height if row_end is None else row_end
        rows = row_end - row_begin
        if tile_cols:
            self.words = tile_buffer_words(width, rows, band_rows or max(1, rows), tile_cols, nranks)
        else:
            self.words = band_buffer_words(width, rows, band_rows or max(1, rows), nranks)
        opts = _capi.VrRenderOpts()
        check(lib().vr_render_opts_init(ctypes.byref(opts)), "vr_render_opts_init")
        opts.kernel, opts.row_begin, opts.row_end = int(kernel), int(row_begin), int(row_end)
        opts.band_rows, opts.rank, opts.nranks = int(band_rows), int(rank), int(nranks)
        opts.schedule, opts.occupancy = int(schedule), int(occupancy)
        opts.tile_cols, opts.deal_stride = int(tile_cols), int(deal_stride)
        self._keep = (scene, camera, lighting, opts, f3(info.translation))   # (alive while prepared)
        self._fn = lib().vr_render_ex
        self._args = (scene.handle, int(algorithm), ctypes.byref(camera.raw), ctypes.byref(lighting),
                      self._keep[4], int(info.scale), int(width), int(height), ctypes.byref(opts))
        self._checked = set()

    def __call__(self, out: torch.Tensor, stream=None) -> torch.Tensor:
        key = (out.data_ptr(), out.numel(), out.dtype, out.is_contiguous())
        if key not in self._checked:
            _require_u32(out, self.words)
            if len(self._checked) >= 64:          # (a loop over many buffers: keep the set small)
                self._checked.clear()
            self._checked.add(key)
        sh = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        rc = self._fn(*self._args, c_void_p(key[0]), c_void_p(sh))
        if rc:
            check(rc, "vr_render_ex")
        return out


def run_raymarching_kernel(scene: DeviceScene, algorithm: RayMarchAlgorithm, camera: Camera,
                           lighting: _capi.VrLighting, info: VoxelSceneInfo, width: int, height: int,
                           out: torch.Tensor | None = None, row_begin: int = 0, row_end: int | None = None,
                           stream=None, kernel: Kernel = Kernel.AUTO) -> torch.Tensor:
    """Launch the ray march for rows [row_begin,row_end) (Main.cu:105-163); asynchronous."""
    row_end = height if row_end is None else row_end
    words = (row_end - row_begin) * width
    if out is None:
        out = torch.empty(words, dtype=torch.int32, device=f"cuda:{scene.info()['device']}")
    if kernel == Kernel.AUTO:
        _require_u32(out, words)
        check(lib().vr_render(scene.handle, int(algorithm), ctypes.byref(camera.raw), ctypes.byref(lighting),
                              f3(info.translation), int(info.scale), int(width), int(height), int(row_begin),
                              int(row_end), c_void_p(out.data_ptr()), _stream_ptr(stream)), "vr_render")
        return out
    return render_ex(scene, algorithm, camera, lighting, info, width, height, out, row_begin, row_end,
                     kernel=kernel, stream=stream)


def render_count(scene: DeviceScene, algorithm: RayMarchAlgorithm, camera: Camera, lighting: _capi.VrLighting,
                 info: VoxelSceneInfo, width: int, height: int, out: torch.Tensor, counter: torch.Tensor,
                 row_begin: int = 0, row_end: int | None = None, stream=None,
                 kernel: Kernel = Kernel.AUTO) -> None:
    """Instrumented render: adds the SURVEY 8(d) algorithmic bytes into counter (int64 cuda scalar)."""
    render_ex(scene, algorithm, camera, lighting, info, width, height, out, row_begin, row_end,
              counter=counter, kernel=kernel, stream=stream)


def band_buffer_words(width: int, height: int, band_rows: int, nranks: int) -> int:
    return int(lib().vr_band_buffer_words(width, height, band_rows, nranks))


def render_bands(scene: DeviceScene, algorithm: RayMarchAlgorithm, camera: Camera, lighting: _capi.VrLighting,
                 info: VoxelSceneInfo, width: int, height: int, band_rows: int, rank: int, nranks: int,
                 out: torch.Tensor, stream=None) -> torch.Tensor:
    """This rank's interleaved row bands (band b -> rank b % nranks), packed."""
    _require_u32(out, band_buffer_words(width, height, band_rows, nranks))
    check(lib().vr_render_bands(scene.handle, int(algorithm), ctypes.byref(camera.raw), ctypes.byref(lighting),
                                f3(info.translation), int(info.scale), int(width), int(height), int(band_rows),
                                int(rank), int(nranks), c_void_p(out.data_ptr()), _stream_ptr(stream)),
          "vr_render_bands")
    return out


def tile_buffer_words(width: int, height: int, band_rows: int, tile_cols: int, nranks: int) -> int:
    return int(lib().vr_tile_buffer_words(width, height, band_rows, tile_cols, nranks))


def deal_stride_default(nranks: int) -> int:
    return int(lib().vr_deal_stride_default(nranks))


def forget_orders(device: int = 0) -> None:
    """Drop the work and lane orders the device learned (vr_forget_orders): the next launch
    renders as a first render of its view."""
    check(lib().vr_forget_orders(int(device)), "vr_forget_orders")


def debug_skip_next_crawl(device: int = 0) -> None:
    """Test hook (vr_debug_skip_next_crawl): the device's next launch skips its crawl pass as
    if its slot had seen the view defer nothing -- for the test of the crawl-skip safety net."""
    check(lib().vr_debug_skip_next_crawl(int(device)), "vr_debug_skip_next_crawl")


def render_tiles(scene: DeviceScene, algorithm: RayMarchAlgorithm, camera: Camera, lighting: _capi.VrLighting,
                 info: VoxelSceneInfo, width: int, height: int, band_rows: int, tile_cols: int, rank: int,
                 nranks: int, out: torch.Tensor, stream=None) -> torch.Tensor:
    """This rank's tiles of the 2-D deal (block j of band b -> rank (j + stride * b) % nranks), packed."""
    _require_u32(out, tile_buffer_words(width, height, band_rows, tile_cols, nranks))
    check(lib().vr_render_tiles(scene.handle, int(algorithm), ctypes.byref(camera.raw), ctypes.byref(lighting),
                                f3(info.translation), int(info.scale), int(width), int(height), int(band_rows),
                                int(tile_cols), int(rank), int(nranks), c_void_p(out.data_ptr()),
                                _stream_ptr(stream)), "vr_render_tiles")
    return out


def assemble_tiles_device(parts: torch.Tensor, frame: torch.Tensor, elem_bytes: int, width: int, height: int,
                          band_rows: int, tile_cols: int, nranks: int, deal_stride: int = 0,
                          stream=None) -> torch.Tensor:
    """vr_assemble_tiles: rank 0's reassembly on the device.  parts: the nranks tile buffers back to back
    (contiguous, elem_bytes per pixel); frame: width x height pixels of elem_bytes (contiguous)."""
    need = tile_buffer_words(width, height, band_rows, tile_cols, nranks) * nranks * elem_bytes
    for name, t, n in (("parts", parts, need), ("frame", frame, width * height * elem_bytes)):
        if not t.is_cuda or not t.is_contiguous() or t.numel() * t.element_size() < n:
            raise ValueError(f"{name} must be a contiguous CUDA tensor of >= {n} bytes")
    check(lib().vr_assemble_tiles(c_void_p(parts.data_ptr()), c_void_p(frame.data_ptr()), int(elem_bytes),
                                  int(width), int(height), int(band_rows), int(tile_cols), int(nranks),
                                  int(deal_stride), _stream_ptr(stream)), "vr_assemble_tiles")
    return frame


def pack_rgb8(words: torch.Tensor, stream=None, out: torch.Tensor | None = None) -> torch.Tensor:
    """writeColorToFramebuffer (Renderer.cuh:1024-1031) on the device: words -> RGB8 bytes
    (into `out`, uint8 of 3 x words.numel(), when given)."""
    rgb = torch.empty(words.numel() * 3, dtype=torch.uint8, device=words.device) if out is None else out
    if rgb.dtype != torch.uint8 or rgb.numel() != words.numel() * 3 or not rgb.is_contiguous():
        raise ValueError("out must be a contiguous uint8 tensor of 3 x words.numel() bytes")
    check(lib().vr_pack_rgb8(c_void_p(words.data_ptr()), c_void_p(rgb.data_ptr()), words.numel(),
                             _stream_ptr(stream)), "vr_pack_rgb8")
    return rgb


@dataclass
class RenderConfig:
    """One BASELINE.json config."""
    name: str
    grid: int
    p_region: float
    p_cluster: float
    p_voxel: float
    seed: int
    width: int
    height: int
    store: StorageType
    algorithm: RayMarchAlgorithm
    gpus: int = 1
    notes: str = ""
    scale: int = field(init=False)

    def __post_init__(self):
        self.scale = 3 * self.grid // 16        # eye at (6s,2s,6s): just outside the grid's x/z faces

    def voxels(self):
        return synth_scene(self.grid, self.p_region, self.p_cluster, self.p_voxel, self.seed)


CONFIGS = {
    "C1": RenderConfig("C1", 64, 1.0, 0.5, 0.10, 0x1, 256, 256, StorageType.HASH_TABLE, RayMarchAlgorithm.ORIGINAL,
                       notes="scene.vox 64^3, hashtable+original (host-CPU plumbing config)"),
    "C2": RenderConfig("C2", 256, 1.0, 0.30, 0.08, 0x256, 1920, 1080, StorageType.VOXEL_CLUSTER_STORE,
                       RayMarchAlgorithm.ORIGINAL, notes="256^3 synthetic, vcs+original"),
    "C3": RenderConfig("C3", 256, 1.0, 0.30, 0.08, 0x256, 1920, 1080, StorageType.VOXEL_CLUSTER_STORE,
                       RayMarchAlgorithm.LONGEST_AXIS, notes="256^3 synthetic, vcs+longestaxis"),
    "C4": RenderConfig("C4", 512, 1.0, 1.0, 0.15, 0x512, 1920, 1080, StorageType.HASH_TABLE,
                       RayMarchAlgorithm.ORIGINAL, notes="512^3 dense, hashtable+original"),
    "C5": RenderConfig("C5", 1024, 0.35, 0.05, 0.25, 0x1024, 3840, 2160, StorageType.VOXEL_CLUSTER_STORE,
                       RayMarchAlgorithm.ORIGINAL, gpus=8, notes="1024^3 sparse, vcs+original, 8-GPU tiles"),
}
