"""Frame output: the step after the ray march.

Reference: writeColorToFramebuffer (renderer/Renderer.cuh:1024-1031) writes 3
bytes per pixel from the kernel; writeResultingImageToDisk (main/Main.cu:165-174)
does a blocking cudaMemcpy into malloc'd memory and ImageWriter::writeImage
(renderer/images/ImageWriter.cpp:8-16) calls stbi_write_png.

Here the kernel writes packed 0x00RRGGBB words (one coalesced 4-B store per
pixel). `FrameWriter` turns a stream of such frames into PNG files without
stalling the renderer: the RGB8 pack runs on the device on a side stream that
waits for the frame, the D2H copy goes into pinned host memory, and the PNG is
deflated by libvr's parallel encoder on a worker thread (ctypes drops the GIL
for the call), so frame k+1 renders while frame k is packed, copied and
encoded. The encoder is native (vr_png_write); only the orchestration is here.
"""
from __future__ import annotations

import ctypes
from concurrent.futures import Future, ThreadPoolExecutor
from ctypes import c_size_t, c_void_p

import numpy as np
import torch

from ._capi import check, lib
from .renderer import _stream_ptr


def _image_args(image: np.ndarray):
    img = np.ascontiguousarray(image, dtype=np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    if img.ndim != 3 or not 1 <= img.shape[2] <= 4:
        raise ValueError("image must be (H, W) or (H, W, C) with 1 <= C <= 4")
    return img, int(img.shape[1]), int(img.shape[0]), int(img.shape[2])


def write_png(path: str, image: np.ndarray, level: int = 6) -> None:
    """stbi_write_png(path, w, h, c, image, 0) (ImageWriter.cpp:10) via vr_png_write."""
    img, w, h, c = _image_args(image)
    check(lib().vr_png_write(path.encode(), c_void_p(img.ctypes.data), w, h, c, int(level)), "vr_png_write")


def encode_png(image: np.ndarray, level: int = 6, threads: int = 0) -> bytes:
    """The same encoder into memory."""
    img, w, h, c = _image_args(image)
    n = c_size_t(0)
    check(lib().vr_png_encode(c_void_p(img.ctypes.data), w, h, c, int(level), int(threads), None, 0,
                              ctypes.byref(n)), "vr_png_encode")
    buf = np.empty(n.value, np.uint8)
    check(lib().vr_png_encode(c_void_p(img.ctypes.data), w, h, c, int(level), int(threads), c_void_p(buf.ctypes.data),
                              n.value, ctypes.byref(n)), "vr_png_encode")
    return buf[: n.value].tobytes()


class ImageWriter:
    """ImageWriter (renderer/images/ImageWriter.h): writeImage(filename, image, width, height, colorChannels)."""

    def write_image(self, filename: str, image, width: int, height: int, color_channels: int = 3) -> bool:
        img = np.frombuffer(memoryview(image), dtype=np.uint8, count=width * height * color_channels)
        try:
            write_png(filename, img.reshape(height, width, color_channels))
        except Exception as e:  # the reference prints and returns false (ImageWriter.cpp:11-14)
            print(f"ERROR: Failed to write image to: {filename} ({e})")
            return False
        return True


def pack_rgb8_into(words: torch.Tensor, rgb: torch.Tensor, stream=None) -> torch.Tensor:
    """vr_pack_rgb8 into a caller-provided device buffer (>= 3 bytes per word)."""
    if not rgb.is_cuda or rgb.dtype != torch.uint8 or not rgb.is_contiguous() or rgb.numel() < 3 * words.numel():
        raise ValueError("rgb must be a contiguous CUDA uint8 tensor of >= 3*len(words) bytes")
    check(lib().vr_pack_rgb8(c_void_p(words.data_ptr()), c_void_p(rgb.data_ptr()), words.numel(),
                             _stream_ptr(stream)), "vr_pack_rgb8")
    return rgb


class FrameWriter:
    """Pipelined frame output: device pack -> async D2H (pinned) -> PNG on a worker.

    `submit(words, path)` returns at once; `depth` frames may be in flight (each
    with its own device RGB buffer and pinned host buffer, reused only after its
    PNG is written). `close()` waits for everything and re-raises the first error.
    """

    def __init__(self, width: int, height: int, device: int = 0, depth: int = 2, level: int = 6):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.width, self.height, self.level = int(width), int(height), int(level)
        n = self.width * self.height * 3
        dev = torch.device("cuda", device)
        self._rgb = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(depth)]
        self._host = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(depth)]
        self._done = [torch.cuda.Event() for _ in range(depth)]
        self._pending: list[Future | None] = [None] * depth
        self._stream = torch.cuda.Stream(device=dev)
        self._pool = ThreadPoolExecutor(max_workers=depth)
        self._next = 0
        self._all: list[Future] = []
        self.written: list[str] = []

    def submit(self, words: torch.Tensor, path: str, stream=None) -> None:
        if words.numel() != self.width * self.height:
            raise ValueError(f"frame has {words.numel()} words, expected {self.width * self.height}")
        slot = self._next % len(self._rgb)
        self._next += 1
        if self._pending[slot] is not None:
            self._pending[slot].result()                 # buffers of this slot are free again
        producer = stream if stream is not None else torch.cuda.current_stream(words.device)
        ready = torch.cuda.Event()
        ready.record(producer)
        self._stream.wait_event(ready)
        consumed = torch.cuda.Event()
        with torch.cuda.stream(self._stream):
            pack_rgb8_into(words, self._rgb[slot], stream=self._stream)
            consumed.record(self._stream)
            self._host[slot].copy_(self._rgb[slot], non_blocking=True)
            self._done[slot].record(self._stream)
        # The caller may render the next frame into `words` at once: its stream
        # waits for the pack (a few us), not for the copy or the encode.
        producer.wait_event(consumed)
        words.record_stream(self._stream)
        self._pending[slot] = self._pool.submit(self._encode, slot, path)
        self._all.append(self._pending[slot])

    def _encode(self, slot: int, path: str) -> str:
        self._done[slot].synchronize()
        img = self._host[slot].numpy().reshape(self.height, self.width, 3)
        write_png(path, img, self.level)
        return path

    def flush(self) -> list[str]:
        """Wait for every submitted frame; returns all written paths in submission order."""
        self._pending = [None] * len(self._pending)
        for f in self._all[len(self.written):]:
            self.written.append(f.result())
        return self.written

    def close(self) -> list[str]:
        try:
            return self.flush()
        finally:
            self._pool.shutdown(wait=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
