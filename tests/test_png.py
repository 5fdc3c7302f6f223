"""PNG output: libvr's parallel encoder must produce a
valid PNG whose pixels are the input bytes (the reference's stbi_write_png
output is compared by pixels, not bytes -- SURVEY 8(c)). Host only."""
from __future__ import annotations

import struct
import zlib

import numpy as np
import pytest

import voxelraymarcher_amd as vr


def decode_png(data: bytes) -> np.ndarray:
    """Minimal 8-bit non-interlaced PNG decoder (test infrastructure)."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF, typ
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
        if typ == b"IEND":
            break
    assert pos == len(data)
    w, h, depth, ctype, comp, filt, interlace = hdr
    assert (depth, comp, filt, interlace) == (8, 0, 0, 0)
    ch = {0: 1, 4: 2, 2: 3, 6: 4}[ctype]
    raw = zlib.decompress(idat)                     # checks the combined Adler-32
    stride = w * ch
    assert len(raw) == h * (stride + 1)
    out = np.zeros((h, stride), np.int32)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, y * (stride + 1) + 1).astype(np.int32)
        cur = np.zeros(stride, np.int32)
        for i in range(stride):
            a = cur[i - ch] if i >= ch else 0
            b = prev[i]
            c = prev[i - ch] if i >= ch else 0
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = b
            elif f == 3:
                p = (a + b) >> 1
            else:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                p = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
            cur[i] = (line[i] + p) & 0xFF
        out[y] = cur
        prev = cur
    return out.astype(np.uint8).reshape(h, w, ch)


def image(h, w, c, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.stack([(xx * (k + 1) + yy * (3 - k)) & 0xFF for k in range(c)], -1).astype(np.uint8)
    noise = rng.random((h, w)) < 0.2
    img[noise] = rng.integers(0, 256, size=(noise.sum(), c), dtype=np.uint8)
    return img


@pytest.mark.parametrize("h,w,c", [(1, 1, 3), (7, 5, 1), (31, 40, 2), (64, 33, 3), (150, 90, 4), (257, 64, 3)])
@pytest.mark.parametrize("threads", [1, 8])
def test_png_roundtrip(h, w, c, threads):
    img = image(h, w, c, h * 1000 + w)
    png = vr.encode_png(img, level=6, threads=threads)
    assert np.array_equal(decode_png(png), img)


@pytest.mark.parametrize("level", [0, 1, 9])
def test_png_levels_and_file(tmp_path, level):
    img = image(100, 80, 3, level)
    p = str(tmp_path / "out.png")
    vr.write_png(p, img, level=level)
    assert np.array_equal(decode_png(open(p, "rb").read()), img)


def test_png_parallel_chunks_equal_single_stream_pixels():
    img = image(1080 // 8, 1920 // 8, 3, 7)
    a, b = vr.encode_png(img, threads=1), vr.encode_png(img, threads=16)
    assert np.array_equal(decode_png(a), decode_png(b))


def test_image_writer_mirror_and_errors(tmp_path):
    img = image(20, 30, 3, 1)
    assert vr.ImageWriter().write_image(str(tmp_path / "a.png"), img.tobytes(), 30, 20, 3)
    assert np.array_equal(decode_png(open(tmp_path / "a.png", "rb").read()), img)
    assert not vr.ImageWriter().write_image(str(tmp_path / "missing" / "a.png"), img.tobytes(), 30, 20, 3)
    with pytest.raises(ValueError):
        vr.encode_png(np.zeros((4, 4, 5), np.uint8))
    with pytest.raises(vr.VrError):
        vr.write_png(str(tmp_path / "nodir" / "x.png"), img)


@pytest.mark.parametrize("level", [0, 9])
def test_png_size_query_is_an_upper_bound(level):
    import ctypes
    from voxelraymarcher_amd._capi import lib
    noise = np.random.default_rng(level).integers(0, 256, size=(300, 211, 4), dtype=np.uint8)   # incompressible
    bound = ctypes.c_size_t(0)
    assert lib().vr_png_encode(ctypes.c_void_p(noise.ctypes.data), 211, 300, 4, level, 8, None, 0,
                               ctypes.byref(bound)) == 0
    png = vr.encode_png(noise, level=level, threads=8)
    assert len(png) <= bound.value and np.array_equal(decode_png(png), noise)
