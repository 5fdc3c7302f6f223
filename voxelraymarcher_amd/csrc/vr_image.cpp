// PNG output: the host side of writeResultingImageToDisk
// (Main.cu:165-174) -> ImageWriter::writeImage -> stbi_write_png
// (ImageWriter.cpp:8-16). Same image (8-bit, 1-4 channels, tightly packed
// rows); the compressed bytes are not stb's (compare pixels, not
// PNG bytes).
//
// The frame is split into row chunks that are filtered and deflated on
// separate threads; every chunk but the last ends with a sync flush (byte
// aligned, no final block), so their concatenation is one valid raw deflate
// stream, and the per-chunk Adler-32 sums are combined into the zlib trailer.
// The dictionary restarts at each chunk boundary (a few hundred bytes lost per
// chunk at 1080p), which is what buys the parallelism.
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "vr.h"
#include "vr_internal.h"

namespace {

void put32(uint8_t* p, uint32_t x) {
    p[0] = (uint8_t)(x >> 24); p[1] = (uint8_t)(x >> 16); p[2] = (uint8_t)(x >> 8); p[3] = (uint8_t)x;
}

// One filtered scanline: the filter with the smallest sum of |signed bytes|
// (the usual PNG heuristic, also stb's), written as [type, bytes...]. Each
// filter is its own branch-free loop so the compiler vectorises it; `prev` is
// a zero row for the first scanline. tmp holds 5 * len bytes.
void filter_row(const uint8_t* cur, const uint8_t* prev, size_t len, int bpp, uint8_t* out, uint8_t* tmp) {
    uint8_t* t[5] = {tmp, tmp + len, tmp + 2 * len, tmp + 3 * len, tmp + 4 * len};
    const size_t k = std::min(len, (size_t)bpp);
    for (size_t i = 0; i < len; ++i) t[0][i] = cur[i];
    for (size_t i = 0; i < k; ++i) t[1][i] = cur[i];
    for (size_t i = k; i < len; ++i) t[1][i] = (uint8_t)(cur[i] - cur[i - bpp]);
    for (size_t i = 0; i < len; ++i) t[2][i] = (uint8_t)(cur[i] - prev[i]);
    for (size_t i = 0; i < k; ++i) t[3][i] = (uint8_t)(cur[i] - (prev[i] >> 1));
    for (size_t i = k; i < len; ++i) t[3][i] = (uint8_t)(cur[i] - ((cur[i - bpp] + prev[i]) >> 1));
    for (size_t i = 0; i < k; ++i) t[4][i] = (uint8_t)(cur[i] - prev[i]);      // Paeth(0, b, 0) = b
    for (size_t i = k; i < len; ++i) {
        int a = cur[i - bpp], b = prev[i], c = prev[i - bpp];
        int pa = std::abs(b - c), pb = std::abs(a - c), pc = std::abs(a + b - 2 * c);
        int pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
        t[4][i] = (uint8_t)(cur[i] - pred);
    }
    int best = 0;
    uint64_t best_sum = ~uint64_t(0);
    for (int f = 0; f < 5; ++f) {
        uint64_t sum = 0;
        for (size_t i = 0; i < len; ++i) sum += (uint32_t)std::abs((int)(int8_t)t[f][i]);
        if (sum < best_sum) { best_sum = sum; best = f; }
    }
    out[0] = (uint8_t)best;
    std::memcpy(out + 1, t[best], len);
}

struct Chunk {
    std::vector<uint8_t> z;   // raw deflate bytes
    uLong adler = 1;
    size_t raw = 0;
    int status = Z_OK;
};

void deflate_rows(const uint8_t* img, uint32_t w, int ch, uint32_t y0, uint32_t y1, int level, bool last, Chunk& c) {
    const size_t len = (size_t)w * ch, stride = len + 1;
    std::vector<uint8_t> raw((size_t)(y1 - y0) * stride), tmp(5 * len), zero(len, 0);
    for (uint32_t y = y0; y < y1; ++y)
        filter_row(img + (size_t)y * len, y ? img + (size_t)(y - 1) * len : zero.data(), len, ch,
                   raw.data() + (size_t)(y - y0) * stride, tmp.data());
    c.raw = raw.size();
    c.adler = adler32(1L, raw.data(), (uInt)raw.size());
    z_stream s{};
    if ((c.status = deflateInit2(&s, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY)) != Z_OK) return;
    c.z.resize(deflateBound(&s, (uLong)raw.size()) + 16);
    s.next_in = raw.data();
    s.avail_in = (uInt)raw.size();
    s.next_out = c.z.data();
    s.avail_out = (uInt)c.z.size();
    int r = deflate(&s, last ? Z_FINISH : Z_SYNC_FLUSH);
    c.status = (last ? r == Z_STREAM_END : (r == Z_OK && s.avail_in == 0)) ? Z_OK : Z_BUF_ERROR;
    c.z.resize(s.total_out);
    deflateEnd(&s);
}

void append_chunk(std::vector<uint8_t>& png, const char* type, const uint8_t* data, size_t n) {
    uint8_t hdr[8];
    put32(hdr, (uint32_t)n);
    std::memcpy(hdr + 4, type, 4);
    png.insert(png.end(), hdr, hdr + 8);
    if (n) png.insert(png.end(), data, data + n);
    uLong crc = crc32(0L, (const Bytef*)type, 4);
    if (n) crc = crc32(crc, data, (uInt)n);     // crc32(c, NULL, 0) would return 0, not c
    uint8_t t[4];
    put32(t, (uint32_t)crc);
    png.insert(png.end(), t, t + 4);
}

int encode(const uint8_t* img, uint32_t w, uint32_t h, int ch, int level, int threads, std::vector<uint8_t>& png) {
    if (!img || !w || !h || ch < 1 || ch > 4) return vr::set_error(VR_E_INVALID, "png: bad image arguments");
    if ((uint64_t)w * ch + 1 > (1u << 30) || (uint64_t)h * ((uint64_t)w * ch + 1) > (1ull << 34))
        return vr::set_error(VR_E_INVALID, "png: image too large");
    if (level < 0 || level > 9) level = 6;
    // Chunks of >= 32 rows; at most `threads` (default: hardware threads, <= 16).
    int T = threads > 0 ? threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    uint32_t nchunks = std::max(1u, std::min<uint32_t>((uint32_t)T, h / 32));
    std::vector<Chunk> chunks(nchunks);
    std::vector<std::thread> pool;
    for (uint32_t i = 0; i < nchunks; ++i) {
        uint32_t y0 = (uint32_t)((uint64_t)h * i / nchunks), y1 = (uint32_t)((uint64_t)h * (i + 1) / nchunks);
        bool last = i + 1 == nchunks;
        if (last) deflate_rows(img, w, ch, y0, y1, level, true, chunks[i]);
        else pool.emplace_back(deflate_rows, img, w, ch, y0, y1, level, false, std::ref(chunks[i]));
    }
    for (auto& t : pool) t.join();
    size_t zlen = 2 + 4;
    uLong adler = 1;
    for (auto& c : chunks) {
        if (c.status != Z_OK) return vr::set_error(VR_E_NOMEM, "png: deflate failed");
        zlen += c.z.size();
        adler = adler32_combine(adler, c.adler, (z_off_t)c.raw);
    }
    std::vector<uint8_t> z;
    z.reserve(zlen);
    z.push_back(0x78);                                   // CM 8, 32K window
    z.push_back(level >= 7 ? 0xDA : level >= 6 ? 0x9C : level >= 2 ? 0x5E : 0x01);   // FLEVEL + FCHECK
    for (auto& c : chunks) z.insert(z.end(), c.z.begin(), c.z.end());
    uint8_t t[4];
    put32(t, (uint32_t)adler);
    z.insert(z.end(), t, t + 4);

    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    static const uint8_t color_type[5] = {0, 0, 4, 2, 6};   // gray, gray+alpha, RGB, RGBA
    png.assign(sig, sig + 8);
    uint8_t ihdr[13];
    put32(ihdr, w);
    put32(ihdr + 4, h);
    ihdr[8] = 8;
    ihdr[9] = color_type[ch];
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    append_chunk(png, "IHDR", ihdr, 13);
    append_chunk(png, "IDAT", z.data(), z.size());
    append_chunk(png, "IEND", nullptr, 0);
    return VR_OK;
}

}  // namespace

extern "C" {

int vr_png_encode(const uint8_t* image, uint32_t width, uint32_t height, int channels, int level, int threads,
                  uint8_t* out, size_t capacity, size_t* out_len) {
    if (!out_len) return vr::set_error(VR_E_INVALID, "png: NULL out_len");
    if (!out) {
        // Upper bound without encoding: stored deflate blocks cost 5 B per
        // 64 KiB (raw >> 8 covers it), plus per-chunk flush markers and headers.
        if (!width || !height || channels < 1 || channels > 4) return vr::set_error(VR_E_INVALID, "png: bad image arguments");
        uint64_t raw = (uint64_t)height * ((uint64_t)width * channels + 1);
        *out_len = (size_t)(raw + (raw >> 8) + 64 * 16 + 1024);
        return VR_OK;
    }
    std::vector<uint8_t> png;
    int rc = encode(image, width, height, channels, level, threads, png);
    if (rc != VR_OK) return rc;
    *out_len = png.size();
    if (!out) return VR_OK;
    if (capacity < png.size()) return vr::set_error(VR_E_INVALID, "png: output buffer too small");
    std::memcpy(out, png.data(), png.size());
    return VR_OK;
}

int vr_png_write(const char* path, const uint8_t* image, uint32_t width, uint32_t height, int channels, int level) {
    if (!path) return vr::set_error(VR_E_INVALID, "png: NULL path");
    std::vector<uint8_t> png;
    int rc = encode(image, width, height, channels, level, 0, png);
    if (rc != VR_OK) return rc;
    FILE* f = std::fopen(path, "wb");
    if (!f) return vr::set_error(VR_E_IO, std::string("png: cannot open ") + path);
    size_t n = std::fwrite(png.data(), 1, png.size(), f);
    if (std::fclose(f) != 0 || n != png.size()) return vr::set_error(VR_E_IO, std::string("png: write failed: ") + path);
    return VR_OK;
}

}  // extern "C"
