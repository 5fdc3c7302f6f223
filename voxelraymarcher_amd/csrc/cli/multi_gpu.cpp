// multi_gpu.cpp -- see multi_gpu.h.  One host thread drives every device: HIP calls on a
// device's stream after hipSetDevice(device); the RCCL gather of all ranks is enqueued in
// ONE ncclGroupStart/End (one thread, several communicators, as rccl.h requires).
#include "multi_gpu.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>

namespace vrx {

namespace {
std::string hip_msg(hipError_t e) { return hipGetErrorString(e); }
}  // namespace

bool MultiGpuFrame::fail(const std::string& msg) {
    err_ = msg;
    return false;
}

MultiGpuFrame::~MultiGpuFrame() {
    for (Rank& r : ranks_) {
        (void)hipSetDevice(r.device);
        if (r.stream) (void)hipStreamSynchronize((hipStream_t)r.stream);
        if (r.comm) (void)ncclCommDestroy((ncclComm_t)r.comm);
        if (r.ev0) (void)hipEventDestroy((hipEvent_t)r.ev0);
        if (r.ev1) (void)hipEventDestroy((hipEvent_t)r.ev1);
        if (r.words) (void)hipFree(r.words);
        if (r.rgb) (void)hipFree(r.rgb);
        if (r.stream) (void)hipStreamDestroy((hipStream_t)r.stream);
        vr_scene_destroy(r.scene);
    }
    if (!ranks_.empty()) {
        (void)hipSetDevice(ranks_[0].device);
        if (gathered_) (void)hipFree(gathered_);
        if (frame_) (void)hipFree(frame_);
    }
}

bool MultiGpuFrame::init(int ngpus, vr_store store, const std::vector<int32_t>& xyz, const std::vector<uint32_t>& rgb,
                         uint32_t width, uint32_t height, uint32_t band_rows, uint32_t tile_cols) {
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess) visible = 0;
    if (ngpus < 1) return fail("--gpus must be >= 1");
    if (ngpus > visible)
        return fail("--gpus " + std::to_string(ngpus) + " but only " + std::to_string(visible) +
                    " HIP device(s) are visible");
    if (!width || !height || !band_rows || !tile_cols || tile_cols > width) return fail("bad frame / tile layout");
    W_ = width;
    H_ = height;
    band_rows_ = band_rows;
    tile_cols_ = tile_cols;
    rank_words_ = vr_tile_buffer_words(width, height, band_rows, tile_cols, (uint32_t)ngpus);
    ranks_.resize((size_t)ngpus);
    std::vector<int> devs((size_t)ngpus);
    const size_t n = rgb.size();
    for (int i = 0; i < ngpus; ++i) {
        Rank& r = ranks_[(size_t)i];
        r.device = devs[(size_t)i] = i;
        hipError_t e = hipSetDevice(i);
        if (e != hipSuccess) return fail("hipSetDevice(" + std::to_string(i) + "): " + hip_msg(e));
        // the scene is replicated: each device builds its own from the host voxels (VR_BUILD_AUTO =
        // the device build), as every rank of the torch.distributed bench does
        if (vr_scene_create(i, store, xyz.data(), rgb.data(), n, &r.scene) != VR_OK)
            return fail("scene on device " + std::to_string(i) + ": " + vr_last_error());
        hipStream_t st = nullptr;
        e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (e != hipSuccess) return fail("hipStreamCreate: " + hip_msg(e));
        r.stream = st;
        hipEvent_t a = nullptr, b = nullptr;
        if ((e = hipEventCreate(&a)) != hipSuccess || (e = hipEventCreate(&b)) != hipSuccess)
            return fail("hipEventCreate: " + hip_msg(e));
        r.ev0 = a;
        r.ev1 = b;
        if ((e = hipMalloc(&r.words, rank_words_ * 4)) != hipSuccess || (e = hipMalloc(&r.rgb, rank_words_ * 3)) != hipSuccess)
            return fail("rank buffers on device " + std::to_string(i) + ": " + hip_msg(e));
    }
    hipError_t e = hipSetDevice(0);
    if (e == hipSuccess) e = hipMalloc(&gathered_, rank_words_ * 3 * (size_t)ngpus);
    if (e == hipSuccess) e = hipMalloc(&frame_, (size_t)width * height * 3);
    if (e != hipSuccess) return fail("device 0 frame buffers: " + hip_msg(e));
    std::vector<ncclComm_t> comms((size_t)ngpus);
    const ncclResult_t nr = ncclCommInitAll(comms.data(), ngpus, devs.data());
    if (nr != ncclSuccess) return fail(std::string("ncclCommInitAll: ") + ncclGetErrorString(nr));
    for (int i = 0; i < ngpus; ++i) ranks_[(size_t)i].comm = comms[(size_t)i];
    return true;
}

bool MultiGpuFrame::render(vr_algo algo, const vr_camera& cam, const vr_lighting& lit, const float translation[3],
                           uint32_t scale, MultiGpuTiming* timing) {
    const uint32_t N = (uint32_t)ranks_.size();
    if (!N) return fail("not initialised");
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < N; ++i) {                 // every rank's tiles, on its own stream
        Rank& r = ranks_[i];
        hipError_t e = hipSetDevice(r.device);
        if (e == hipSuccess) e = hipEventRecord((hipEvent_t)r.ev0, (hipStream_t)r.stream);
        if (e != hipSuccess) return fail("rank " + std::to_string(i) + ": " + hip_msg(e));
        if (vr_render_tiles(r.scene, algo, &cam, &lit, translation, scale, W_, H_, band_rows_, tile_cols_, i, N,
                            r.words, r.stream) != VR_OK ||
            vr_pack_rgb8(r.words, r.rgb, rank_words_, r.stream) != VR_OK)
            return fail("rank " + std::to_string(i) + ": " + vr_last_error());
        if ((e = hipEventRecord((hipEvent_t)r.ev1, (hipStream_t)r.stream)) != hipSuccess)
            return fail("rank " + std::to_string(i) + ": " + hip_msg(e));
    }
    // the exchange: every rank's RGB8 tiles to device 0 (equal sizes: one gather)
    ncclResult_t nr = ncclGroupStart();
    for (uint32_t i = 0; i < N && nr == ncclSuccess; ++i) {
        Rank& r = ranks_[i];
        nr = ncclGather(r.rgb, i == 0 ? gathered_ : nullptr, rank_words_ * 3, ncclUint8, 0, (ncclComm_t)r.comm,
                        (hipStream_t)r.stream);
    }
    const ncclResult_t ng = ncclGroupEnd();
    if (nr == ncclSuccess) nr = ng;
    if (nr != ncclSuccess) return fail(std::string("ncclGather: ") + ncclGetErrorString(nr));
    Rank& r0 = ranks_[0];
    hipError_t e = hipSetDevice(r0.device);
    if (e != hipSuccess) return fail(hip_msg(e));
    if (vr_assemble_tiles(gathered_, frame_, 3, W_, H_, band_rows_, tile_cols_, N, 0, r0.stream) != VR_OK)
        return fail(std::string("assemble: ") + vr_last_error());
    if ((e = hipStreamSynchronize((hipStream_t)r0.stream)) != hipSuccess) return fail("device 0: " + hip_msg(e));
    const auto t1 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; i < N; ++i) {                 // (their gathers are done: device 0 has the data)
        if ((e = hipSetDevice(ranks_[i].device)) != hipSuccess ||
            (e = hipStreamSynchronize((hipStream_t)ranks_[i].stream)) != hipSuccess)
            return fail("rank " + std::to_string(i) + ": " + hip_msg(e));
    }
    if (timing) {
        timing->frame_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        timing->rank_render_ms.assign(N, 0.0f);
        for (uint32_t i = 0; i < N; ++i) {
            (void)hipSetDevice(ranks_[i].device);
            (void)hipEventElapsedTime(&timing->rank_render_ms[i], (hipEvent_t)ranks_[i].ev0, (hipEvent_t)ranks_[i].ev1);
        }
    }
    (void)hipSetDevice(r0.device);
    return true;
}

bool MultiGpuFrame::download(std::vector<uint8_t>& out) {
    if (ranks_.empty()) return fail("not initialised");
    out.resize((size_t)W_ * H_ * 3);
    hipError_t e = hipSetDevice(ranks_[0].device);
    if (e == hipSuccess) e = hipMemcpy(out.data(), frame_, out.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail("frame download: " + hip_msg(e));
    return true;
}

}  // namespace vrx
