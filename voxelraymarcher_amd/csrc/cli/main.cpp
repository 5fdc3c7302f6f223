// VoxelRaymarcher CLI -- the reference's command line (main/Main.cu:176-229)
// on the MI355X renderer:
//   VoxelRaymarcher [scale] {hashtable|vcs} {original|longestaxis}
//                   [--scene resources/scene.vox] [--width 1920] [--height 1080]
//                   [--out output.png] [--device 0] [--synth N] [--repeat K]
//                   [--write-vxb F]   (convert the scene to the .vxb sidecar and exit)
// Defaults follow Main.cu: VCS unless "hashtable", longest axis unless
// "original" (:45-68), 1920x1080 (:195-196), camera (6,2,6)->(0,0,-1) fov 60
// (:199), translation 0 (:215), scene file resources/scene.vox (:96-103).
// The kernel time is measured with HIP events (the reference: std::chrono
// around launch + sync, :114,160-162).
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "vr.hpp"

namespace {

bool is_integer(const char* s) {
    if (!s || !*s) return false;
    if (*s == '-' || *s == '+') ++s;
    if (!*s) return false;
    for (; *s; ++s)
        if (*s < '0' || *s > '9') return false;
    return true;
}

void put32(std::vector<unsigned char>& v, uint32_t x) {
    v.push_back((unsigned char)(x >> 24)); v.push_back((unsigned char)(x >> 16));
    v.push_back((unsigned char)(x >> 8)); v.push_back((unsigned char)x);
}

void chunk(FILE* f, const char* type, const std::vector<unsigned char>& data) {
    std::vector<unsigned char> buf;
    put32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    uLong crc = crc32(0L, Z_NULL, 0);
    crc = crc32(crc, buf.data() + 4, (uInt)(buf.size() - 4));
    put32(buf, (uint32_t)crc);
    fwrite(buf.data(), 1, buf.size(), f);
}

// ImageWriter::writeImage -> stbi_write_png (ImageWriter.cpp:8-16): 8-bit RGB PNG.
bool write_png(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h) {
    std::vector<unsigned char> raw((size_t)(3 * w + 1) * h);
    for (uint32_t y = 0; y < h; ++y) {
        raw[(size_t)y * (3 * w + 1)] = 0;
        std::memcpy(&raw[(size_t)y * (3 * w + 1) + 1], rgb + (size_t)y * 3 * w, 3 * (size_t)w);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<unsigned char> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
    z.resize(zlen);
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    fwrite(sig, 1, 8, f);
    std::vector<unsigned char> ihdr;
    put32(ihdr, w); put32(ihdr, h);
    ihdr.push_back(8); ihdr.push_back(2); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
    chunk(f, "IHDR", ihdr);
    chunk(f, "IDAT", z);
    chunk(f, "IEND", {});
    return std::fclose(f) == 0;
}

#define HIP_OK(x)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::cerr << #x << ": " << hipGetErrorString(e_) << std::endl;               \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

}  // namespace

int main(int argc, char* argv[]) {
    std::vector<const char*> pos;
    std::string scene_path = "resources/scene.vox", out_path = "output.png", vxb_path;
    uint32_t width = 1920, height = 1080, synth = 0;
    int device = 0, repeat = 1;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&](const char* name) -> const char* {
            if (i + 1 >= argc) { std::cerr << name << " needs a value" << std::endl; std::exit(2); }
            return argv[++i];
        };
        if (a == "--scene") scene_path = next("--scene");
        else if (a == "--out") out_path = next("--out");
        else if (a == "--width") width = (uint32_t)std::strtoul(next("--width"), nullptr, 10);
        else if (a == "--height") height = (uint32_t)std::strtoul(next("--height"), nullptr, 10);
        else if (a == "--device") device = std::atoi(next("--device"));
        else if (a == "--synth") synth = (uint32_t)std::strtoul(next("--synth"), nullptr, 10);
        else if (a == "--repeat") repeat = std::max(1, std::atoi(next("--repeat")));
        else if (a == "--write-vxb") vxb_path = next("--write-vxb");
        else if (a == "-h" || a == "--help") {
            std::cout << "usage: VoxelRaymarcher [scale] {hashtable|vcs} {original|longestaxis} [--scene F] "
                         "[--width W] [--height H] [--out F] [--device N] [--synth N] [--repeat K] [--write-vxb F]" << std::endl;
            return 0;
        } else pos.push_back(argv[i]);
    }
    if (!vxb_path.empty()) {                 // scene conversion only: no GPU needed
        try {
            vrx::VoxelFile::writeBinary(scene_path, vxb_path);
        } catch (const vrx::Error& e) {
            std::cerr << e.what() << std::endl;
            return 1;
        }
        std::cout << "wrote " << vxb_path << std::endl;
        return 0;
    }
    // argv[1] = scale (Main.cu:181-186); optional here (README.md:22-25 omits it).
    uint32_t scale = 1;
    size_t p = 0;
    if (p < pos.size() && is_integer(pos[p])) scale = (uint32_t)std::atoi(pos[p++]);
    const char* store_arg = p < pos.size() ? pos[p++] : "";
    const char* algo_arg = p < pos.size() ? pos[p++] : "";
    vrx::StorageType store = vrx::StorageType::VOXEL_CLUSTER_STORE;
    if (std::strcmp(store_arg, "hashtable") == 0) {          // Main.cu:45-55
        std::cout << "Storage Type: Cuckoo Hash Table" << std::endl;
        store = vrx::StorageType::HASH_TABLE;
    } else {
        std::cout << "Storage Type: Voxel Cluster Storage" << std::endl;
    }
    vrx::RayMarchAlgorithm algo = vrx::RayMarchAlgorithm::LONGEST_AXIS;
    if (std::strcmp(algo_arg, "original") == 0) {            // Main.cu:58-68
        std::cout << "Raymarching Algorithm: Original" << std::endl;
        algo = vrx::RayMarchAlgorithm::ORIGINAL;
    } else {
        if (std::strcmp(algo_arg, "optimized") == 0)          // :71-80 launches nothing; we render
            std::cout << "Optimized functions are currently disabled" << std::endl;
        std::cout << "Raymarching Algorithm: Longest Axis" << std::endl;
    }

    int ndev = 0;
    HIP_OK(hipGetDeviceCount(&ndev));
    std::printf("Device Count: %d\n", ndev);                   // pickCudaDevice (:82-94)
    if (device >= ndev) { std::cerr << "no such device" << std::endl; return 1; }
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device));
    std::printf("Device: %s (%s)\n", prop.name, prop.gcnArchName);
    HIP_OK(hipSetDevice(device));

    try {
        vrx::VoxelSceneCPU cpu;
        if (synth) {
            vr_synth_params sp{synth, 1.0, 0.3, 0.08, 0x256};
            size_t n = 0;
            vrx::check(vr_synth_generate(&sp, nullptr, nullptr, 0, &n), "synth");
            std::vector<int32_t> xyz(3 * n + 3);
            std::vector<uint32_t> rgb(n + 1);
            vrx::check(vr_synth_generate(&sp, xyz.data(), rgb.data(), n, &n), "synth");
            for (size_t i = 0; i < n; ++i) cpu.insertVoxel(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], rgb[i]);
        } else {
            vrx::VoxelFile::readVoxelFile(cpu, scene_path);
        }
        vrx::DeviceScene scene = cpu.generateVoxelScene(store, device);
        vr_scene_info info = scene.info();
        uint64_t slots = (uint64_t)info.diameter * info.diameter * info.diameter;
        std::cout << "There are : " << info.region_count << "/" << slots << " regions that are filled" << std::endl;

        float aspect = (float)width / (float)height;             // Main.cu:197
        vrx::Camera camera({6.0f, 2.0f, 6.0f}, {0.0f, 0.0f, -1.0f}, {0.0f, 1.0f, 0.0f}, 60.0f, aspect);
        vrx::VoxelSceneInfo sinfo({0.0f, 0.0f, 0.0f}, scale);
        vr_lighting lit = vrx::defaultLighting();

        uint32_t* fb = nullptr;
        uint8_t* rgb = nullptr;
        HIP_OK(hipMalloc(&fb, (size_t)width * height * 4));
        HIP_OK(hipMalloc(&rgb, (size_t)width * height * 3));
        hipEvent_t e0, e1;
        HIP_OK(hipEventCreate(&e0));
        HIP_OK(hipEventCreate(&e1));
        float best_ms = 1e30f;
        for (int r = 0; r < repeat; ++r) {
            HIP_OK(hipEventRecord(e0, nullptr));
            vrx::runRaymarchingKernel(width, height, algo, camera, sinfo, scene, lit, fb, nullptr);
            HIP_OK(hipEventRecord(e1, nullptr));
            HIP_OK(hipEventSynchronize(e1));
            float ms = 0;
            HIP_OK(hipEventElapsedTime(&ms, e0, e1));
            best_ms = std::min(best_ms, ms);
        }
        std::cout << hipGetErrorString(hipGetLastError()) << std::endl;
        std::cout << "Execution Time for Ray Marching Algorithm is: " << (long long)(best_ms * 1000.0f)
                  << " microseconds (" << (double)width * height / (best_ms * 1e3) << " Mrays/s)" << std::endl;
        vrx::check(vr_pack_rgb8(fb, rgb, (uint64_t)width * height, nullptr), "pack");
        std::vector<uint8_t> host((size_t)width * height * 3);
        HIP_OK(hipMemcpy(host.data(), rgb, host.size(), hipMemcpyDeviceToHost));
        if (!write_png(out_path.c_str(), host.data(), width, height)) {
            std::cerr << "cannot write " << out_path << std::endl;
            return 1;
        }
        std::cout << "Wrote " << out_path << std::endl;
        (void)hipFree(fb);
        (void)hipFree(rgb);
    } catch (const vrx::Error& e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
    return 0;
}
