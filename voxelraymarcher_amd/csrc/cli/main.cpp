// VoxelRaymarcher CLI -- the reference's command line (main/Main.cu:176-229)
// on the MI355X renderer:
//   VoxelRaymarcher [scale] {hashtable|vcs} {original|longestaxis}
//                   [--scene resources/scene.vox] [--width 1920] [--height 1080]
//                   [--out output.png] [--device 0] [--synth N] [--repeat K]
//                   [--write-vxb F]   (convert the scene to the .vxb sidecar and exit)
//                   [--no-shadows] [--point-light X,Y,Z] [--light-dir X,Y,Z] [--light-color R,G,B]
//                   (the setupConstantValues toggles, Main.cu:26-42, as flags)
//                   [--gpus N]   (the frame image-tiled over devices 0..N-1 of the node and
//                                 gathered to device 0 over RCCL: multi_gpu.h; N = 1 takes the
//                                 same RCCL path with one rank)
// Defaults follow Main.cu: VCS unless "hashtable", longest axis unless
// "original" (:45-68), 1920x1080 (:195-196), camera (6,2,6)->(0,0,-1) fov 60
// (:199), translation 0 (:215), scene file resources/scene.vox (:96-103).
// The kernel time is measured with HIP events (the reference: std::chrono
// around launch + sync, :114,160-162).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "multi_gpu.h"
#include "vr.hpp"

namespace {

// "x,y,z" -> 3 floats; false on malformed input.
bool parse_vec3(const char* s, float out[3]) {
    char* end = nullptr;
    for (int i = 0; i < 3; ++i) {
        out[i] = std::strtof(s, &end);
        if (end == s) return false;
        s = end;
        if (i < 2) {
            if (*s != ',') return false;
            ++s;
        }
    }
    return *s == 0;
}

bool is_integer(const char* s) {
    if (!s || !*s) return false;
    if (*s == '-' || *s == '+') ++s;
    if (!*s) return false;
    for (; *s; ++s)
        if (*s < '0' || *s > '9') return false;
    return true;
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
    int device = 0, repeat = 1, gpus = 0;
    bool multi = false;                      // --gpus given: the RCCL-tiled frame
    bool shadows = true, point_light = false, has_dir = false;
    float light_pos[3] = {10.0f, 10.0f, -10.0f}, light_dir[3] = {1.0f, 1.0f, 1.0f}, light_color[3] = {1.0f, 1.0f, 1.0f};
    auto vec3 = [](const char* name, const char* v, float out[3]) {
        if (!parse_vec3(v, out)) { std::cerr << name << " needs X,Y,Z" << std::endl; std::exit(2); }
    };
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
        else if (a == "--gpus") { multi = true; gpus = std::atoi(next("--gpus")); }
        else if (a == "--repeat") repeat = std::max(1, std::atoi(next("--repeat")));
        else if (a == "--write-vxb") vxb_path = next("--write-vxb");
        else if (a == "--no-shadows") shadows = false;
        else if (a == "--point-light") { point_light = true; vec3("--point-light", next("--point-light"), light_pos); }
        else if (a == "--light-dir") { has_dir = true; vec3("--light-dir", next("--light-dir"), light_dir); }
        else if (a == "--light-color") vec3("--light-color", next("--light-color"), light_color);
        else if (a == "-h" || a == "--help") {
            std::cout << "usage: VoxelRaymarcher [scale] {hashtable|vcs} {original|longestaxis} [--scene F] "
                         "[--width W] [--height H] [--out F] [--device N] [--synth N] [--repeat K] [--write-vxb F] "
                         "[--no-shadows] [--point-light X,Y,Z] [--light-dir X,Y,Z] [--light-color R,G,B] [--gpus N]" << std::endl;
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
    if (multi && (gpus < 1 || gpus > ndev)) {
        std::cerr << "ERROR: --gpus " << gpus << ": " << ndev << " HIP device(s) visible (need 1.." << ndev << ")"
                  << std::endl;
        return 2;
    }
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
        if (has_dir) vrx::setLightDirection(lit, light_dir[0], light_dir[1], light_dir[2]);
        for (int i = 0; i < 3; ++i) {
            lit.light_color[i] = light_color[i];
            lit.light_pos[i] = light_pos[i];
        }
        lit.use_point_light = point_light;                       // Main.cu:37
        lit.use_shadows = shadows;                               // Main.cu:40

        if (multi) {
            // The frame image-tiled over devices 0..gpus-1, RCCL-gathered to device 0 (multi_gpu.h)
            vrx::MultiGpuFrame mg;
            if (!mg.init(gpus, (vr_store)store, cpu.coords(), cpu.colors(), width, height)) {
                std::cerr << "ERROR: " << mg.error() << std::endl;
                return 1;
            }
            const float t[3] = {sinfo.translationVector.x, sinfo.translationVector.y, sinfo.translationVector.z};
            vrx::MultiGpuTiming best, tm;
            best.frame_ms = 1e30;
            for (int r = 0; r < repeat; ++r) {
                if (!mg.render((vr_algo)algo, camera.raw(), lit, t, sinfo.scale, &tm)) {
                    std::cerr << "ERROR: " << mg.error() << std::endl;
                    return 1;
                }
                if (tm.frame_ms < best.frame_ms) best = tm;
            }
            std::cout << "Execution Time for Ray Marching Algorithm is: " << (long long)(best.frame_ms * 1000.0)
                      << " microseconds on " << gpus << " GPU(s), tiled + RCCL gather + assembly ("
                      << (double)width * height / (best.frame_ms * 1e3) << " Mrays/s)" << std::endl;
            for (size_t i = 0; i < best.rank_render_ms.size(); ++i)
                std::cout << "  rank " << i << " render " << (long long)(best.rank_render_ms[i] * 1000.0f)
                          << " microseconds" << std::endl;
            std::vector<uint8_t> host;
            if (!mg.download(host)) {
                std::cerr << "ERROR: " << mg.error() << std::endl;
                return 1;
            }
            if (vr_png_write(out_path.c_str(), host.data(), width, height, 3, 6) != VR_OK) {
                std::cerr << "ERROR: Failed to write image to: " << out_path << " (" << vr_last_error() << ")" << std::endl;
                return 1;
            }
            std::cout << "Wrote " << out_path << std::endl;
            return 0;
        }
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
        // writeResultingImageToDisk (Main.cu:165-174): RGB8 pack on the device,
        // async copy into pinned memory, parallel PNG encode (vr_png_write).
        const size_t nbytes = (size_t)width * height * 3;
        uint8_t* host = nullptr;
        HIP_OK(hipHostMalloc((void**)&host, nbytes, hipHostMallocDefault));
        auto t0 = std::chrono::steady_clock::now();
        vrx::check(vr_pack_rgb8(fb, rgb, (uint64_t)width * height, nullptr), "pack");
        HIP_OK(hipMemcpyAsync(host, rgb, nbytes, hipMemcpyDeviceToHost, nullptr));
        HIP_OK(hipStreamSynchronize(nullptr));
        auto t1 = std::chrono::steady_clock::now();
        int rc = vr_png_write(out_path.c_str(), host, width, height, 3, 6);
        auto t2 = std::chrono::steady_clock::now();
        (void)hipHostFree(host);
        (void)hipFree(fb);
        (void)hipFree(rgb);
        if (rc != VR_OK) {
            std::cerr << "ERROR: Failed to write image to: " << out_path << " (" << vr_last_error() << ")" << std::endl;
            return 1;
        }
        std::cout << "Wrote " << out_path << " (pack+copy "
                  << std::chrono::duration<double, std::milli>(t1 - t0).count() << " ms, png "
                  << std::chrono::duration<double, std::milli>(t2 - t1).count() << " ms)" << std::endl;
    } catch (const vrx::Error& e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
    return 0;
}
