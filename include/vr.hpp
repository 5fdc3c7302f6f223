// vr.hpp -- C++ host interface over the C ABI (vr.h), mirroring the
// reference's host-side names so code written against
// lukeduball/VoxelRaymarcher reads the same:
//   StorageType            (geometry/VoxelFunctions.cuh:37)
//   Camera                 (renderer/camera/Camera.cuh:8-40)
//   VoxelSceneInfo         (renderer/VoxelSceneInfo.cuh:5-15)
//   VoxelSceneCPU          (geometry/VoxelSceneCPU.cuh:13-131)
//   VoxelFile::readVoxelFile (geometry/VoxelFile.cuh:6-37)
//   runRaymarchingKernel   (main/Main.cu:105-163)
// Errors surface as vrx::Error (the reference ignores them).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "vr.h"

namespace vrx {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, const char* where) {
    if (rc != VR_OK) throw Error(rc, std::string(where) + ": " + vr_last_error());
}

enum class StorageType { VOXEL_CLUSTER_STORE = VR_STORE_VCS, HASH_TABLE = VR_STORE_HASHTABLE };
enum class RayMarchAlgorithm { LONGEST_AXIS = VR_ALGO_LONGESTAXIS, ORIGINAL = VR_ALGO_ORIGINAL };

struct Vector3f {
    float x = 0, y = 0, z = 0;
};

class Camera {
public:
    Camera(Vector3f o, Vector3f lookAt, Vector3f globalUp, float fieldOfView, float aspectRatio) {
        float e[3] = {o.x, o.y, o.z}, l[3] = {lookAt.x, lookAt.y, lookAt.z}, u[3] = {globalUp.x, globalUp.y, globalUp.z};
        check(vr_camera_make(e, l, u, fieldOfView, aspectRatio, &cam_), "Camera");
    }
    const vr_camera& raw() const { return cam_; }

private:
    vr_camera cam_{};
};

struct VoxelSceneInfo {
    Vector3f translationVector{};
    uint32_t scale = 1;
    VoxelSceneInfo() = default;
    VoxelSceneInfo(Vector3f location, uint32_t s = 1) : translationVector(location), scale(s) {}
};

// Owns one device scene (the reference's deviceVoxelScene + per-region stores).
class DeviceScene {
public:
    DeviceScene() = default;
    explicit DeviceScene(vr_scene* s) : s_(s) {}
    DeviceScene(const DeviceScene&) = delete;
    DeviceScene& operator=(const DeviceScene&) = delete;
    DeviceScene(DeviceScene&& o) noexcept : s_(o.s_) { o.s_ = nullptr; }
    DeviceScene& operator=(DeviceScene&& o) noexcept {
        if (this != &o) { vr_scene_destroy(s_); s_ = o.s_; o.s_ = nullptr; }
        return *this;
    }
    ~DeviceScene() { vr_scene_destroy(s_); }
    const vr_scene* get() const { return s_; }
    vr_scene_info info() const {
        vr_scene_info i{};
        check(vr_scene_get_info(s_, &i), "vr_scene_get_info");
        return i;
    }

private:
    vr_scene* s_ = nullptr;
};

class VoxelSceneCPU {
public:
    void insertVoxel(int32_t x, int32_t y, int32_t z, uint32_t color) {
        xyz_.push_back(x); xyz_.push_back(y); xyz_.push_back(z);
        rgb_.push_back(color);
    }
    // Builds the storage structures and uploads them (generateVoxelScene).
    DeviceScene generateVoxelScene(StorageType storageType, int device = 0) const {
        vr_scene* s = nullptr;
        check(vr_scene_create(device, (vr_store)storageType, xyz_.data(), rgb_.data(), rgb_.size(), &s),
              "generateVoxelScene");
        return DeviceScene(s);
    }
    size_t size() const { return rgb_.size(); }
    const std::vector<int32_t>& coords() const { return xyz_; }
    const std::vector<uint32_t>& colors() const { return rgb_; }

private:
    std::vector<int32_t> xyz_;
    std::vector<uint32_t> rgb_;
};

struct VoxelFile {
    // .vox CSV or, detected by its magic, the .vxb binary sidecar.
    static void readVoxelFile(VoxelSceneCPU& scene, const std::string& path) {
        size_t n = 0;
        check(vr_scene_file_read(path.c_str(), nullptr, nullptr, 0, &n), "readVoxelFile");
        std::vector<int32_t> xyz(3 * n + 3);
        std::vector<uint32_t> rgb(n + 1);
        check(vr_scene_file_read(path.c_str(), xyz.data(), rgb.data(), n, &n), "readVoxelFile");
        for (size_t i = 0; i < n; ++i) scene.insertVoxel(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], rgb[i]);
    }
    // Write the binary sidecar of a scene file (vr_vxb_write).
    static void writeBinary(const std::string& src, const std::string& dst) {
        size_t n = 0;
        check(vr_scene_file_read(src.c_str(), nullptr, nullptr, 0, &n), "readVoxelFile");
        std::vector<int32_t> xyz(3 * n + 3);
        std::vector<uint32_t> rgb(n + 1);
        check(vr_scene_file_read(src.c_str(), xyz.data(), rgb.data(), n, &n), "readVoxelFile");
        check(vr_vxb_write(dst.c_str(), xyz.data(), rgb.data(), n), "vr_vxb_write");
    }
};

inline vr_lighting defaultLighting() {
    vr_lighting l{};
    check(vr_lighting_default(&l), "setupConstantValues");
    return l;
}

// LIGHT_DIRECTION = makeUnitVector(dir) (Main.cu:28).
inline void setLightDirection(vr_lighting& l, float x, float y, float z) {
    const float d[3] = {x, y, z};
    check(vr_lighting_set_direction(&l, d), "setLightDirection");
}

// Launch on `stream` (hipStream_t as void*); asynchronous.
inline void runRaymarchingKernel(uint32_t width, uint32_t height, RayMarchAlgorithm algo, const Camera& camera,
                                 const VoxelSceneInfo& info, const DeviceScene& scene, const vr_lighting& lighting,
                                 uint32_t* framebufferDev, void* stream = nullptr) {
    float t[3] = {info.translationVector.x, info.translationVector.y, info.translationVector.z};
    check(vr_render(scene.get(), (vr_algo)algo, &camera.raw(), &lighting, t, info.scale, width, height, 0, height,
                    framebufferDev, stream),
          "runRaymarchingKernel");
}

}  // namespace vrx
