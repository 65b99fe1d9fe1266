// yrt_raytrace.hpp -- the reference's C++ host interface for the hot path, over the
// C-ABI of yrt.h (header-only; link libyrt.so).
//
// Same names, argument meaning and results as the reference (sebcossu/yocto_raytracing):
//     auto scn = yrt_cpp::load_scene(path);                     // load_scene, src/scene.cpp:113
//     yrt_cpp::build_bvh(scn, false);                           // build_bvh,  src/scene.cpp:554
//     auto hdr = yrt_cpp::raytrace(scn, {a, a, a}, res, s);     // raytrace,   src/raytrace.cpp:213
//     yrt_cpp::save_hdr_or_ldr(out, hdr);                       // image.cpp:81
//     yrt_cpp::intersect_first(scn, ray) / intersect_any(...)   // scene.h:236-237
// image4f is the reference's framebuffer (image.h:8-17): width, height, row-major
// pixels[j*width+i] of RGBA float. The render runs on the GPU; the scene is copied
// to HBM on the first render/trace call and stays resident with the scene.
//
// Error behaviour: the reference exits in the loader (scene.cpp:119-122) and has no
// status on the hot path; here every failure throws yrt_cpp::error carrying the
// yrt status code and message (a host program that wants the reference's behaviour
// catches it in main and exits).
#pragma once

#include <cfloat>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "yrt.h"

namespace yrt_cpp {

struct vec3f {
    float x = 0, y = 0, z = 0;
};
struct vec4f {
    float x = 0, y = 0, z = 0, w = 0;
};

// image4f, image.h:8-17
struct image4f {
    int width = 0, height = 0;
    std::vector<vec4f> pixels;

    image4f() {}
    image4f(int w, int h) : width(w), height(h), pixels((size_t)w * h) {}
    vec4f& at(int i, int j) { return pixels[(size_t)j * width + i]; }
    const vec4f& at(int i, int j) const { return pixels[(size_t)j * width + i]; }
};

// ray3f, vmath.h:264-271 (defaults tmin 1e-4, tmax FLT_MAX)
struct ray3f {
    vec3f o, d = {0, 0, 1};
    float tmin = 1e-4f, tmax = FLT_MAX;
};

// intersection3f, scene.h:227-234; `ist` is the instance index (-1: miss) instead of
// a pointer into the host scene
struct intersection3f {
    int ist = -1;
    int ei = -1;
    vec4f ew;
    float dist = 0;
    explicit operator bool() const { return ist >= 0; }
};

class error : public std::runtime_error {
   public:
    error(int status, const std::string& what) : std::runtime_error(what), status(status) {}
    int status;
};

inline void check(int status, const char* where) {
    if (status != YRT_OK) {
        std::string msg = std::string(where) + ": " + yrt_status_string(status);
        const char* detail = yrt_last_error();
        if (detail && *detail) msg += std::string(" (") + detail + ")";
        throw error(status, msg);
    }
}

// the reference's scene* (scene.h:136-155): host arrays + BVH, plus the device copies
struct scene {
    yrt_host_scene* host = nullptr;
    int device = 0;                          // GPU used by raytrace/intersect_* (gpus == 1)
    int gpus = 1;                            // raytrace on GPUs device..device+gpus-1 (yrt_multi)
    yrt_render_params params{};              // extras beyond the reference's signature
    mutable std::map<int, yrt_scene*> dev;   // uploaded lazily, one per device
    mutable yrt_multi* multi = nullptr;      // the replicas for gpus > 1, made lazily
    mutable int multi_key[2] = {-1, 0};      // {device, gpus} of `multi`

    scene() { yrt_render_params_default(&params); }
    scene(const scene&) = delete;
    scene& operator=(const scene&) = delete;
    ~scene() {
        release();
        if (host) yrt_host_scene_free(host);
    }
    void release() const {
        for (auto& kv : dev) yrt_scene_free(kv.second);
        dev.clear();
        if (multi) yrt_multi_free(multi);
        multi = nullptr;
    }
    yrt_multi* on_devices() const {
        if (multi && multi_key[0] == device && multi_key[1] == gpus) return multi;
        if (multi) yrt_multi_free(multi);
        multi = nullptr;
        std::vector<int> ids(gpus);
        for (int k = 0; k < gpus; k++) ids[k] = device + k;
        check(yrt_multi_create(host, ids.data(), gpus, &multi), "yrt_multi_create");
        multi_key[0] = device, multi_key[1] = gpus;
        return multi;
    }
    yrt_scene* on_device() const {
        auto it = dev.find(device);
        if (it != dev.end()) return it->second;
        yrt_scene* ds = nullptr;
        check(yrt_scene_upload(host, device, &ds), "yrt_scene_upload");
        dev[device] = ds;
        return ds;
    }
};

// load_scene (src/scene.cpp:113-225): Yocto OBJ or .yrtscene
inline std::unique_ptr<scene> load_scene(const std::string& filename) {
    auto scn = std::make_unique<scene>();
    check(yrt_scene_load(filename.c_str(), &scn->host), "load_scene");
    return scn;
}

// build_bvh (src/scene.cpp:554-565)
inline void build_bvh(const std::unique_ptr<scene>& scn, bool equal_num) {
    scn->release();
    check(yrt_host_scene_build_bvh(scn->host, equal_num ? 1 : 0), "build_bvh");
}

// raytrace (src/raytrace.cpp:213-254): resolution = vertical size, samples per axis.
// With scn->gpus > 1 the frame is split over that many GPUs (8-row bands, RCCL gather).
inline image4f raytrace(const std::unique_ptr<scene>& scn, const vec3f& amb, int resolution, int samples) {
    yrt_scene* ds = scn->on_device();
    yrt_render_params p = scn->params;
    p.ambient[0] = amb.x, p.ambient[1] = amb.y, p.ambient[2] = amb.z;
    p.resolution = resolution;
    p.samples = samples;
    int w = 0, h = 0;
    check(yrt_image_size(ds, &p, &w, &h), "raytrace");
    image4f img(w, h);
    if (scn->gpus > 1)
        check(yrt_multi_render(scn->on_devices(), &p, &img.pixels[0].x, YRT_MEM_HOST), "raytrace");
    else
        check(yrt_render(ds, &p, &img.pixels[0].x, YRT_MEM_HOST, nullptr), "raytrace");
    return img;
}

// counters of the last raytrace (summed over the GPUs when gpus > 1)
inline yrt_stats last_stats(const std::unique_ptr<scene>& scn) {
    yrt_stats st{};
    if (scn->gpus > 1 && scn->multi)
        check(yrt_multi_last_stats(scn->multi, &st), "last_stats");
    else
        check(yrt_last_stats(scn->on_device(), &st), "last_stats");
    return st;
}

// batch intersect_first (scene.cpp:483-488)
inline std::vector<intersection3f> intersect_first(const std::unique_ptr<scene>& scn,
                                                   const std::vector<ray3f>& rays) {
    static_assert(sizeof(ray3f) == 8 * sizeof(float), "ray3f layout");
    const int n = (int)rays.size();
    std::vector<intersection3f> out(n);
    if (!n) return out;
    std::vector<unsigned char> hit(n);
    std::vector<int> inst(n), ei(n);
    std::vector<float> ew(4 * (size_t)n), dist(n);
    check(yrt_trace_first(scn->on_device(), &rays[0].o.x, n, hit.data(), inst.data(), ei.data(), ew.data(),
                          dist.data(), YRT_MEM_HOST, nullptr),
          "intersect_first");
    for (int k = 0; k < n; k++) {
        if (!hit[k]) continue;
        out[k].ist = inst[k];
        out[k].ei = ei[k];
        out[k].ew = {ew[4 * k], ew[4 * k + 1], ew[4 * k + 2], ew[4 * k + 3]};
        out[k].dist = dist[k];
    }
    return out;
}

// batch intersect_any (scene.cpp:489-493)
inline std::vector<bool> intersect_any(const std::unique_ptr<scene>& scn, const std::vector<ray3f>& rays) {
    const int n = (int)rays.size();
    std::vector<unsigned char> hit(n);
    if (n) check(yrt_trace_any(scn->on_device(), &rays[0].o.x, n, hit.data(), YRT_MEM_HOST, nullptr), "intersect_any");
    return std::vector<bool>(hit.begin(), hit.end());
}

inline intersection3f intersect_first(const std::unique_ptr<scene>& scn, const ray3f& ray) {
    return intersect_first(scn, std::vector<ray3f>{ray})[0];
}
inline bool intersect_any(const std::unique_ptr<scene>& scn, const ray3f& ray) {
    return intersect_any(scn, std::vector<ray3f>{ray})[0];
}

// save_hdr_or_ldr (src/image.cpp:81-88)
inline void save_hdr_or_ldr(const std::string& filename, const image4f& img) {
    check(yrt_save_image(filename.c_str(), img.pixels.empty() ? nullptr : &img.pixels[0].x, img.width, img.height),
          "save_hdr_or_ldr");
}

}  // namespace yrt_cpp
