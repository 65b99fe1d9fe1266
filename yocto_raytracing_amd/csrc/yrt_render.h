// yrt_render.h -- internal host API between the C-ABI layer (capi.cpp), the device
// scene builder (device_scene.cpp) and the kernel launchers (render.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <string>
#include <vector>

#include "yrt_device.h"
#include "yrt_scene.h"

namespace yrt {

// one scene resident in one GPU's HBM (a single hipMalloc arena)
struct device_scene {
    int device = 0;
    void* arena = nullptr;
    size_t arena_bytes = 0;
    dev_scene_view view = {};
    std::vector<camera> cameras;
    int top_depth = 0;    // instance-BVH depth (stack entries needed)
    int shape_depth = 0;  // deepest shape BVH
    size_t ntnodes = 0, nsnodes = 0, nsprims = 0, ninst = 0;
};

// Flatten a host scene (with BVH built) into the HBM layout and upload it.
// Throws std::runtime_error on unsupported input or HIP failure.
device_scene* device_scene_create(const scene& scn, int device);
void device_scene_destroy(device_scene* ds);

// camera constants (raytrace.cpp:16-24): h = 2*focus*tanf(fovy/2), w = h*aspect, y negated
dev_camera make_dev_camera(const camera& c);

// kernels (render.hip)
hipError_t launch_render(const device_scene& ds, const dev_render_args& args, void* out_rgba,
                         unsigned long long* counters, bool count_work, hipStream_t stream);
hipError_t launch_trace(const device_scene& ds, const float* rays, int n, int any,
                        unsigned char* hit, int* inst, int* ei, float* ew, float* dist,
                        unsigned long long* counters, hipStream_t stream);
hipError_t launch_tonemap(const float* rgba, int n, unsigned char* out, hipStream_t stream);

// stack capacities compiled into the kernels (entries per lane, LDS resident)
constexpr int top_stack_cap = 24;
constexpr int shape_stack_cap = 24;

}  // namespace yrt
