// yrt_render.h -- internal host API between the C-ABI layer (capi.cpp), the device
// scene builder (device_scene.cpp) and the kernel launchers (render.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <string>
#include <vector>

#include "yrt_device.h"
#include "yrt_scene.h"

namespace yrt {

// per-phase GPU time of the last render call: HIP events recorded on the launch
// stream around every kernel launch of a phase (enabled by yrt_render_params.timing)
enum render_phase {
    phase_primary = 0,   // camera rays + closest hit + surface (k_primary)
    phase_shadow = 1,    // shadow rays, any hit (k_shadow)
    phase_shade = 2,     // lighting + mirror-ray compaction (k_shade)
    phase_bounce = 3,    // closest hit of mirror rays (k_bounce)
    phase_fold = 4,      // reflection fold (k_fold_children)
    phase_accumulate = 5,
    phase_megakernel = 6,
    phase_lists = 7,     // per-render records and candidate lists (k_relative_records, k_camera_lists, k_bundle_lists, k_list_stats)
    phase_count = 8
};

struct phase_timer {
    bool on = false;
    std::vector<hipEvent_t> pool;  // start/stop pairs
    std::vector<int> phase_of;     // per pair
    size_t used = 0;
    int begin(int phase, hipStream_t s);  // -1 when off
    void end(int idx, hipStream_t s);
    void reset(bool enable) {
        on = enable;
        used = 0;
    }
    // sums elapsed ms per phase (synchronises the recorded events)
    void collect(float* ms, int* launches);
    void destroy();
};

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
    size_t max_shape_nodes = 0;
    bool narrow_stack = true;  // all node indices fit 16-bit stack entries
    bool reflective = false;   // any material with kr > 0 (bounce levels needed)
    bool wide_ok = false;      // the 4-wide any-hit walk's stack fits (else the binary walk)
    // the instance-level spine records with the camera origin subtracted from every bound
    // (wavefront.hip k_relative_records, rewritten per render): the primary rays' box tests
    f4* trel = nullptr;
    int nlights = 0;
    int num_cus = 256;  // compute units of the device (persistent grids)
    // wavefront workspace (device), grown on demand
    void* work = nullptr;
    size_t work_bytes = 0;
    // mirror levels: the next level's ray count, copied back behind the level's kernels
    int* level_count_host = nullptr;  // pinned
    hipEvent_t level_count_ev = nullptr;
    // the candidate lists (wavefront.hip k_camera_lists / k_bundle_lists): each render that
    // builds them sums their lengths on the device and copies the sums back behind its kernels
    // (yrt_scene_tile_lists reads them). Lists on or off give the same image.
    // pinned: {camera entries, camera tiles, bundle entries, bundle lists, instances the camera
    // lists' masks exclude, instances the bundle lists' masks exclude} (wavefront.hip list_sums)
    unsigned long long* list_stats_host = nullptr;
    hipEvent_t list_stats_ev = nullptr;
    bool list_stats_recorded = false;  // list_stats_ev has been recorded (yrt_scene_tile_lists waits on it)
    // YRT_LISTS_AUTO / YRT_LISTS_ON: lists whenever the scene allows (ON also puts level 0's
    // shadow rays on the persistent grid at any frame size); YRT_LISTS_OFF: never
    int lists_mode = 0;
    bool last_camera_lists = false, last_bundles = false;  // what the last render used
    // yrt_scene_set_lds_staging: the persistent walks read the instance tree's top from LDS
    int lds_staging = 0;
    int last_lds_staging = 0;  // what the last render staged: bit 0 closest hit, bit 1 any hit
    phase_timer timer;
};

// Flatten a host scene (with BVH built) into the HBM layout and upload it.
// Throws std::runtime_error on unsupported input or HIP failure.
device_scene* device_scene_create(const scene& scn, int device);
void device_scene_destroy(device_scene* ds);

// camera constants (raytrace.cpp:16-24): h = 2*focus*tanf(fovy/2), w = h*aspect, y negated
dev_camera make_dev_camera(const camera& c);

// kernels (render.hip)
hipError_t launch_render(device_scene& ds, const dev_render_args& args, void* out_rgba,
                         unsigned long long* counters, bool count_work, hipStream_t stream);
hipError_t launch_trace(const device_scene& ds, const float* rays, int n, int any,
                        unsigned char* hit, int* inst, int* ei, float* ew, float* dist,
                        unsigned long long* counters, bool packet, hipStream_t stream);
// tonemap on the device against the host's thresholds (tonemap_thresholds): bit-exact
// with tonemap_rgba8, i.e. with the host libm's powf
struct tonemap_table {
    float thr[256];
    int neg_inf_level;  // pow(-inf, 1/2.2) = +inf: the one non-positive input that is not 0
};
hipError_t launch_tonemap(const float* rgba, int n, unsigned char* out, const tonemap_table& table,
                          hipStream_t stream);
// the .hdr writer's RGBE bytes on the device (rgbe.h; the layout of rgbe_encode)
hipError_t launch_rgbe(const float* rgba, int w, int h, unsigned char* out, hipStream_t stream);

// mirror levels the megakernel records per lane (render.hip); the wavefront pipeline
// keeps per-level records in HBM and takes any max_depth
constexpr int megakernel_max_depth = 16;

// traversal stack entries per lane (LDS resident): instance level + shape level
constexpr int traversal_stack_cap = 40;

// wavefront pipeline (wavefront.hip): same contract as launch_render
hipError_t launch_render_wavefront(device_scene& ds, const dev_render_args& args, void* out_rgba,
                                   unsigned long long* counters, bool count_work, bool packet, hipStream_t stream);

}  // namespace yrt
