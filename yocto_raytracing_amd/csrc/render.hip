// render.hip -- gfx950 kernels with one lane per pixel (the "megakernel" render:
// raytrace(), src/raytrace.cpp:213-254, with shade() inlined), the batch
// intersect_first / intersect_any queries (src/scene.cpp:483-494) and tonemap
// (src/image.cpp:55-77). The default render path is the wavefront pipeline in
// wavefront.hip; this megakernel is kept as the structurally simplest restatement
// (one lane walks the reference's loops) and as an A/B baseline.
//
// Parity contract: see trace_common.h. Per pixel the s*s samples
// are summed in the reference's jj-major / ii-minor order.
#include <hip/hip_runtime.h>

#include "packet_trace.h"
#include "rgbe.h"
#include "trace_common.h"
#include "yrt_render.h"

namespace yrt {
namespace {

constexpr int BLOCK_X = 16, BLOCK_Y = 8, BLOCK = BLOCK_X * BLOCK_Y;
constexpr int MAX_BOUNCES = megakernel_max_depth;  // compile-time size of the per-level shading records

template <typename SE>
struct lane_state {
    SE* stk;  // this lane's column of the LDS traversal stack (16- or 32-bit node indices)
    work_counts wc;
    unsigned long long rays = 0;
    unsigned long long truncated = 0;
};

// shade() (raytrace.cpp:88-211) with the recursion unrolled: level k records its
// light sum D_k, ambient la_k and kr_k; the result folds back to front as
// R_k = (D_k + R_{k+1}*kr_k) + la_k, the reference's accumulation order (:182,203,206).
template <bool COUNT, typename SE>
__device__ vec3f shade_path(const dev_scene_view& S, const dev_render_args& A, ray3 ray, lane_state<SE>& L) {
    vec3f rec_d[MAX_BOUNCES], rec_la[MAX_BOUNCES], rec_kr[MAX_BOUNCES];
    int depth = 0;
    vec3f R = {0, 0, 0};
    int max_depth = A.max_depth < MAX_BOUNCES ? A.max_depth : MAX_BOUNCES;
    for (;;) {
        hit_record hr = {-1, -1, {0, 0, 0, 0}, 0};
        L.rays++;
        if (!traverse<false, COUNT, BLOCK>(S, ray, hr, L.stk, L.wc)) {
            R = {0, 0, 0};
            break;
        }
        if (COUNT) L.wc.hits++;
        surface sf = eval_surface(S, hr.slot, hr.ei, hr.ew);
        float4 m0 = ld4(S.mats + 4 * sf.mat), m1 = ld4(S.mats + 4 * sf.mat + 1);
        float4 m2 = ld4(S.mats + 4 * sf.mat + 2), m3 = ld4(S.mats + 4 * sf.mat + 3);
        vec3f kd0 = xyz(m0), ks0 = xyz(m1), kr = xyz(m2);
        float ns = m0.w;
        int kd_txt = ibits(m1.w), ks_txt = ibits(m2.w);
        bool reflective = ibits(m3.w) & mat_reflective;
        vec3f amb = {A.amb[0], A.amb[1], A.amb[2]};
        vec3f la = amb * kd0;
        vec3f tkd = {1, 1, 1}, tks = {1, 1, 1};
        if (kd_txt >= 0) {
            tkd = eval_texture<COUNT>(S, kd_txt, sf.uv, L.wc, S.srgb);
            la = la * tkd;
        }
        if (ks_txt >= 0) tks = eval_texture<COUNT>(S, ks_txt, sf.uv, L.wc, S.srgb);
        vec3f c = {0.0f, 0.0f, 0.0f};
        for (int li = 0; li < S.nlights; li++) {
            const f4* lr = S.lights + 6 * li;
            frame3f lf = {xyz(ld4(lr)), xyz(ld4(lr + 1)), xyz(ld4(lr + 2)), xyz(ld4(lr + 3))};
            vec3f lp0 = xyz(ld4(lr + 4)), ke = xyz(ld4(lr + 5));
            vec3f tp = transform_point(lf, lp0 - sf.p);
            vec3f l = normalize(tp);
            float r = length(tp);
            ray3 sr = {sf.p, l, 0.01f, r - 0.01f};
            L.rays++;
            if (occluded<COUNT, BLOCK>(S, sr, L.stk, L.wc)) continue;
            vec3f v = normalize(ray.o - sf.p);
            vec3f h = normalize(v + l);
            vec3f kd = kd0, ks = ks0;
            if (kd_txt >= 0) kd = kd * tkd;
            if (ks_txt >= 0) ks = ks * tks;
            vec3f ld = kd * (ke / (r * r));
            vec3f ls = ks * (ke / (r * r));
            if (sf.kind == kind_lines) {
                float prodnl = dot(sf.n, l);
                float prodnh = dot(sf.n, h);
                if (prodnl < 0.0f) prodnl *= -1;
                if (prodnh < 0.0f) prodnh *= -1;
                float sinnl = __builtin_sqrtf(1.0f - prodnl);
                float sinnh = __builtin_sqrtf(1.0f - prodnh);
                ld = ld * sinnl;
                ls = ls * spec_pow(sinnh, ns, ls);
            } else {
                ld = ld * smax(0.0f, dot(sf.n, l));
                ls = ls * spec_pow(smax(0.0f, dot(sf.n, h)), ns, ls);
            }
            c = c + (ld + ls);
        }
        if (!reflective) {
            R = c + la;
            break;
        }
        rec_d[depth] = c;
        rec_la[depth] = la;
        rec_kr[depth] = kr;
        depth++;
        if (depth >= max_depth) {
            // the reference recurses without bound; here the cap counts as a miss
            L.truncated++;
            R = {0, 0, 0};
            break;
        }
        vec3f v = normalize(ray.o - sf.p);
        vec3f dr = (sf.n * 2.0f * dot(sf.n, v)) - v;
        ray = {sf.p, dr, ray_eps, flt_max};
    }
    for (int k = depth - 1; k >= 0; k--) {
        vec3f c = rec_d[k];
        c = c + vec3f{R.x * rec_kr[k].x, R.y * rec_kr[k].y, R.z * rec_kr[k].z};
        R = c + rec_la[k];
    }
    return R;
}

template <bool COUNT, typename SE>
__device__ void flush_counters(unsigned long long* counters, const lane_state<SE>& L, unsigned long long samples) {
    unsigned long long vals[9] = {L.rays, samples, L.truncated, 0, L.wc.box, L.wc.inst, L.wc.prim, L.wc.hits,
                                  L.wc.tex};
    int n = COUNT ? 9 : 3;
    for (int k = 0; k < n; k++) {
        unsigned long long s = wave_sum(vals[k]);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(counter_line(counters) + k, s);
    }
}

// raytrace() (raytrace.cpp:213-254) for the window/bands in A; one lane = one pixel.
// SE: the stack entry type -- 16-bit node indices while every tree has < 65 536 nodes
// (half the LDS), 32-bit otherwise (instance100k's instance tree has 67 727)
template <bool COUNT, typename SE>
__global__ __launch_bounds__(BLOCK) void render_kernel(dev_scene_view S, dev_render_args A,
                                                       float4* __restrict__ out, unsigned long long* counters) {
    __shared__ SE lds[traversal_stack_cap * BLOCK];
    lane_state<SE> L;
    L.stk = lds + threadIdx.x;
    int lx = blockIdx.x * BLOCK_X + (threadIdx.x % BLOCK_X);
    int ly = blockIdx.y * BLOCK_Y + (threadIdx.x / BLOCK_X);
    unsigned long long samples = 0;
    if (lx < A.tile_w && ly < A.tile_h) {
        int i = A.x0 + lx;
        int b = ly / A.band, r = ly % A.band;
        int j = A.y0 + (b * A.band_stride + A.band_offset) * A.band + r;
        if (i >= A.width || j >= A.height) {
            // local rows past the image edge (last partial band of a shard) read as zeros
            out[(size_t)ly * A.out_stride + lx] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else {
            int ns = A.samples;
            vec4f acc = {0, 0, 0, 0};
            for (int jj = 0; jj < ns; jj++) {
                for (int ii = 0; ii < ns; ii++) {
                    ray3 ray = camera_ray(A.cam, A.width, A.height, ns, i, j, ii, jj);
                    vec3f c = shade_path<COUNT>(S, A, ray, L);
                    acc = {acc.x + c.x, acc.y + c.y, acc.z + c.z, acc.w + 1.0f};
                    samples++;
                }
            }
            float d = float(ns * ns);
            out[(size_t)ly * A.out_stride + lx] = make_float4(acc.x / d, acc.y / d, acc.z / d, 1.0f);
        }
    }
    flush_counters<COUNT>(counters, L, samples);
}

// batch intersect_first / intersect_any (scene.cpp:483-494), one lane per ray
constexpr int TRACE_BLOCK = 256;
template <bool ANY>
__global__ __launch_bounds__(TRACE_BLOCK) void trace_kernel(dev_scene_view S, const float* __restrict__ rays,
                                                            int n, unsigned char* hit, int* inst, int* eis,
                                                            float* ews, float* dists,
                                                            unsigned long long* counters) {
    __shared__ uint32_t lds[traversal_stack_cap * TRACE_BLOCK];
    int k = blockIdx.x * TRACE_BLOCK + threadIdx.x;
    work_counts wc;
    if (k < n) {
        const float* r = rays + (size_t)k * 8;
        ray3 ray = {{r[0], r[1], r[2]}, {r[3], r[4], r[5]}, r[6], r[7]};
        hit_record hr = {-1, -1, {0, 0, 0, 0}, 0};
        bool h = ANY ? occluded<false, TRACE_BLOCK>(S, ray, lds + threadIdx.x, wc)
                     : traverse<false, false, TRACE_BLOCK>(S, ray, hr, lds + threadIdx.x, wc);
        hit[k] = h ? 1 : 0;
        if (!ANY) {
            // intersect_first returns a default record on a miss (scene.cpp:485-486)
            inst[k] = h ? S.tinst_id[hr.slot] : -1;
            eis[k] = h ? hr.ei : -1;
            ews[4 * k + 0] = h ? hr.ew.x : 0;
            ews[4 * k + 1] = h ? hr.ew.y : 0;
            ews[4 * k + 2] = h ? hr.ew.z : 0;
            ews[4 * k + 3] = h ? hr.ew.w : 0;
            dists[k] = h ? hr.dist : 0;
        }
    }
    unsigned long long s = wave_sum(k < n ? 1ull : 0ull);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(counter_line(counters) + cnt_rays, s);
}

// the same queries through the render path's walks: the wave-coherent closest-hit walk
// and the 4-wide any-hit walk (packet_trace.h); every lane reaches the walk
template <bool ANY>
__global__ __launch_bounds__(TRACE_BLOCK) void trace_packet_kernel(dev_scene_view S, const float* __restrict__ rays,
                                                                   int n, unsigned char* hit, int* inst, int* eis,
                                                                   float* ews, float* dists,
                                                                   unsigned long long* counters) {
    const int k = blockIdx.x * TRACE_BLOCK + threadIdx.x;
    const bool valid = k < n;
    ray3 ray = {{0, 0, 0}, {0, 0, 1}, 0, 0};
    if (valid) {
        const float* r = rays + (size_t)k * 8;
        ray = {{r[0], r[1], r[2]}, {r[3], r[4], r[5]}, r[6], r[7]};
    }
    hit_record hr = {-1, -1, {0, 0, 0, 0}, 0};
    work_counts wc;
    bool h;
    if (ANY)
        h = S.wide ? packet_occluded_wide2(S, ray, valid) : packet_any<false>(S, ray, valid, wc);
    else
        h = packet_first<false>(S, ray, valid, hr, wc);
    if (valid) {
        hit[k] = h ? 1 : 0;
        if (!ANY) {
            inst[k] = h ? S.tinst_id[hr.slot] : -1;
            eis[k] = h ? hr.ei : -1;
            ews[4 * k + 0] = h ? hr.ew.x : 0;
            ews[4 * k + 1] = h ? hr.ew.y : 0;
            ews[4 * k + 2] = h ? hr.ew.z : 0;
            ews[4 * k + 3] = h ? hr.ew.w : 0;
            dists[k] = h ? hr.dist : 0;
        }
    }
    unsigned long long s = wave_sum(valid ? 1ull : 0ull);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(counter_line(counters) + cnt_rays, s);
}

// tonemap (image.cpp:55-77): exposure 0, no filmic, gamma 1/2.2, truncating *255. A
// channel's 8-bit value is the number of host thresholds at or below it (tonemap_table:
// the host powf's exact level boundaries), found by an 8-step bisection; NaN, zero and
// negative values give 0 as the select clamp does (-inf: pow gives +inf, so 255). Alpha has no pow: computed directly.
__device__ __forceinline__ unsigned char tonemap_level(const tonemap_table& T, float x) {
    if (!(x > 0.0f)) return x == -__builtin_inff() ? (unsigned char)T.neg_inf_level : 0;
    int lo = 0;  // invariant: thr[lo] <= x (thr[0] = 0 < x)
#pragma unroll
    for (int step = 128; step >= 1; step >>= 1)
        if (lo + step < 256 && T.thr[lo + step] <= x) lo += step;
    return (unsigned char)lo;
}

__global__ void tonemap_kernel(const float4* __restrict__ in, int n, uchar4* __restrict__ out, tonemap_table T) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    float4 h = in[k];
    out[k] = make_uchar4(tonemap_level(T, h.x), tonemap_level(T, h.y), tonemap_level(T, h.z),
                         (unsigned char)(sclamp(h.w, 0.0f, 1.0f) * 255));
}

// the .hdr writer's RGBE bytes (rgbe.h, stbiw__linear_to_rgbe), one lane per pixel, in
// the layout save_hdr_rgbe consumes: per row four component planes for run-length
// encoded widths (neighbouring lanes write neighbouring bytes of a plane), else
// interleaved quadruples. Only these 4 B/pixel cross PCIe instead of the 16 B floats.
__global__ void rgbe_kernel(const float4* __restrict__ in, int w, int h, unsigned char* __restrict__ out) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= (long long)w * h) return;
    const float4 p = in[k];
    unsigned char e[4];
    linear_to_rgbe(p.x, p.y, p.z, e);
    if (rgbe_rle_width(w)) {
        const long long j = k / w, i = k - j * w;
        unsigned char* row = out + j * 4 * w + i;
        row[0] = e[0], row[w] = e[1], row[2 * (long long)w] = e[2], row[3 * (long long)w] = e[3];
    } else {
        reinterpret_cast<uchar4*>(out)[k] = make_uchar4(e[0], e[1], e[2], e[3]);
    }
}

}  // namespace

hipError_t launch_rgbe(const float* rgba, int w, int h, unsigned char* out, hipStream_t stream) {
    if (w <= 0 || h <= 0) return hipSuccess;
    const long long n = (long long)w * h;
    hipLaunchKernelGGL(rgbe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const float4*)rgba, w,
                       h, out);
    return hipGetLastError();
}

hipError_t launch_render(device_scene& ds, const dev_render_args& args, void* out_rgba,
                         unsigned long long* counters, bool count_work, hipStream_t stream) {
    if (args.tile_w <= 0 || args.tile_h <= 0) return hipSuccess;
    dim3 grid((args.tile_w + BLOCK_X - 1) / BLOCK_X, (args.tile_h + BLOCK_Y - 1) / BLOCK_Y);
    int t = ds.timer.begin(phase_megakernel, stream);
#define YRT_MK(C, SE) \
    hipLaunchKernelGGL((render_kernel<C, SE>), grid, dim3(BLOCK), 0, stream, ds.view, args, (float4*)out_rgba, counters)
    if (ds.narrow_stack) {
        if (count_work)
            YRT_MK(true, uint16_t);
        else
            YRT_MK(false, uint16_t);
    } else {
        if (count_work)
            YRT_MK(true, uint32_t);
        else
            YRT_MK(false, uint32_t);
    }
#undef YRT_MK
    ds.timer.end(t, stream);
    return hipGetLastError();
}

hipError_t launch_trace(const device_scene& ds, const float* rays, int n, int any, unsigned char* hit, int* inst,
                        int* ei, float* ew, float* dist, unsigned long long* counters, bool packet,
                        hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    dim3 grid((n + TRACE_BLOCK - 1) / TRACE_BLOCK);
    if (packet) {
        if (any)
            hipLaunchKernelGGL(trace_packet_kernel<true>, grid, dim3(TRACE_BLOCK), 0, stream, ds.view, rays, n, hit,
                               inst, ei, ew, dist, counters);
        else
            hipLaunchKernelGGL(trace_packet_kernel<false>, grid, dim3(TRACE_BLOCK), 0, stream, ds.view, rays, n, hit,
                               inst, ei, ew, dist, counters);
        return hipGetLastError();
    }
    if (any)
        hipLaunchKernelGGL(trace_kernel<true>, grid, dim3(TRACE_BLOCK), 0, stream, ds.view, rays, n, hit, inst, ei,
                           ew, dist, counters);
    else
        hipLaunchKernelGGL(trace_kernel<false>, grid, dim3(TRACE_BLOCK), 0, stream, ds.view, rays, n, hit, inst,
                           ei, ew, dist, counters);
    return hipGetLastError();
}

hipError_t launch_tonemap(const float* rgba, int n, unsigned char* out, const tonemap_table& table,
                          hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(tonemap_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, (const float4*)rgba, n,
                       (uchar4*)out, table);
    return hipGetLastError();
}

}  // namespace yrt
