// wavefront.hip -- the default render path: raytrace() (src/raytrace.cpp:213-254)
// as a wavefront pipeline of small gfx950 kernels over one lane per CAMERA SAMPLE.
//
// Per chunk of camera samples (a whole 1080p x 64 spp frame is one chunk; the
// per-sample state, ~70 B, lives in HBM -- 9 GB at c4 -- rather than in registers):
//   k_primary   eval_camera (:6-37) + closest hit (intersect_first, scene.cpp:483)
//               + eval_pos/eval_norm/eval_texcoord (scene.h:159-218) -> surface SoA
//   k_shadow    per light: the shadow ray of shade() (raytrace.cpp:129-133),
//               intersect_any (scene.cpp:489) -> occlusion byte
//   k_shade     the rest of shade() (:99-206): ambient, textures, Blinn-Phong or
//               lines lighting per unoccluded light, and for reflective hits the
//               mirror ray, compacted into the next level with one ballot + one
//               atomic per wave
//   (levels 1..max_depth-1: k_bounce (closest hit of the compacted rays), k_shadow,
//    k_shade; a sample whose value is final folds it up its chain of parents at once:
//    R_k = (D_k + R_{k+1}*kr_k) + la_k)
//   k_accumulate  the ordered per-pixel sum of raytrace.cpp:232-249
//
// Why: every traversal kernel carries only its ray and stack (few VGPRs, high
// occupancy), lanes of one wave are 64 samples of one pixel (s=8) or an 8x8 pixel
// tile (s=1), so their rays are nearly identical and stay converged through both
// BVH levels, and shadow rays of one light are traced together.
//
// Parity: each sample's arithmetic is shade()'s, in its order (trace_common.h);
// samples are summed per pixel in the reference's jj-major / ii-minor order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "packet_trace.h"
#include "trace_common.h"
#include "yrt_render.h"

namespace yrt {
namespace {

constexpr int WF_BLOCK = 256;
#ifndef YRT_PRIMARY_BLOCK
#define YRT_PRIMARY_BLOCK 64  // threads per k_primary block (<= packet_block; a multiple of 64). A/B at c4: 256 -> 64 is -3 %
#endif
#ifndef YRT_SHADOW_BLOCK
#define YRT_SHADOW_BLOCK 64
#endif
// threads per block of the packet shadow kernel: one wave. Walks of very different
// lengths share a CU; a block's slots are only refilled once all its waves are done, so
// the smallest block keeps the CU fullest (A/B at c4: 256 -> 64 is -5 % on k_shadow;
// 1024 is +22 %). k_primary stays at WF_BLOCK: its LDS (the parked world 1/d) and the
// per-block counter flush would cap the blocks per CU. The per-lane walks keep WF_BLOCK
// (their stacks are in LDS).
template <bool PACKET>
constexpr int shadow_block() { return PACKET ? YRT_SHADOW_BLOCK : WF_BLOCK; }
#ifndef YRT_TRACE_WAVES
#define YRT_TRACE_WAVES 8  // waves per SIMD the traversal kernels are register-budgeted for (A/B at c4 with the structured walks: 7 -> 8 is -3.5 %)
#endif
#ifndef YRT_SHADOW_WAVES
#define YRT_SHADOW_WAVES YRT_TRACE_WAVES  // the same for k_shadow
#endif
#ifndef YRT_SHADOW_BLOCK_CHUNK
// k_shadow_persist: queue positions per block chunk (A/B at c4 against per-wave grabs of 8:
// 8 / 16 / 32 / 64 / 128 / 256 / 512: -2.8 / -2.7 / -2.6 / -2.7 / -2.2 / -1.0 / 0 %)
#define YRT_SHADOW_BLOCK_CHUNK 16
#endif
constexpr int CHUNK_LOG2 = 29;  // samples per chunk, non-reflective scenes (~70 B of HBM each)
constexpr int TILE = 8;         // pixel tiles of TILE x TILE in the sample enumeration

// the render's list sums (k_list_stats, yrt_scene_tile_lists / yrt_scene_tile_list_masks):
// camera-list entries, camera lists, bundle-list entries, bundle lists, then the instances the
// camera lists' and the bundle lists' masks exclude
constexpr int list_sums = 6;

struct wf_buffers {
    f4* surf0;          // {p.xyz, info}: info = mat*4+kind, -1 miss, -2 not a sample
    f4* surf1;          // {n.xyz, u}
    float* surfv;       // v
    unsigned char* occl;  // [light][sample]
    f4* rad;            // level-0 radiance per sample
    // bounce levels (reflective scenes only)
    // mirror levels (reflective scenes): one slab per record kind, `capacity` records per
    // level, so any number of levels is plain indexing (the reference recursion has no cap)
    f4* ray_o_;  // level k >= 1 at (k - 1) * capacity: {o.xyz, parent index}
    f4* ray_d_;  // level k >= 1: {d.xyz, -}
    f4* rec0_;   // level k < nlevels - 1 at k * capacity: {D.xyz, material index}
    f4* rec1_;   // {la.xyz, -}; kr is the material's, re-read where the fold needs it
    __device__ __forceinline__ f4* ray_o(int k) const { return ray_o_ + (size_t)(k - 1) * capacity; }
    __device__ __forceinline__ f4* ray_d(int k) const { return ray_d_ + (size_t)(k - 1) * capacity; }
    __device__ __forceinline__ f4* rec0(int k) const { return rec0_ + (size_t)k * capacity; }
    __device__ __forceinline__ f4* rec1(int k) const { return rec1_ + (size_t)k * capacity; }
    int* count;             // level k >= 1, segment g: rays at count[(k * level_segments + g) * count_stride]
    int seg;                // slots per segment of a mirror level (seg_count)
    unsigned* queue;        // work counters of the persistent grids: shadow [0, 8) per XCD + [8] shared, primary [16, 24) + [24]
    const f4* trel;         // instance-level spine records relative to the camera origin
    int capacity;           // samples per chunk
    int nlevels;            // levels allocated
    int need_v;             // the scene has textures: the surface's v (surfv) is stored and read
    // shadow bundles (level 0 of the persistent any-hit grid, k_bundle_lists)
    int bundles;            // 1: this chunk's k_primary writes pbox and its shadow items walk lists
    f4* pbox;               // per 64-sample item: {lo.xyz, -1 if a hit point is not finite} {hi.xyz, -}
    int* lcount;            // per (bundle, light): candidate leaves, -1 = walk the tree
    int* lskip;             // per (bundle, light): instances of its listed leaves its hull excludes
    f4* lists;              // per (bundle, light): bundle_recs wide records (wide_record_bytes each)
    f4* slists;             // per (super-bundle, light): a leaf list (YRT_BUNDLE_SUPER)
    // camera lists (the closest hit of the camera rays, k_camera_lists)
    int cam_lists;          // 1: this chunk's camera rays walk their tile's list
    int* ccount;            // per 8x8-pixel tile of the chunk: listed leaves, -1 = walk the tree
    int* cskip;             // per tile: instances of its listed leaves its cone excludes
    f4* clist;              // per tile: camera_list_max entries of 2 f4 {lo - o, first} {hi - o, count}
    unsigned long long* lstats;  // the render's list sums (k_list_stats, list_sums of them)
};

// Mirror levels are compacted into level_segments segments of B.seg slots: segment g of
// level k + 1 holds the mirror rays spawned by k_shade's blocks b with b % 8 == g, at
// [g * seg, g * seg + count), each segment behind its own counter on its own 128-byte
// line. (One counter for the whole level serialised k_shade's block atomics: about 7 ns
// each on one address, ~1 ms of c3's level-0 shading.) Consumers walk the segments in
// turn, so their waves stay full except for each segment's last one.
#ifndef YRT_LEVEL_SEGMENTS
#define YRT_LEVEL_SEGMENTS 8
#endif
constexpr int level_segments = YRT_LEVEL_SEGMENTS;  // divides the 2048-block grid of the mirror levels
static_assert(2048 % level_segments == 0, "segment bound (run()) assumes level_segments | 2048");
constexpr int count_stride = 32;  // ints: one 128-byte line per counter
__device__ __forceinline__ int* seg_counter(int* count, int level, int g) {
    return count + (level * level_segments + g) * count_stride;
}

struct chunk_args {
    long long pix0;  // first pixel (in tile enumeration order) of this chunk
    int npix;        // pixels in this chunk
    int spp;
    int tiles_x;     // 8x8 tiles across the window
};

// pixel enumeration: 8x8 tiles across the local window, row-major tiles, row-major
// pixels inside a tile; samples of a pixel consecutive in jj-major / ii-minor order
__device__ __forceinline__ bool pixel_of(const dev_render_args& A, int tiles_x, long long p, int& lx, int& ly,
                                         int& i, int& j) {
    long long t = p / (TILE * TILE);
    int w = (int)(p % (TILE * TILE));
    lx = (int)(t % tiles_x) * TILE + (w % TILE);
    ly = (int)(t / tiles_x) * TILE + (w / TILE);
    if (lx >= A.tile_w || ly >= A.tile_h) return false;
    i = A.x0 + lx;
    int b = ly / A.band, r = ly % A.band;
    j = A.y0 + (b * A.band_stride + A.band_offset) * A.band + r;
    return i < A.width && j < A.height;
}

__device__ __forceinline__ void flush(unsigned long long* counters, int idx, unsigned long long v) {
    unsigned long long s = wave_sum(v);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(counter_line(counters) + idx, s);
}

// the timed kernels' counters: wave sums combined per block in LDS, then ONE device
// atomic per counter per block into the block's counter line (a per-wave atomic
// costs ~4x as many fabric atomics; the c4 shadow pass has 1.5 M blocks)
template <int N, int BS = WF_BLOCK>
__device__ __forceinline__ void flush_block(unsigned long long* counters, const int (&idx)[N],
                                            const unsigned long long (&v)[N]) {
    __shared__ unsigned long long part[BS / 64][N];
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < N; k++) {
        const unsigned long long s = wave_sum(v[k]);
        if ((threadIdx.x & 63) == 0) part[w][k] = s;
    }
    __syncthreads();
    if (threadIdx.x < N) {
        unsigned long long t = 0;
#pragma unroll
        for (int q = 0; q < BS / 64; q++) t += part[q][threadIdx.x];
        const unsigned b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        if (t) atomicAdd(counters + (size_t)(b % cnt_slots) * cnt_count + idx[threadIdx.x], t);
    }
}

__device__ __forceinline__ void flush_work(unsigned long long* counters, const work_counts& wc) {
    flush(counters, cnt_box_tests, wc.box);
    flush(counters, cnt_inst_entries, wc.inst);
    flush(counters, cnt_prim_tests, wc.prim);
    flush(counters, cnt_shaded_hits, wc.hits);
    flush(counters, cnt_tex_lookups, wc.tex);
    flush(counters, cnt_wave_node_visits, wc.wnode);
    flush(counters, cnt_wave_prim_visits, wc.wprim);
}

// A workspace pointer as a global-memory pointer. k_primary_persist reads its buffer
// arguments back from an LDS copy, and a pointer loaded from memory is generic to the
// compiler: its stores would be FLAT, which count against LGKM_CNT as well, so the walk's
// next s_waitcnt lgkmcnt(0) (every record fetch) would wait for them to reach memory.
typedef float gvec4 __attribute__((ext_vector_type(4)));
#ifndef YRT_NT_STREAMS
// the per-sample workspace streams (surface records, occlusion bytes) are written and read
// with the non-temporal hint, so that they pass through L2 without evicting the scene
// (A/B in one process, profiles/r4/ab_nt: c4 24.77 -> 24.62 ms, rank 0 of 8 / 4 and c3
// -0.6 to -0.8 %, identical images)
#define YRT_NT_STREAMS 1
#endif
// a constant made where it is used: v_mov of the immediate in volatile asm, which the compiler
// does not hoist out of a persistent kernel's item loop (a hoisted {0, 0, 0, -1} register
// tuple is held across the walk and spilled: the tuple is not rematerialised)
#ifndef YRT_R5_VCONST
#define YRT_R5_VCONST 1
#endif
template <int IMM>
__device__ __forceinline__ float vconst() {
    if (!YRT_R5_VCONST) return __int_as_float(IMM);
    float r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "n"(IMM));
    return r;
}
__device__ __forceinline__ void gstore(f4* p, int idx, float x, float y, float z, float w) {
    auto* q = (__attribute__((address_space(1))) gvec4*)p + idx;
    if (YRT_NT_STREAMS)
        __builtin_nontemporal_store(gvec4{x, y, z, w}, q);
    else
        *q = gvec4{x, y, z, w};
}
__device__ __forceinline__ void gstore(float* p, int idx, float x) {
    auto* q = (__attribute__((address_space(1))) float*)p + idx;
    if (YRT_NT_STREAMS)
        __builtin_nontemporal_store(x, q);
    else
        *q = x;
}
// a workspace stream's record / byte (see YRT_NT_STREAMS)
__device__ __forceinline__ float4 ld4s(const f4* p) {
    if (YRT_NT_STREAMS) {
        const gvec4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) gvec4*)p);
        return make_float4(v.x, v.y, v.z, v.w);
    }
    return ld4(p);
}
__device__ __forceinline__ float lds1(const float* p) {
    if (YRT_NT_STREAMS) return __builtin_nontemporal_load((const __attribute__((address_space(1))) float*)p);
    return *p;
}
__device__ __forceinline__ unsigned char ldb(const unsigned char* p) {
    if (YRT_NT_STREAMS) return __builtin_nontemporal_load((const __attribute__((address_space(1))) unsigned char*)p);
    return *p;
}
__device__ __forceinline__ void stb(unsigned char* p, unsigned char v) {
    if (YRT_NT_STREAMS)
        __builtin_nontemporal_store(v, (__attribute__((address_space(1))) unsigned char*)p);
    else
        *p = v;
}

#ifndef YRT_SKIP_UNUSED_V
#define YRT_SKIP_UNUSED_V 1  // a scene without textures neither writes nor reads the surface's v
#endif
#ifndef YRT_HIT16
// 1: the closest-hit kernels write a 16-byte hit record {slot, ei, w1, w2} per sample into
// surf0 instead of the 36-byte surface {p, mat*4+kind} {n, u} {v}; the shadow setup and
// k_shade evaluate the surface from it (eval_surface) where they need p, n, uv
#define YRT_HIT16 0
#endif
// the sample's record in surf0: HIT16 {slot (-1 miss, -2 not a sample), ei, w1, w2}, else
// {p, info (mat*4+kind, -1 miss, -2 not a sample)}; the slot/info field
__device__ __forceinline__ int sample_state(float4 s0) { return YRT_HIT16 ? ibits(s0.x) : ibits(s0.w); }
__device__ __forceinline__ void store_not_sample(const wf_buffers& B, int idx) {
    if (YRT_HIT16)
        gstore(B.surf0, idx, __int_as_float(-2), 0, 0, 0);
    else
        gstore(B.surf0, idx, vconst<0>(), vconst<0>(), vconst<0>(), vconst<-2>());
}
// a HIT16 record's surface (eval_pos/eval_norm/eval_texcoord, scene.h:159-218); ew.x is
// rebuilt as packet_first builds it (1 - w1 - w2, the same bits)
__device__ __forceinline__ surface hit16_surface(const dev_scene_view& S, float4 s0) {
    return eval_surface(S, ibits(s0.x), ibits(s0.y), vec4f{1 - s0.z - s0.w, s0.z, s0.w, 0});
}
__device__ __forceinline__ void store_hit16(const wf_buffers& B, int idx, bool hit, const hit_record& hr) {
    if (!hit)
        gstore(B.surf0, idx, __int_as_float(-1), 0, 0, 0);
    else
        gstore(B.surf0, idx, __int_as_float(hr.slot), __int_as_float(hr.ei), hr.ew.y, hr.ew.z);
}

// The surface record of a sample: the hit's surface is evaluated and stored on the hit lanes
// only, and a miss stores its marker. (Written as `surface sf = {}; if (hit) sf = ...;` the
// conditional aggregate copy kept the first 28 bytes of sf in a private array, which the
// backend promoted to 28 KB of LDS per 1024-thread block; its 64-bit address then took
// VGPRs the closest-hit walk spilled to scratch.)
// the surface record's info word: shadow class << 26 | material << 2 | kind (material < 2^24,
// so a hit's info is >= 0; -1 miss, -2 not a sample)
__device__ __forceinline__ int surf_info(const surface& sf) { return sf.mcls << 26 | sf.mat << 2 | sf.kind; }
__device__ __forceinline__ int info_mat(int info) { return (info >> 2) & (int)mat_index_mask; }

__device__ __forceinline__ vec3f store_hit_surface(const dev_scene_view& S, const wf_buffers& B, int idx, bool hit,
                                                   const hit_record& hr) {
    if (!hit) {
        gstore(B.surf0, idx, vconst<0>(), vconst<0>(), vconst<0>(), vconst<-1>());
        return {0, 0, 0};
    }
    const surface sf = eval_surface(S, hr.slot, hr.ei, hr.ew);
    gstore(B.surf0, idx, sf.p.x, sf.p.y, sf.p.z, __int_as_float(surf_info(sf)));
    gstore(B.surf1, idx, sf.n.x, sf.n.y, sf.n.z, sf.uv.x);
    // uv is read only by texture lookups: a scene without textures never needs it
    if (!YRT_SKIP_UNUSED_V || B.need_v) gstore(B.surfv, idx, sf.uv.y);
    return sf.p;
}

// the two traversal schedules behind one call: PACKET = wave-coherent walk
// (packet_trace.h, default), otherwise one independent walk per lane
// (trace_common.h). Both are called in wave-uniform control flow.
template <bool ANY, bool COUNT, bool PACKET, typename SE, int BS = packet_block>
struct tracer {
    SE* lane_stk;
    __device__ __forceinline__ bool trace(const dev_scene_view& S, const ray3& ray, bool valid, hit_record& hr,
                                          work_counts& wc) {
        if (PACKET) {
            if constexpr (ANY)
                return packet_any<COUNT>(S, ray, valid, wc);
            else
                return packet_first<COUNT, BS>(S, ray, valid, hr, wc);
        }
        if (!valid) return false;
        if (ANY) return occluded<COUNT, WF_BLOCK>(S, ray, lane_stk, wc);
        return traverse<false, COUNT, WF_BLOCK>(S, ray, hr, lane_stk, wc);
    }
};

// LDS for either schedule: per-lane stack columns; the packet walk keeps its stack
// in VGPR lanes and needs none
template <bool PACKET, typename SE>
struct traversal_lds;
template <typename SE>
struct traversal_lds<false, SE> {
    SE lane[traversal_stack_cap * WF_BLOCK];
};
template <typename SE>
struct traversal_lds<true, SE> {
    int unused;
};

template <bool ANY, bool COUNT, bool PACKET, typename SE>
__device__ __forceinline__ tracer<ANY, COUNT, PACKET, SE> make_tracer(traversal_lds<PACKET, SE>& L) {
    tracer<ANY, COUNT, PACKET, SE> t;
    if constexpr (PACKET)
        t.lane_stk = nullptr;
    else
        t.lane_stk = L.lane + threadIdx.x;
    return t;
}

// Workgroups are dealt round-robin to the 8 XCDs (linear block b runs on XCD b % 8).
// xcd_runs keeps the round-robin sweep over the image but hands each XCD runs of C
// consecutive blocks: the grid is cut into super-chunks of 8 runs, XCD x takes run x of
// each (a bijection; a ragged last super-chunk keeps its blocks). Each XCD then traces
// neighbouring pixels (its L2 and its CUs' scalar caches see one region) while all eight
// still sweep the image together. (Contiguous block ranges per XCD lose: +10 % primary,
// +7.5 % shadow -- image regions differ in cost and the slowest XCD sets the launch time.)
template <unsigned C>
__device__ __forceinline__ unsigned xcd_runs(unsigned b, unsigned n) {
    constexpr unsigned G = 8u * C;
    if (b >= n / G * G) return b;
    const unsigned w = b % G;
    return b - w + (w % 8u) * C + w / 8u;
}

#ifndef YRT_SHADOW_LIGHT_MINOR
#define YRT_SHADOW_LIGHT_MINOR 24  // k_shadow: XCD run length with the light index minor (A/B: shadow -1.1 %)
#endif
#ifndef YRT_XCD_CHUNK_PRIMARY
#define YRT_XCD_CHUNK_PRIMARY 256  // k_primary: XCD runs of this many blocks (A/B: -1.5 %)
#endif

// ke / rr (vec3f / float: three divisions) with fast_div.h's div_nr when every active
// lane's operands are in its range
__device__ __forceinline__ vec3f div3(vec3f ke, float rr) {
    if (YRT_FAST_NORMALIZE &&
        !__ballot(!(div_nr_ok(ke.x, rr) && div_nr_ok(ke.y, rr) && div_nr_ok(ke.z, rr)))) {
        const float y = rcp_nr(rr);
        return {div_nr(ke.x, rr, y), div_nr(ke.y, rr, y), div_nr(ke.z, rr, y)};
    }
    return ke / rr;
}

#ifndef YRT_SHADOW_CULL
#define YRT_SHADOW_CULL 1
#endif
// ---- shadow rays whose light term is exactly zero are not traced ----
// shade() (raytrace.cpp:133-183) adds a light's term c += ld + ls only when intersect_any
// finds no occluder; skipping it and adding it are the same when the term is +-0 in every
// component (c starts at +0 and a sum never turns into -0 under round-to-nearest, so c + +-0
// is c bit for bit). From the hit's material class (yrt_device.h mat_class_shift, set at
// upload) and the geometry alone, the term is +-0 when max(0, n.l) is +-0 and ker = ke / r^2
// is below 2^100 in every component -- then ld = (kd0 * tkd) * ker * max(0, n.l) is a finite
// product (|kd0| <= 2^20, the texture factor in [0, 1]) times +-0 -- and ls is +-0:
//   class 1 (Ks == 0, ns in [0, FLT_MAX]): ks * ker is +-0, and with x = max(0, n.h) in
//     [0, 1] spec_pow takes its shortcut (factor 1), so ls = +-0;
//   class c >= 2 (ns >= mat_class_ns(c) > 0, |Ks| <= 2^20): powf_cr(x, ns) is exactly 0 when
//     x == 0, or when x in [2^-126, 1) and ns * log2(x) < -151 by v_log_f32 -- which
//     mat_class_ns(c) * log2(x) < -151 implies (log2(x) < 0, and rounding is monotone) --, so
//     ls = finite * 0; where spec_pow takes its shortcut instead, ls = +-0 * 1.
// n, l, r, v, h and ker are computed with the functions k_shade uses (normalize_len, div3),
// so the test sees k_shade's values.
// Lines (their sin-based lighting) are always traced. A culled ray is recorded as occluded:
// k_shade skips the light, which leaves c as adding +-0 would. The ray counters keep the
// reference's counts (a culled ray is counted); the instrumented COUNT pass traces every ray.
// n is the surface record's second row, loaded beside the first: no dependent load.
// Called in uniform control flow; a wave in which no lane can pass the cheap first tests
// (class, kind, max(0, n.l) == 0) skips the rest.
__device__ __forceinline__ bool light_term_zero(int info, vec3f nrm, vec3f p, vec3f ro, vec3f l, float r, vec3f ke) {
    const int cls = (info >> 26) & 15;
    const float sd = smax(0.0f, dot(nrm, l));
    const bool first = info >= 0 && cls != 0 && (info & 3) != kind_lines && sd == 0.0f;
    if (!ballot(first)) return false;
    vec3f v, h, ker;
    float vlen, hlen;
    normalize_len(ro - p, v, vlen);
    normalize_len(v + l, h, hlen);
    ker = div3(ke, r * r);
    const float x = smax(0.0f, dot(nrm, h));
    const bool ker_ok = fabsf(ker.x) < 0x1p100f && fabsf(ker.y) < 0x1p100f && fabsf(ker.z) < 0x1p100f;
    const bool ls_zero =
        cls == 1 ? x >= 0.0f && x <= 1.0f
                 : x == 0.0f || (x >= 0x1p-126f && x < 1.0f &&
                                 (float)(16 << ((cls - 2) & 15)) * __builtin_amdgcn_logf(x) < -151.0f);
    return first && ker_ok && ls_zero;
}

// camera_ray (trace_common.h, raytrace.cpp:6-37 with the uv of :235-238) with its four
// divisions and normalize through fast_div.h where every active lane is in range (the
// same bits); called per lane in divergent code (the checks ballot the active lanes)
__device__ __forceinline__ ray3 camera_ray_w(const dev_camera& cam, int W, int H, int ns, int i, int j, int ii,
                                             int jj) {
    const float fns = (float)ns, fw = (float)W, fh = (float)H;
    const float a = ii + 0.5f, b = jj + 0.5f;
    float u, v;
    if (YRT_FAST_NORMALIZE && !__ballot(!(div_nr_ok(a, fns) && div_nr_ok(b, fns)))) {
        const float y = rcp_nr(fns);
        u = i + div_nr(a, fns, y), v = j + div_nr(b, fns, y);
    } else {
        u = i + a / fns, v = j + b / fns;
    }
    if (YRT_FAST_NORMALIZE && !__ballot(!(div_nr_ok(u, fw) && div_nr_ok(v, fh)))) {
        u = div_nr(u, fw, rcp_nr(fw)), v = div_nr(v, fh, rcp_nr(fh));
    } else {
        u = u / fw, v = v / fh;
    }
    vec3f q;
    q.x = cam.ox + (u - 0.5f) * cam.w * cam.xx + (v - 0.5f) * cam.h * cam.yx - cam.focus * cam.zx;
    q.y = cam.oy + (u - 0.5f) * cam.w * cam.xy + (v - 0.5f) * cam.h * cam.yy - cam.focus * cam.zy;
    q.z = cam.oz + (u - 0.5f) * cam.w * cam.xz + (v - 0.5f) * cam.h * cam.yz - cam.focus * cam.zz;
    const vec3f o = {cam.ox, cam.oy, cam.oz};
    vec3f d;
    float len;
    normalize_len(q - o, d, len);
    return {o, d, ray_eps, flt_max};
}

// ---- shadow bundles ----
// The shadow rays of one light from the samples of a bundle (bundle_g consecutive 64-sample
// items: an 8x8-pixel tile at 8x8 spp) all run from points inside the box P of the bundle's
// hit points towards one point, the light's position Lp (raytrace.cpp:129-133; the light
// frame's rotation is the identity, so its ray is p -> transform_point(frame, pos0 - p) =
// pos0 - p + o). Every such segment lies in the convex hull of P and Lp. k_bundle_lists
// collects, per (bundle, light), the instance-level leaves of the any-hit tree whose box no
// bounding plane of that hull separates by more than a margin far above the slab test's
// rounding (its t values carry a few ulps of |t| <= |P - Lp|, the 1.00000024 fudge another
// 2.4e-7): a leaf outside that list fails the exact box test of every ray of the bundle.
// The walk then starts from the list (at most bundle_max leaves as a chain of wide records)
// instead of the tree's root. It tests each listed leaf's own box,
// exactly as the tree walk does, and reaches every leaf the tree walk reaches -- the
// any-hit answer does not depend on which inner boxes were tested.
// A bundle whose light is rotated, whose hit points are not finite or whose list would be
// longer walks the tree.
#ifndef YRT_SHADOW_BUNDLES
#define YRT_SHADOW_BUNDLES 1
#endif
#ifndef YRT_BUNDLE_ITEMS
#define YRT_BUNDLE_ITEMS 64  // 64-sample items per bundle (at most 64: one per lane of the list builder)
#endif
constexpr int bundle_g = YRT_BUNDLE_ITEMS;
static_assert(bundle_g >= 1 && bundle_g <= 64, "one item per lane of k_bundle_lists");
#ifndef YRT_BUNDLE_MIN_TOP
#define YRT_BUNDLE_MIN_TOP 8  // bundles only when the instance level's wide tree has this many records
#endif
#ifndef YRT_BUNDLE_SORT
// a bundle's leaves in the order its rays meet them: 1 from the hit points towards the light,
// 2 from the light towards the hit points, 0 in tree order. A/B in one process
// (profiles/r4/ab_bundle_sort): c4 shadow 11.82 -> 11.72 / 11.62 ms (1 / 2), instance1k
// 7.42 -> 7.30 / 7.39, instance100k (lists off) unchanged; putting the leaf that holds the
// hit points' centre (their own instance) last: 11.71 / 7.39
#define YRT_BUNDLE_SORT 2
#endif
#ifndef YRT_LISTS_MIN_SPP
// the lists' cost is per 8x8-pixel tile (~0.2 ms at 1080p), their gain per sample: in one
// process (profiles/r5/ab/r5t_*) instance10000 at 1080p with lists on / off -- 1 spp 1.79 /
// 1.54 ms, 4 spp 3.00 / 3.06, 16 spp 6.84 / 7.93, 64 spp 19.41 / 24.18; instance100k at 4 spp
// 4.21 / 3.99, instance1k 1.50 / 1.65. YRT_LISTS_AUTO builds them from this many samples per
// pixel (a 3x3 grid)
#define YRT_LISTS_MIN_SPP 9
#endif
#ifndef YRT_INSTANCE_MASKS
// the list builders mark the instances of a listed leaf that their cone / hull excludes, and
// the walks skip them (k_camera_lists, k_bundle_lists; dev_scene_view ibox)
#define YRT_INSTANCE_MASKS 1
#endif
constexpr int bundle_max = 16;        // candidate leaves per list
constexpr int bundle_recs = 5;        // wide records per list: a chain (3 + 3 + 3 + 3 + 4 leaves)
constexpr int bundle_max_lights = 8;  // more lights: no bundles (the lists' memory grows with them)
#ifndef YRT_CAMERA_LISTS
#define YRT_CAMERA_LISTS 1  // camera rays walk per-tile leaf lists (k_camera_lists, packet_first's list mode)
#endif
#ifndef YRT_CAMERA_LIST_MAX
#define YRT_CAMERA_LIST_MAX 32  // leaves per tile list (more: the tile's rays walk the tree)
#endif
constexpr int camera_list_max = YRT_CAMERA_LIST_MAX;

// wave-wide min / max with DPP row rotations and row broadcasts (VALU only, no LDS round
// trips): every row of 16 lanes folds itself, rows 1 and 3 take rows 0 and 2 (row_bcast:15),
// rows 2 and 3 take row 1 (row_bcast:31); lane 63 then holds the result. The floats (no NaN
// here) are folded as integers whose signed order is theirs (b ^ (b >> 31 & 0x7fffffff)), so
// that each step is one v_min_i32 / v_max_i32 with the DPP source and no canonicalisation.
// (the lanes of rows outside ROWS are left undefined: only row 3's lanes, which every step
// writes, reach the result)
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ int fkey(int b) { return b ^ ((b >> 31) & 0x7fffffff); }  // (its own inverse)
template <bool MAX>
__device__ __forceinline__ float wave_fold(float f) {
    auto op = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
    int v = fkey(__float_as_int(f));
    v = op(v, dpp_i<0x121, 0xf>(v));  // row_ror:1
    v = op(v, dpp_i<0x122, 0xf>(v));  // row_ror:2
    v = op(v, dpp_i<0x124, 0xf>(v));  // row_ror:4
    v = op(v, dpp_i<0x128, 0xf>(v));  // row_ror:8
    v = op(v, dpp_i<0x142, 0xa>(v));  // row_bcast:15 into rows 1, 3
    v = op(v, dpp_i<0x143, 0xc>(v));  // row_bcast:31 into rows 2, 3
    return __int_as_float(fkey(__builtin_amdgcn_readlane(v, 63)));
}
__device__ __forceinline__ float wave_fmin(float v) { return wave_fold<false>(v); }
__device__ __forceinline__ float wave_fmax(float v) { return wave_fold<true>(v); }
// a box's six folds in lock step (their DPP steps interleave: no wait states between them)
__device__ __forceinline__ void wave_box(float (&lo)[3], float (&hi)[3]) {
    int v[6];
    for (int a = 0; a < 3; a++) v[a] = fkey(__float_as_int(lo[a])), v[3 + a] = fkey(__float_as_int(hi[a]));
#define YRT_BOX_STEP(CTRL, ROWS)                                                  \
    {                                                                             \
        int t[6];                                                                 \
        for (int a = 0; a < 6; a++) t[a] = dpp_i<CTRL, ROWS>(v[a]);               \
        for (int a = 0; a < 6; a++) v[a] = a < 3 ? min(v[a], t[a]) : max(v[a], t[a]); \
    }
    YRT_BOX_STEP(0x121, 0xf)
    YRT_BOX_STEP(0x122, 0xf)
    YRT_BOX_STEP(0x124, 0xf)
    YRT_BOX_STEP(0x128, 0xf)
    YRT_BOX_STEP(0x142, 0xa)
    YRT_BOX_STEP(0x143, 0xc)
#undef YRT_BOX_STEP
    for (int a = 0; a < 3; a++) {
        lo[a] = __int_as_float(fkey(__builtin_amdgcn_readlane(v[a], 63)));
        hi[a] = __int_as_float(fkey(__builtin_amdgcn_readlane(v[3 + a], 63)));
    }
}

// the box of this wave's hit points (the item idx / 64), for k_bundle_lists; called by
// every lane of the wave
__device__ __forceinline__ void store_item_box(const wf_buffers& B, int idx, bool has_p, vec3f p) {
    const bool fin = has_p && __builtin_isfinite(p.x) && __builtin_isfinite(p.y) && __builtin_isfinite(p.z);
    const bool bad = has_p && !fin;
    float lo[3] = {fin ? p.x : INFINITY, fin ? p.y : INFINITY, fin ? p.z : INFINITY};
    float hi[3] = {fin ? p.x : -INFINITY, fin ? p.y : -INFINITY, fin ? p.z : -INFINITY};
    wave_box(lo, hi);
    const bool any_bad = ballot(bad) != 0;
    if ((threadIdx.x & 63) == 0) {
        const int item = idx >> 6;
        gstore(B.pbox, 2 * item, lo[0], lo[1], lo[2], any_bad ? -1.0f : 0.0f);
        gstore(B.pbox, 2 * item + 1, hi[0], hi[1], hi[2], 0.0f);
    }
}

#ifndef YRT_R5_SURF
#define YRT_R5_SURF 1
#endif
#ifndef YRT_PRIMARY_REL
#define YRT_PRIMARY_REL 1  // camera rays walk the instance level on camera-relative records
#endif

// ---- level 0: camera rays + closest hit + surface ----
// the camera samples idx of one wave: eval_camera, closest hit, surface record
template <bool COUNT, bool PACKET, typename SE, int BS = packet_block, int LDSN = 0, bool LIST = false>
__device__ __forceinline__ bool primary_samples(const dev_scene_view& S, const dev_render_args& A, const chunk_args& C,
                                                const wf_buffers& B, tracer<false, COUNT, PACKET, SE, BS>& T, int idx,
                                                work_counts& wc, const float4* lds = nullptr) {
    const int nsamp = C.npix * C.spp;
    bool valid = false;
    ray3 ray = {{0, 0, 0}, {0, 0, 1}, ray_eps, flt_max};
    if (idx < nsamp) {
        const long long p = C.pix0 + idx / C.spp;
        const int q = idx % C.spp;
        int lx, ly, i, j;
        valid = pixel_of(A, C.tiles_x, p, lx, ly, i, j);
        if (valid) {
            const int ns = A.samples;
            ray = camera_ray_w(A.cam, A.width, A.height, ns, i, j, q % ns, q / ns);
        } else {
            store_not_sample(B, idx);
        }
    }
    hit_record hr = {-1, -1, {0, 0, 0, 0}, 0};
    // every camera ray starts at the camera origin (camera_ray): the packet walk tests the
    // instance level on the records relative to it -- or, with camera lists, walks the list
    // of the 8x8-pixel tile this wave's samples lie in (a wave straddling two tiles walks
    // the tree)
    bool hit;
    if constexpr (PACKET && YRT_PRIMARY_REL) {
        const f4* lbase = nullptr;
        int ln = -1;
        if (LIST && !COUNT) {
            const int nsamp = C.npix * C.spp;
            const int i0 = uniform(idx) & ~63, i1 = min(i0 + 63, nsamp - 1);
            const int t0 = i0 / C.spp / (TILE * TILE), t1 = i1 / C.spp / (TILE * TILE);
            // (a zero direction -- a camera with no extent -- walks the tree)
            const bool zero_dir = valid && ray.d.x == 0.0f && ray.d.y == 0.0f && ray.d.z == 0.0f;
            if (t0 == t1 && i0 < nsamp && !ballot(zero_dir)) {
                ln = uniform(B.ccount[t0]);
                lbase = B.clist + (size_t)t0 * camera_list_max * 2;
            }
        }
        hit = packet_first<COUNT, BS, true, LDSN, LIST>(S, ray, valid, hr, wc, B.trel, lds, lbase, ln);
    } else {
        hit = T.trace(S, ray, valid, hr, wc);
    }
    vec3f hp = {0, 0, 0};
    if (valid) {
        if (COUNT && hit) wc.hits++;
        if (YRT_HIT16) {
            store_hit16(B, idx, hit, hr);
            if (YRT_SHADOW_BUNDLES && hit && B.bundles) hp = eval_surface(S, hr.slot, hr.ei, hr.ew).p;
        } else if (YRT_R5_SURF) {
            hp = store_hit_surface(S, B, idx, hit, hr);
        } else {
            surface sf = {};
            if (hit) sf = eval_surface(S, hr.slot, hr.ei, hr.ew);
            if (!hit)
                gstore(B.surf0, idx, 0, 0, 0, __int_as_float(-1));
            else {
                gstore(B.surf0, idx, sf.p.x, sf.p.y, sf.p.z, __int_as_float(surf_info(sf)));
                gstore(B.surf1, idx, sf.n.x, sf.n.y, sf.n.z, sf.uv.x);
                if (!YRT_SKIP_UNUSED_V || B.need_v) gstore(B.surfv, idx, sf.uv.y);
            }
            hp = sf.p;
        }
    }
    if (YRT_SHADOW_BUNDLES && !COUNT && B.bundles) store_item_box(B, idx, valid && hit, hp);
    return valid;
}

// The instance-level spine records with the camera origin subtracted from every bound, in
// fp32 as the reference's slab test does it ((bbox.min - ray.o), scene.cpp:373-374), are what
// the primary rays' REL walk reads (packet_first); k_chunk_setup writes them once per render.

// ---- per-chunk setup: one launch instead of a kernel and three to five fills ----
// the camera-relative spine records (the first chunk of a packet render: tpair != nullptr),
// and zeros for the persistent grids' work counters (queue), the list sums (lstats, the first
// chunk that builds lists), the mirror levels' ray counts (count_ints) and the render's counter
// lines (counters, the first chunk). Each fill was its own hipMemsetAsync launch of ~4 us of
// GPU time; at a rank's share of an 8-way split a frame is ~2.6 ms.
__global__ __launch_bounds__(WF_BLOCK) void k_chunk_setup(const f4* __restrict__ tpair, int nrec, float ox, float oy,
                                                          float oz, f4* __restrict__ trel, unsigned* queue,
                                                          unsigned long long* lstats, int* count, int count_ints,
                                                          unsigned long long* counters, int counter_words) {
    const int i = blockIdx.x * WF_BLOCK + threadIdx.x;
    const int stride = gridDim.x * WF_BLOCK;
    if (tpair)
        for (int k = i; k < nrec; k += stride) {
            const float4 r = ld4(tpair + k);
            trel[k] = {r.x - ox, r.y - oy, r.z - oz, r.w};
        }
    if (i < 32) queue[i] = 0u;
    if (lstats && i < list_sums) lstats[i] = 0ull;
    for (int k = i; k < count_ints; k += stride) count[k] = 0;
    if (counters)
        for (int k = i; k < counter_words; k += stride) counters[k] = 0ull;
}

// ---- work distribution of the persistent any-hit grid: block chunks ----
// The waves of an XCD share one agent-scope counter over its item sequence, which keeps
// the chip's working window as tight as the hardware's block dealing does (a fixed
// interleave, wave j taking j, j + W, ..., lets the waves drift apart: +21 %). A block
// takes CS consecutive positions per atomic and its waves take them one at a time from
// an LDS counter, so the waves of a CU trace neighbouring items together (per-wave grabs
// of 8 consecutive positions: +2.7 % on the any-hit grid). Chunk g's base sits in ring
// entry g % R behind a tag; the wave taking chunk g's middle slot fetches chunk g + 1,
// once every slot of the entry's previous chunk has been read (each taker reads its base
// right after taking its slot, before it looks at the item, and slots are taken in
// order, so every wait ends). All atomics are vector (lane 0) or LDS operations.
#ifndef YRT_SHARED_TAIL
// the persistent grids' last 1/YRT_SHARED_TAIL items come from one queue that every XCD
// takes from once its own share is done (the XCDs' shares otherwise end up to 2 % of a
// c4 launch apart, 6 % at a rank's share of an 8-way split: tools/tail_stats.py); 0: each
// XCD keeps its static share to the end. A/B in one process (profiles/r4/ab_shared_tail):
// 1/32 / 1/16 / 1/8 -- c4 24.67 -> 24.43 / 24.43 / 24.42 ms, rank 0 of 4 6.42 -> 6.34 /
// 6.37 / 6.35, instance100k 32.92 -> 32.70 / 32.87 / 33.14 (its short any-hit grid pays
// for a larger shared tail), rank 0 of 8 and c3 within 0.3 %
#define YRT_SHARED_TAIL 32
#endif
constexpr unsigned tail_flag = 0x80000000u;  // a position in the shared tail
constexpr unsigned gcd_u(unsigned a, unsigned b) { return b ? gcd_u(b, a % b) : a; }
// items of the per-XCD head: whole super-runs of 8 x lcm(RUN, CS) (so that every XCD's
// share is whole runs and whole block chunks); the rest is the shared tail
template <unsigned RUN, unsigned CS>
__device__ __forceinline__ unsigned head_items(unsigned n_items) {
    constexpr unsigned G = 8u * (RUN / gcd_u(RUN, CS) * CS);
    return YRT_SHARED_TAIL ? (n_items - n_items / YRT_SHARED_TAIL) / G * G : 0u;
}
// a block chunk's first position: from the XCD's own counter while its share lasts
// (limit = positions per XCD), then from the shared one (flagged)
template <unsigned CS>
__device__ __forceinline__ unsigned chunk_fetch(unsigned* counter, unsigned* gcounter, unsigned limit) {
    const unsigned k = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!YRT_SHARED_TAIL || k * CS + CS <= limit) return k * CS;
    return tail_flag | __hip_atomic_fetch_add(gcounter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * CS;
}

struct chunk_ring {
    static constexpr unsigned R = 4;
    unsigned base[R], tag[R], reads[R], taken;
};

template <unsigned CS>
__device__ __forceinline__ void chunk_ring_init(chunk_ring& ring, unsigned* counter, unsigned* gcounter = nullptr,
                                                unsigned limit = ~0u) {
    static_assert(CS >= 2, "a chunk's middle slot fetches the next chunk");
    if (threadIdx.x < chunk_ring::R) {
        ring.tag[threadIdx.x] = threadIdx.x == 0 ? 0u : ~0u;
        ring.reads[threadIdx.x] = threadIdx.x == 0 ? 0u : CS;
    }
    if (threadIdx.x == 0) {
        ring.base[0] = chunk_fetch<CS>(counter, gcounter, limit);
        ring.taken = 0;
    }
    __syncthreads();
}

// the calling wave's next position in its XCD's item sequence (wave-uniform)
template <unsigned CS>
__device__ __forceinline__ unsigned chunk_ring_next(chunk_ring& ring, unsigned* counter, unsigned lane,
                                                    unsigned* gcounter = nullptr, unsigned limit = ~0u) {
    constexpr unsigned R = chunk_ring::R;
    unsigned t = 0;
    if (lane == 0) t = __hip_atomic_fetch_add(&ring.taken, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
    const unsigned g = t / CS, o = t % CS;
    if (o == CS / 2) {  // publish chunk g + 1
        const unsigned e1 = (g + 1) % R;
        unsigned nbase = 0;
        if (lane == 0) nbase = chunk_fetch<CS>(counter, gcounter, limit);
        nbase = (unsigned)__builtin_amdgcn_readfirstlane((int)nbase);
        while (__hip_atomic_load(&ring.reads[e1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != CS)
            __builtin_amdgcn_s_sleep(1);
        if (lane == 0) {
            ring.base[e1] = nbase;
            __hip_atomic_store(&ring.reads[e1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(&ring.tag[e1], g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    const unsigned e = g % R;
    while (__hip_atomic_load(&ring.tag[e], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != g)
        __builtin_amdgcn_s_sleep(1);
    const unsigned q = (unsigned)__builtin_amdgcn_readfirstlane((int)ring.base[e]) + o;
    if (lane == 0) __hip_atomic_fetch_add(&ring.reads[e], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return q;
}

// position q of XCD xcd's sequence -> item: runs of RUN consecutive items per XCD (XCD x
// takes runs x, x + 8, ...), then the items past the last whole super-run round-robin
template <unsigned RUN>
__device__ __forceinline__ unsigned xcd_item(unsigned q, unsigned xcd, unsigned n_items) {
    const unsigned full = n_items / (8u * RUN) * (8u * RUN);
    const unsigned per_xcd = full / 8u;
    return q < per_xcd ? ((q / RUN) * 8u + xcd) * RUN + q % RUN : full + (q - per_xcd) * 8u + xcd;
}
// the same with a shared tail (YRT_SHARED_TAIL): an XCD's own positions cover whole runs of
// the head, a flagged position is the tail's (head + its index; >= n_items: done)
template <unsigned RUN>
__device__ __forceinline__ unsigned split_item(unsigned q, unsigned xcd, unsigned n_items, unsigned head) {
    if (!YRT_SHARED_TAIL) return xcd_item<RUN>(q, xcd, n_items);
    if (q & tail_flag) return head + (q & ~tail_flag);
    return ((q / RUN) * 8u + xcd) * RUN + q % RUN;
}

#ifdef YRT_TAIL_STATS
// diagnostic build only (tools/tail_stats.py): per wave of the persistent grids, its start
// and end on the 100 MHz constant clock, the items it took and its XCD (vector stores)
static __device__ unsigned long long g_tail[2][8192][4];
__device__ __forceinline__ void tail_record(int k, unsigned long long t0, unsigned items) {
    const unsigned gw = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
    if ((threadIdx.x & 63) == 0 && gw < 8192u) {
        unsigned long long* e = g_tail[k][gw];
        e[0] = t0, e[1] = __builtin_amdgcn_s_memrealtime(), e[2] = items, e[3] = blockIdx.x % 8u;
    }
}
#endif

// (LIST: the camera rays walk their tiles' lists, k_camera_lists)
template <bool COUNT, bool PACKET, typename SE, bool LIST = false>
__global__ __launch_bounds__(YRT_PRIMARY_BLOCK, YRT_TRACE_WAVES) void k_primary(dev_scene_view S, dev_render_args A,
                                                               chunk_args C, wf_buffers B,
                                                               unsigned long long* counters) {
    constexpr int BS = YRT_PRIMARY_BLOCK;
    __shared__ traversal_lds<PACKET, SE> lds;
    auto T = make_tracer<false, COUNT, PACKET, SE>(lds);
    const int idx = (int)xcd_runs<YRT_XCD_CHUNK_PRIMARY>(blockIdx.x, gridDim.x) * BS + threadIdx.x;
    work_counts wc;
    const bool valid = primary_samples<COUNT, PACKET, SE, packet_block, 0, LIST>(S, A, C, B, T, idx, wc);
    flush_block<2, BS>(counters, {cnt_rays, cnt_samples}, {valid ? 1ull : 0ull, valid ? 1ull : 0ull});
    if (COUNT) flush_work(counters, wc);
}

// ---- level 0, persistent: k_primary's work on a grid that fills the chip once (two
// SP_BLOCK-thread blocks per CU), each wave taking 64-sample items through its block's
// chunk ring (counters B.queue[8..15]). The render, chunk and buffer arguments are read
// from LDS copies for each item (a compiler barrier per item), so they are not held in
// registers across the walk.
constexpr int SP_BLOCK = 1024;  // threads per persistent block (two blocks per CU at 8 waves/SIMD)
#ifndef YRT_PRIMARY_WAVES
#define YRT_PRIMARY_WAVES YRT_TRACE_WAVES  // k_primary_persist: waves per SIMD (register budget and grid)
#endif
#ifndef YRT_PRIMARY_SP_BLOCK
// k_primary_persist: threads per block, whole blocks filling YRT_PRIMARY_WAVES per SIMD
#define YRT_PRIMARY_SP_BLOCK \
    (YRT_PRIMARY_WAVES == 7 ? 448 : YRT_PRIMARY_WAVES == 6 ? 768 : YRT_PRIMARY_WAVES == 5 ? 640 : SP_BLOCK)
#endif
static_assert((YRT_PRIMARY_WAVES * 4 * 64) % YRT_PRIMARY_SP_BLOCK == 0, "whole blocks per CU");
#ifndef YRT_PRIMARY_LDS_RECORDS
// k_primary_persist with LDS staging on (yrt_scene_set_lds_staging): the first records of the
// camera-relative instance level (breadth first, device_scene.cpp) staged in LDS per block and
// read by the walk instead of through the scalar cache (A/B, DESIGN.md §5: 1 023 / 511 / 255
// records +4.1 / +3.7 / +4.3 %; the handle's default is off)
#define YRT_PRIMARY_LDS_RECORDS 511
#endif
#ifndef YRT_PRIMARY_PERSIST_MIN_ITEMS
// A/B against k_primary (items = 64-sample blocks; profiles/r3/ab_primary_persist): 2.07 M
// (c4) primary 11.55 -> 11.37 ms; instance100k 27.16 -> 27.01. Round 4
// (profiles/r4/ab_persist): the band shares of an N-rank split, which the old 1 M threshold
// sent to k_primary, lose most: c4 rank 0 of 8 / 4 primary 2.89 -> 1.52 / 4.60 -> 2.89 ms,
// instance100k rank 0 of 8 13.91 -> 3.74; c3 1.14 -> 1.10, 640x360 c4 1.49 -> 0.98; c1/c2
// equal. The timed path is persistent at every size. (Holding the arguments in registers
// instead: 62 SGPR and 12 VGPR spills, c4 unchanged.)
#define YRT_PRIMARY_PERSIST_MIN_ITEMS 0
#endif
#ifndef YRT_R5_IDXLANE
#define YRT_R5_IDXLANE 1
#endif
#ifndef YRT_PRIMARY_BLOCK_CHUNK
#define YRT_PRIMARY_BLOCK_CHUNK 16  // (64: the same)
#endif
template <typename SE, int LDSN, bool LIST = false>
__global__ __launch_bounds__(YRT_PRIMARY_SP_BLOCK, YRT_PRIMARY_WAVES) void k_primary_persist(dev_scene_view S,
                                                                                dev_render_args A, chunk_args C,
                                                                                wf_buffers B,
                                                                                unsigned long long* counters) {
    constexpr unsigned CS = YRT_PRIMARY_BLOCK_CHUNK;
    constexpr int SPB = YRT_PRIMARY_SP_BLOCK;
    __shared__ chunk_ring ring;
    __shared__ dev_render_args A_lds;
    __shared__ chunk_args C_lds;
    __shared__ wf_buffers B_lds;
    __shared__ float4 lds_rec[LDSN > 0 ? LDSN * spine_record_f4 : 1];
    if constexpr (LDSN > 0) {
        // (the instance level may have fewer records: the walk never addresses past them)
        const int n = min(LDSN, S.ntnodes) * spine_record_f4;
        const float4* src = reinterpret_cast<const float4*>(B.trel);
        for (int i = (int)threadIdx.x; i < n; i += SPB) lds_rec[i] = src[i];
    }
    if (threadIdx.x == 0) A_lds = A, C_lds = C, B_lds = B;
    const unsigned lane = threadIdx.x & 63;
    const unsigned xcd = blockIdx.x % 8u;
    unsigned* counter = B.queue + 16 + xcd;
    unsigned* gcounter = B.queue + 24;
    const unsigned n_items = (unsigned)((C.npix * C.spp + 63) / 64);
    const unsigned head = head_items<YRT_XCD_CHUNK_PRIMARY, CS>(n_items);
    chunk_ring_init<CS>(ring, counter, gcounter, head / 8u);  // (its barrier also publishes the copies)
    tracer<false, false, true, SE, SPB> T;
    T.lane_stk = nullptr;
    work_counts wc;
    unsigned valid_n = 0;  // wave-uniform: camera samples of this wave
#ifdef YRT_TAIL_STATS
    const unsigned long long tail_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned tail_items = 0;
#endif
    for (;;) {
        const unsigned q = chunk_ring_next<CS>(ring, counter, lane, gcounter, head / 8u);
        const unsigned it = split_item<YRT_XCD_CHUNK_PRIMARY>(q, xcd, n_items, head);
        if (it >= n_items) break;
#ifdef YRT_TAIL_STATS
        tail_items++;
#endif
        asm volatile("" ::: "memory");
        const bool valid = primary_samples<false, true, SE, SPB, LDSN, LIST>(S, A_lds, C_lds, B_lds, T,
                                                                            (int)(it * 64) + (YRT_R5_IDXLANE ? lane_now() : (int)lane), wc, lds_rec);
        valid_n += (unsigned)__popcll(ballot(valid));
    }
#ifdef YRT_TAIL_STATS
    tail_record(0, tail_t0, tail_items);
#endif
    const unsigned long long mine = lane == 0 ? (unsigned long long)valid_n : 0ull;
    flush_block<2, SPB>(counters, {cnt_rays, cnt_samples}, {mine, mine});
}

// ---- levels >= 1: closest hit of the compacted mirror rays (grid-stride) ----
template <bool COUNT, bool PACKET, typename SE>
__global__ __launch_bounds__(WF_BLOCK, YRT_TRACE_WAVES) void k_bounce(dev_scene_view S, int level, wf_buffers B,
                                                     unsigned long long* counters) {
    __shared__ traversal_lds<PACKET, SE> lds;
    auto T = make_tracer<false, COUNT, PACKET, SE>(lds);
    work_counts wc;
    unsigned long long rays = 0;
    const int stride = gridDim.x * WF_BLOCK;
    for (int g = 0; g < level_segments; g++) {
    const int n = *seg_counter(B.count, level, g);
    const int nround = (n + stride - 1) / stride;  // uniform: every lane reaches the traversal
    for (int round = 0; round < nround; round++) {
        const int j = round * stride + blockIdx.x * WF_BLOCK + threadIdx.x;
        const bool valid = j < n;
        const int idx = g * B.seg + j;
        ray3 ray = {{0, 0, 0}, {0, 0, 1}, ray_eps, flt_max};
        if (valid) {
            float4 o = ld4(B.ray_o(level) + idx), d = ld4(B.ray_d(level) + idx);
            ray = {xyz(o), xyz(d), ray_eps, flt_max};
            rays++;
        }
        hit_record hr = {-1, -1, {0, 0, 0, 0}, 0};
        const bool hit = T.trace(S, ray, valid, hr, wc);
        if (valid) {
            if (COUNT && hit) wc.hits++;
            if (YRT_HIT16) {
                store_hit16(B, idx, hit, hr);
            } else {
                store_hit_surface(S, B, idx, hit, hr);
            }
        }
    }
    }
    flush_block<1>(counters, {cnt_rays}, {rays});
    if (COUNT) flush_work(counters, wc);
}

// ---- shadow rays (raytrace.cpp:128-133): one light per blockIdx.y ----
// WIDE: the 4-wide any-hit walk (timed kernels on scenes whose wide stack fits);
// otherwise the tracer's binary walk (and always for the instrumented COUNT pass)
template <bool COUNT, bool PACKET, typename SE, bool WIDE>
__global__ __launch_bounds__(shadow_block<PACKET>(), YRT_SHADOW_WAVES) void k_shadow(dev_scene_view S, int level,
                                                                     int nsamp_level0, wf_buffers B,
                                                                     unsigned long long* counters, float4 cam4) {
    const vec3f cam_o = xyz(cam4);  // the camera rays' origin (level 0's view point)
    constexpr int BS = shadow_block<PACKET>();
    __shared__ traversal_lds<PACKET, SE> lds;
    auto T = make_tracer<true, COUNT, PACKET, SE>(lds);
    // level 0 (one block per 256 samples and light): the remap runs over the whole
    // (x, light) grid; levels >= 1 are grid-stride and keep their blocks
    // a pixel block's lights in neighbouring blocks (light index minor), dealt in XCD runs
    const unsigned lin = level ? blockIdx.x
                               : xcd_runs<YRT_SHADOW_LIGHT_MINOR>(blockIdx.y * gridDim.x + blockIdx.x,
                                                                  gridDim.x * gridDim.y);
    const int li = level ? (int)blockIdx.y : (int)(lin % gridDim.y);
    const int bx = level ? (int)blockIdx.x : (int)(lin / gridDim.y);
    const f4* lr = S.lights + 6 * li;
    const frame3f lf = {xyz(ld4(lr)), xyz(ld4(lr + 1)), xyz(ld4(lr + 2)), xyz(ld4(lr + 3))};
    const vec3f lp0 = xyz(ld4(lr + 4)), ke = xyz(ld4(lr + 5));
    work_counts wc;
    unsigned long long rays = 0, culled = 0;  // culled: counted in rays, answered without a walk
    const int stride = gridDim.x * BS;
    for (int g = 0; g < (level ? level_segments : 1); g++) {
    const int n = level ? *seg_counter(B.count, level, g) : nsamp_level0;
    const int nround = (n + stride - 1) / stride;
    for (int round = 0; round < nround; round++) {
        const int j = round * stride + bx * BS + threadIdx.x;
        const int idx = g * B.seg + j;
        bool valid = false;
        int info = -1;
        float r = 1.0f;
        float4 s1 = {0, 0, 0, 0}, ro4 = make_float4(cam_o.x, cam_o.y, cam_o.z, 0.0f);
        ray3 sr = {{0, 0, 0}, {0, 0, 1}, 0.01f, 1.0f};
        constexpr bool CULL = YRT_SHADOW_CULL && !COUNT && !YRT_HIT16;
        if (j < n) {
            float4 s0 = ld4s(B.surf0 + idx);
            if (CULL) {  // n and the view point, for light_term_zero
                s1 = ld4s(B.surf1 + idx);
                if (level) ro4 = ld4(B.ray_o(level) + idx);
            }
            info = sample_state(s0);
            if (info >= 0) {
                const vec3f p = YRT_HIT16 ? hit16_surface(S, s0).p : xyz(s0);
                vec3f tp = transform_point(lf, lp0 - p);
                vec3f l;
                normalize_len(tp, l, r);
                sr = {p, l, 0.01f, r - 0.01f};
                valid = true;
                rays++;
            }
        }
        if (CULL) {  // (uniform control flow; a lane that is not a hit has info < 0)
            if (light_term_zero(info, xyz(s1), sr.o, xyz(ro4), sr.d, r, ke)) {
                stb(B.occl + (size_t)li * B.capacity + idx, 1);
                valid = false;
                culled++;
            }
        }
        hit_record hr;
        bool occ;
        if constexpr (WIDE)
            occ = packet_occluded_wide2(S, sr, valid);
        else
            occ = T.trace(S, sr, valid, hr, wc);
        if (valid) stb(B.occl + (size_t)li * B.capacity + idx, occ ? 1 : 0);
    }
    }
    // shadow rays are counted once, here; yrt_last_stats reports rays = cnt_rays + this
    flush_block<2, BS>(counters, {cnt_shadow_rays, cnt_shadow_culled}, {rays, culled});
    if (COUNT) {
        flush_work(counters, wc);
        flush(counters, cnt_shadow_box_tests, wc.box);
        flush(counters, cnt_shadow_inst_entries, wc.inst);
        flush(counters, cnt_shadow_prim_tests, wc.prim);
        flush(counters, cnt_shadow_wave_node_visits, wc.wnode);
    }
}

// The hull of box P = [P0, P1] and the point Lp, as the 16 lanes of a slot group hold it:
// lane j = lane % 16, j == 0 the hull's box (P's box with Lp), j = 1..12 the plane through
// Lp and box edge j - 1 of P when that edge is on P's silhouette seen from Lp (one adjacent
// face turned towards Lp, the other away). A box is dropped only when some lane finds it
// entirely outside its plane by more than the margin -- a conservative test (the hull's
// other separating axes are not tried); every plane bounds the hull, so a hull holding more
// rays (a super-bundle's) keeps everything a smaller one does.
struct hull_t {
    float bxl, bxh, byl, byh, bzl, bzh;   // j == 0
    float nx, ny, nz, nd, nmargin;        // j >= 1 (nmargin infinite: no plane)
    int j;
};
__device__ __forceinline__ hull_t make_hull(float plx, float ply, float plz, float phx, float phy, float phz, vec3f Lp,
                                            int lane) {
    hull_t H;
    const float M = fmaxf(fmaxf(fmaxf(fabsf(plx), fabsf(ply)), fmaxf(fabsf(plz), fabsf(phx))),
                          fmaxf(fmaxf(fabsf(phy), fabsf(phz)), fmaxf(fmaxf(fabsf(Lp.x), fabsf(Lp.y)), fabsf(Lp.z))));
    const float eps = 1e-3f + 3e-5f * M;
    H.j = lane & 15;
    const float P0[3] = {plx, ply, plz}, P1[3] = {phx, phy, phz}, L3[3] = {Lp.x, Lp.y, Lp.z};
    H.bxl = fminf(plx, Lp.x) - eps, H.bxh = fmaxf(phx, Lp.x) + eps;
    H.byl = fminf(ply, Lp.y) - eps, H.byh = fmaxf(phy, Lp.y) + eps;
    H.bzl = fminf(plz, Lp.z) - eps, H.bzh = fmaxf(phz, Lp.z) + eps;
    H.nx = 0.0f, H.ny = 0.0f, H.nz = 0.0f, H.nd = 0.0f, H.nmargin = INFINITY;
    if (H.j >= 1 && H.j <= 12) {
        const int e = H.j - 1, a = e >> 2, b = (a + 1) % 3, c = (a + 2) % 3;
        const bool bh = e & 1, ch = (e >> 1) & 1;  // the edge's sides on axes b and c
        // a face faces Lp when Lp lies strictly outside the box on that face's side
        const bool fb = bh ? L3[b] > P1[b] : L3[b] < P0[b];
        const bool fc = ch ? L3[c] > P1[c] : L3[c] < P0[c];
        if (fb != fc) {
            float e0[3], e1[3];
            e0[a] = P0[a], e1[a] = P1[a];
            e0[b] = e1[b] = bh ? P1[b] : P0[b];
            e0[c] = e1[c] = ch ? P1[c] : P0[c];
            const float ux = e1[0] - e0[0], uy = e1[1] - e0[1], uz = e1[2] - e0[2];
            const float vx = L3[0] - e0[0], vy = L3[1] - e0[1], vz = L3[2] - e0[2];
            float nx = uy * vz - uz * vy, ny = uz * vx - ux * vz, nz = ux * vy - uy * vx;
            // the box centre on the inner (negative) side
            const float cx = 0.5f * (P0[0] + P1[0]) - e0[0], cy = 0.5f * (P0[1] + P1[1]) - e0[1],
                        cz = 0.5f * (P0[2] + P1[2]) - e0[2];
            if (nx * cx + ny * cy + nz * cz > 0.0f) nx = -nx, ny = -ny, nz = -nz;
            H.nx = nx, H.ny = ny, H.nz = nz;
            H.nd = nx * e0[0] + ny * e0[1] + nz * e0[2];
            H.nmargin = (fabsf(nx) + fabsf(ny) + fabsf(nz)) * (eps + 1e-5f * M);
        }
    }
    return H;
}
// this lane's plane has the box entirely outside (a NaN bound never separates: the
// reference's select-based slab test can pass a box with a NaN plane)
__device__ __forceinline__ bool hull_sep(const hull_t& H, float clx, float cly, float clz, float chx, float chy,
                                         float chz) {
    if (H.j == 0) return clx > H.bxh || chx < H.bxl || cly > H.byh || chy < H.byl || clz > H.bzh || chz < H.bzl;
    const float mn = H.nx * (H.nx > 0.0f ? clx : chx) + H.ny * (H.ny > 0.0f ? cly : chy) +
                     H.nz * (H.nz > 0.0f ? clz : chz);
    return mn - H.nd > H.nmargin;
}
// the instance-level leaves the hull does not exclude, from a walk of the any-hit tree (lane
// 16 s + j tests slot s of the current wide record against plane j; a lane-indexed stack):
// up to CAP of them into cand (lane 0 writes), else overflow
// only_slot >= 0: of the root record, only that slot's subtree (k_bundle_lists<FUSED> splits a
// super-bundle's walk over a block's four waves by root slot)
template <int CAP>
__device__ __forceinline__ void hull_walk(const dev_scene_view& S, const hull_t& H, int lane, float (*cand)[8], int& nc,
                                          bool& overflow, int only_slot = -1) {
    const int s = lane >> 4;  // the slot this lane tests
    const f4* wbase = sgpr_ptr(S.wnodes);
    int stk = 0, sp = 0;
    nc = 0, overflow = false;
    uint32_t cur = (uint32_t)S.wtop_root;
    bool root = true;
    for (;;) {
        float4 r[7];
        ld_wide_record(wbase, cur, r);
        const float4 rs[7] = {r[0], r[1], r[2], r[3], r[4], r[5], r[6]};
        auto comp = [&](float4 v) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; };
        const bool sep = hull_sep(H, comp(rs[0]), comp(rs[1]), comp(rs[2]), comp(rs[3]), comp(rs[4]), comp(rs[5]));
        const unsigned long long sm = ballot(sep);
        unsigned long long m = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t wq = ubits(q == 0 ? r[6].x : q == 1 ? r[6].y : q == 2 ? r[6].z : r[6].w);
            if (wq != wide_leaf && !((sm >> (16 * q)) & 0xffffull)) m |= 0xffffull << (16 * q);
        }
        if (root && only_slot >= 0) m &= 0xffffull << (16 * only_slot);
        root = false;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (!((m >> (16 * q)) & 0xffffull)) continue;
            const uint32_t word = ubits(q == 0 ? r[6].x : q == 1 ? r[6].y : q == 2 ? r[6].z : r[6].w);
            if (word & wide_leaf) {
                if (nc == CAP) {
                    overflow = true;
                    continue;
                }
                if (lane == 0) {
                    float* e = cand[nc];
                    e[0] = q == 0 ? r[0].x : q == 1 ? r[0].y : q == 2 ? r[0].z : r[0].w;
                    e[1] = q == 0 ? r[1].x : q == 1 ? r[1].y : q == 2 ? r[1].z : r[1].w;
                    e[2] = q == 0 ? r[2].x : q == 1 ? r[2].y : q == 2 ? r[2].z : r[2].w;
                    e[3] = q == 0 ? r[3].x : q == 1 ? r[3].y : q == 2 ? r[3].z : r[3].w;
                    e[4] = q == 0 ? r[4].x : q == 1 ? r[4].y : q == 2 ? r[4].z : r[4].w;
                    e[5] = q == 0 ? r[5].x : q == 1 ? r[5].y : q == 2 ? r[5].z : r[5].w;
                    e[6] = __uint_as_float(word);
                }
                nc++;
            } else {
                stk = writelane(stk, (int)word, sp);
                sp++;
            }
        }
        if (overflow || sp == 0) break;
        sp--;
        cur = (uint32_t)__builtin_amdgcn_readlane(stk, sp);
    }
}

// the box of the hit points of items [i0, i0 + n) (n <= 4 * 64: each lane takes up to four),
// whether any is not finite, and the light's position if its frame is the identity
__device__ __forceinline__ void bundle_box(const wf_buffers& B, int i0, int n, int n_items, int lane, float& plx,
                                           float& ply, float& plz, float& phx, float& phy, float& phz, bool& bad) {
    plx = ply = plz = INFINITY, phx = phy = phz = -INFINITY;
    bad = false;
    for (int k = 0; k < 4; k++) {
        const int o = k * 64 + lane, it = i0 + o;
        if (o < n && it < n_items) {
            const float4 a = ld4(B.pbox + 2 * it), b = ld4(B.pbox + 2 * it + 1);
            plx = fminf(plx, a.x), ply = fminf(ply, a.y), plz = fminf(plz, a.z);
            phx = fmaxf(phx, b.x), phy = fmaxf(phy, b.y), phz = fmaxf(phz, b.z);
            bad = bad || a.w < 0.0f;
        }
    }
    float lo[3] = {plx, ply, plz}, hi[3] = {phx, phy, phz};
    wave_box(lo, hi);
    plx = lo[0], ply = lo[1], plz = lo[2], phx = hi[0], phy = hi[1], phz = hi[2];
}
__device__ __forceinline__ bool light_position(const dev_scene_view& S, int li, vec3f& Lp) {
    float4 lrec[5];
    ld_records_at<5>(S.lights, (unsigned)(6 * li), lrec);
    const bool ident = ubits(lrec[0].x) == 0x3f800000u && ubits(lrec[0].y) == 0 && ubits(lrec[0].z) == 0 &&
                       ubits(lrec[1].x) == 0 && ubits(lrec[1].y) == 0x3f800000u && ubits(lrec[1].z) == 0 &&
                       ubits(lrec[2].x) == 0 && ubits(lrec[2].y) == 0 && ubits(lrec[2].z) == 0x3f800000u;
    Lp = xyz(lrec[4]) + xyz(lrec[3]);
    return ident && __builtin_isfinite(Lp.x) && __builtin_isfinite(Lp.y) && __builtin_isfinite(Lp.z);
}

#ifdef YRT_LIST_TIMING
// diagnostic build only (tools/list_timing.py): per wave of the list builders, phase times
// on the 100 MHz constant clock and a size (vector stores by lane 0)
static __device__ unsigned long long g_list_time[3][65536][4];
#define YRT_LT_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#define YRT_LT_WRITE(k, i, a, b, c, d)                                                          \
    do {                                                                                        \
        if (lane == 0 && (unsigned)(i) < 65536u) {                                              \
            unsigned long long* e_ = g_list_time[k][i];                                         \
            e_[0] = (a), e_[1] = (b), e_[2] = (c), e_[3] = (d);                                 \
        }                                                                                       \
    } while (0)
#else
#define YRT_LT_STAMP(v)
#define YRT_LT_WRITE(k, i, a, b, c, d)
#endif

#ifndef YRT_BUNDLE_SUPER
// two-level build: one tree walk per (super-bundle of 4 consecutive bundles, light) into a
// list of up to super_max leaves, which each bundle then filters with its own planes
// instead of walking the tree (a super list that overflows: the bundles walk). A/B in one
// process (profiles/r4/ab_bundle_super): the lists phase at c4 0.28 -> 0.24 ms, c5 rank 0
// of 8 0.82 -> 0.67 ms; identical images
#define YRT_BUNDLE_SUPER 1
#endif
#ifndef YRT_BUNDLE_FUSED
// the super lists and the bundle lists in one launch (k_bundle_lists<true>). A/B in one process
// (profiles/r6/ab/r6e_*): lists phase c4 0.31 -> 0.37 ms, instance100k 0.47 -> 0.60, c5 rank 0
// of 8 0.82 -> 1.00, rank 0 of 8 0.10 -> 0.09; the block's four waves wait at its barrier for
// the longest root slot's walk. Off.
#define YRT_BUNDLE_FUSED 0
#endif
constexpr int super_bundles = 4;
constexpr int super_max = 32;
constexpr int super_list_f4 = 1 + 2 * super_max;  // {count} then {lo, word} {hi, 0} per leaf

// one wave per (super-bundle, light): its list at B.slists
__global__ __launch_bounds__(256) void k_bundle_super(dev_scene_view S, wf_buffers B, int n_items) {
    __shared__ float cand[4][super_max][8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nl = S.nlights;
    const int nsuper = (n_items + super_bundles * bundle_g - 1) / (super_bundles * bundle_g);
    const int sl = blockIdx.x * 4 + w;
    if (sl >= nsuper * nl) return;  // (whole waves)
    YRT_LT_STAMP(lt0);
    const int sg = sl / nl, li = sl - sg * nl;
    f4* out = B.slists + (size_t)sl * super_list_f4;
    float plx, ply, plz, phx, phy, phz;
    bool bad;
    bundle_box(B, sg * super_bundles * bundle_g, super_bundles * bundle_g, n_items, lane, plx, ply, plz, phx, phy, phz,
               bad);
    vec3f Lp;
    const bool lok = light_position(S, li, Lp);
    int nc = -1;
    YRT_LT_STAMP(lt1);
    if (!ballot(bad) && lok) {
        if (!(plx <= phx)) {
            nc = 0;
        } else {
            const hull_t H = make_hull(plx, ply, plz, phx, phy, phz, Lp, lane);
            bool overflow;
            hull_walk<super_max>(S, H, lane, cand[w], nc, overflow);
            if (overflow) nc = -1;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // lane 0's candidate stores
    if (lane < 2 * max(nc, 0)) {
        const float* e = cand[w][lane >> 1];
        reinterpret_cast<float4*>(out)[1 + lane] =
            (lane & 1) ? float4{e[3], e[4], e[5], 0.0f} : float4{e[0], e[1], e[2], e[6]};
    }
    if (lane == 0) reinterpret_cast<float4*>(out)[0] = float4{__int_as_float(nc), 0.0f, 0.0f, 0.0f};
    YRT_LT_STAMP(lt2);
    YRT_LT_WRITE(1, sl, lt1 - lt0, lt2 - lt1, 0ull, (unsigned long long)(unsigned)nc);
}

// one wave per (bundle, light): the candidate list (see above) -- from the super-bundle's
// list (YRT_BUNDLE_SUPER) or a walk of the tree -- as a chain of wide records.
// FUSED (YRT_BUNDLE_FUSED): one block per (super-bundle, light), wave w its bundle w, and the
// super-bundle's list is built in the same launch: the four waves write their bundles' boxes to
// LDS, each walks one root slot's subtree with the super-bundle's hull (the union box), and the
// four shares, in slot order, are the super list every wave then filters -- k_bundle_super's
// list, one launch and one wave's walk fewer
template <bool FUSED>
__global__ __launch_bounds__(256) void k_bundle_lists(dev_scene_view S, wf_buffers B, int n_items) {
    __shared__ float cand[4][bundle_max][8];  // per wave: lo.xyz, hi.xyz, word
    __shared__ float scand[FUSED ? 4 : 1][super_max][8];  // FUSED: root slot w's share of the super list
    __shared__ float sbox[FUSED ? 4 : 1][8];             // FUSED: bundle w's box, and whether it is bad
    __shared__ int scount[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nl = S.nlights;
    const int ngroups = (n_items + bundle_g - 1) / bundle_g;
    int g, li;
    if constexpr (FUSED) {
        const int nsuper = (ngroups + super_bundles - 1) / super_bundles;
        if ((int)blockIdx.x >= nsuper * nl) return;  // (whole blocks)
        const int sg = (int)blockIdx.x / nl;
        li = (int)blockIdx.x - sg * nl, g = sg * super_bundles + w;
    } else {
        const int gl0 = blockIdx.x * 4 + w;
        if (gl0 >= ngroups * nl) return;  // (whole waves)
        g = gl0 / nl, li = gl0 - g * nl;
    }
    const int gl = g * nl + li;
    YRT_LT_STAMP(lt0);
    float plx, ply, plz, phx, phy, phz;
    bool bad;
    // (a bundle past the last, FUSED's padding: no items, an empty box)
    bundle_box(B, g * bundle_g, bundle_g, n_items, lane, plx, ply, plz, phx, phy, phz, bad);
    int sc = -1;  // the super-bundle's list length, -1: walk the tree
    const f4* sup = nullptr;
    if constexpr (FUSED) {
        const bool wbad = ballot(bad) != 0;
        if (lane == 0) {
            float* b = sbox[w];
            b[0] = plx, b[1] = ply, b[2] = plz, b[3] = phx, b[4] = phy, b[5] = phz, b[6] = wbad ? 1.0f : 0.0f;
        }
        __syncthreads();
        // the super-bundle's box: the union of its bundles' (bundle_box's fminf / fmaxf fold)
        float Plx = INFINITY, Ply = INFINITY, Plz = INFINITY, Phx = -INFINITY, Phy = -INFINITY, Phz = -INFINITY;
        bool sbad = false;
        for (int q = 0; q < super_bundles; q++) {
            const float* b = sbox[q];
            Plx = fminf(Plx, b[0]), Ply = fminf(Ply, b[1]), Plz = fminf(Plz, b[2]);
            Phx = fmaxf(Phx, b[3]), Phy = fmaxf(Phy, b[4]), Phz = fmaxf(Phz, b[5]);
            sbad = sbad || b[6] != 0.0f;
        }
        vec3f Ls;
        const bool lok = light_position(S, li, Ls);
        int nq = -1;
        if (!sbad && lok) {
            if (!(Plx <= Phx)) {
                nq = 0;
            } else {
                const hull_t Hs = make_hull(Plx, Ply, Plz, Phx, Phy, Phz, Ls, lane);
                bool of;
                hull_walk<super_max>(S, Hs, lane, scand[w], nq, of, w);
                if (of) nq = -1;
            }
        }
        if (lane == 0) scount[w] = nq;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // lane 0's candidate stores
        __syncthreads();
        const int c0 = scount[0], c1 = scount[1], c2 = scount[2], c3 = scount[3];
        sc = (c0 < 0 || c1 < 0 || c2 < 0 || c3 < 0 || c0 + c1 + c2 + c3 > super_max) ? -1 : c0 + c1 + c2 + c3;
        if (g >= ngroups) return;  // (after the block's barriers)
    }
    vec3f Lp;
    if (ballot(bad) || !light_position(S, li, Lp)) {
        if (lane == 0) B.lcount[gl] = -1, B.lskip[gl] = 0;
        return;
    }
    if (!(plx <= phx)) {  // no hit point in the bundle: no shadow ray
        if (lane == 0) B.lcount[gl] = 0, B.lskip[gl] = 0;
        return;
    }
    const hull_t H = make_hull(plx, ply, plz, phx, phy, phz, Lp, lane);
    int nc = 0;
    bool overflow = false;
    if (!FUSED && YRT_BUNDLE_SUPER && bundle_g * super_bundles <= 256) {
        sup = B.slists + (size_t)((g / super_bundles) * nl + li) * super_list_f4;
        sc = __builtin_amdgcn_readfirstlane(__float_as_int(ld4(sup).x));
    }
    if (sc >= 0) {
        // the super list's leaves that this bundle's own planes do not exclude: lane 16 s + j
        // tests leaf c0 + s against plane j, four leaves a pass
        for (int c0 = 0; c0 < sc && !overflow; c0 += 4) {
            const int e = c0 + (lane >> 4);
            float4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
            if (e < sc) {
                if constexpr (FUSED) {  // entry e of the four shares, in slot order
                    int q = 0, k = e;
                    while (k >= scount[q]) k -= scount[q], q++;
                    const float* d = scand[q][k];
                    a = {d[0], d[1], d[2], d[6]}, b = {d[3], d[4], d[5], 0.0f};
                } else {
                    a = ld4(sup + 1 + 2 * e), b = ld4(sup + 2 + 2 * e);
                }
            }
            const bool sep = e >= sc || hull_sep(H, a.x, a.y, a.z, b.x, b.y, b.z);
            const unsigned long long sm = ballot(sep);
            unsigned keep = 0;  // bit q: leaf c0 + q stays
            for (int q = 0; q < 4; q++) keep |= ((sm >> (16 * q)) & 0xffffull) ? 0u : 1u << q;
            const int k = __popc(keep);
            if (nc + k > bundle_max) {
                overflow = true;
                break;
            }
            const int q = lane >> 4;
            if ((lane & 15) == 0 && ((keep >> q) & 1u)) {
                float* d = cand[w][nc + __popc(keep & ((1u << q) - 1u))];
                d[0] = a.x, d[1] = a.y, d[2] = a.z, d[3] = b.x, d[4] = b.y, d[5] = b.z, d[6] = a.w;
            }
            nc += k;
        }
    } else {
        hull_walk<bundle_max>(S, H, lane, cand[w], nc, overflow);
    }
    if (overflow) {
        if (lane == 0) B.lcount[gl] = -1, B.lskip[gl] = 0;
        return;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the candidate stores, before any lane reads them
    YRT_LT_STAMP(lt1);
    if (YRT_BUNDLE_SORT && nc > 1) {
        // the leaves in the order the bundle's rays meet them (box centres projected on the
        // direction from the hit points to the light; YRT_BUNDLE_SORT), so that the chain's
        // later records are compact boxes the rays can pass by and an occluded bundle meets
        // its occluder sooner. The any-hit answer does not depend on the order.
        const float cx = 0.5f * (plx + phx), cy = 0.5f * (ply + phy), cz = 0.5f * (plz + phz);
        const float dx = Lp.x - cx, dy = Lp.y - cy, dz = Lp.z - cz;
        float e[7] = {};
        float key = INFINITY;
        if (lane < nc) {
            for (int q = 0; q < 7; q++) e[q] = cand[w][lane][q];
            key = (0.5f * (e[0] + e[3]) - cx) * dx + (0.5f * (e[1] + e[4]) - cy) * dy + (0.5f * (e[2] + e[5]) - cz) * dz;
            if (YRT_BUNDLE_SORT == 2) key = -key;
            if (!(key == key)) key = INFINITY;  // (a NaN bound: last)
        }
        int rank = 0;  // a permutation of 0 .. nc - 1: ties go by index
        for (int j = 0; j < nc; j++) {
            const float kj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(key), j));
            rank += (kj < key || (kj == key && j < (int)lane)) ? 1 : 0;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's reads, before the writes
        if (lane < nc)
            for (int q = 0; q < 7; q++) cand[w][rank][q] = e[q];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // the instances of each listed leaf that the hull excludes: their world boxes
    // (dev_scene_view ibox) outside a hull plane by more than the margin fail every ray's
    // root box test in the instance's space, so the walk skips them (skip bits in the leaf's
    // word: the bundle records' format, bundle_leaf_word)
    int nskip = 0;  // (wave-uniform) instances the hull excludes, over the listed leaves
    if (YRT_INSTANCE_MASKS && S.inst_masks) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int e = 0; e < nc; e++) {
            const uint32_t wu = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(cand[w][e][6]));
            const int first = (int)(wu & wide_index_mask), count = (int)((wu >> wide_count_shift) & 7u);
            uint32_t skip = 0;
            for (int i0 = 0; count > 1 && i0 < count; i0 += 4) {
                const int i = i0 + (lane >> 4);  // lane 16 s + j: instance i0 + s against plane j
                bool sep = false;
                if (i < count) {
                    const float4 a = ld4(S.ibox + 2 * (first + i)), b = ld4(S.ibox + 2 * (first + i) + 1);
                    sep = hull_sep(H, a.x, a.y, a.z, b.x, b.y, b.z);
                }
                const unsigned long long sm = ballot(sep);
                for (int q = 0; q < 4; q++)
                    if (i0 + q < count && ((sm >> (16 * q)) & 0xffffull)) skip |= 1u << (i0 + q);
            }
            if (lane == 0) cand[w][e][6] = __uint_as_float(bundle_leaf_word(first, count, skip));
            nskip += __popc(skip);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // a leaf whose every instance is excluded leaves the list (the walk would test its box
        // and enter nothing); the others keep their order
        float e[7] = {};
        bool keep = false;
        if (lane < nc) {
            for (int q = 0; q < 7; q++) e[q] = cand[w][lane][q];
            const uint32_t wu = ubits(e[6]);
            const int count = (int)((wu >> wide_count_shift) & 7u);
            const uint32_t all = (1u << count) - 1u;
            keep = count == 0 || ((wu >> bundle_skip_shift) & 0x7fu) != all;
        }
        const unsigned long long km = ballot(keep);
        const int pos = __popcll(km & ((1ull << lane) - 1ull));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's reads, before the writes
        if (keep)
            for (int q = 0; q < 7; q++) cand[w][pos][q] = e[q];
        nc = __popcll(km);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    YRT_LT_STAMP(lt2);
    // the list as wide records at B.lists + gl * bundle_recs: up to 4 leaves in the root;
    // more in up to 4 child records of 4, the root's slot c holding child c's box (the union
    // of its leaves' boxes) and its byte offset from B.lists
    // a chain: record r holds leaves 3r, 3r + 1, 3r + 2 and, in slot 3, record r + 1 (its box
    // the union of every leaf after them) -- the last record holds the last <= 4 leaves
    const int nrec = nc <= 4 ? 1 : 1 + (nc - 4 + 2) / 3;
    const uint32_t rec0 = (uint32_t)gl * bundle_recs;
    // lane q (< nrec * 4) builds slot q % 4 of record q / 4 -- then lanes write the rows
    __shared__ float slot[4][bundle_recs * 4][8];
    if (lane < nrec * 4) {
        const int rq = lane / 4, c = lane % 4;
        float v[7] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY, __uint_as_float(wide_leaf)};
        if (rq == nrec - 1 || c < 3) {  // a leaf
            const int e = 3 * rq + c;
            if (e < nc)
                for (int q = 0; q < 7; q++) v[q] = cand[w][e][q];
        } else {  // the rest of the chain
            // the union of the later leaves' boxes, a NaN bound sticking: the walk's slab test
            // ignores a NaN plane, so a leaf with one passes more rays than its finite bounds
            // say, and the chain box must let all of those through too (fminf / fmaxf alone
            // would drop the NaN and could narrow the box below that leaf's reach)
            for (int e = 3 * rq + 3; e < nc; e++)
                for (int q = 0; q < 3; q++) {
                    const float lo = cand[w][e][q], hi = cand[w][e][q + 3];
                    v[q] = (lo != lo || v[q] != v[q]) ? __builtin_nanf("") : fminf(v[q], lo);
                    v[q + 3] = (hi != hi || v[q + 3] != v[q + 3]) ? __builtin_nanf("") : fmaxf(v[q + 3], hi);
                }
            v[6] = __uint_as_float((rec0 + rq + 1) * (uint32_t)wide_record_bytes);
        }
        for (int q = 0; q < 7; q++) slot[w][lane][q] = v[q];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane < nrec * 8) {
        const int rq = lane / 8, row = lane % 8;
        const float* a = slot[w][4 * rq];
        float4 o = row < 7 ? make_float4(a[row], a[8 + row], a[16 + row], a[24 + row]) : make_float4(0, 0, 0, 0);
        reinterpret_cast<float4*>(B.lists)[(size_t)(rec0 + rq) * 8 + row] = o;
    }
    if (lane == 0) B.lcount[gl] = nc, B.lskip[gl] = nskip;
    YRT_LT_STAMP(lt3);
    YRT_LT_WRITE(2, gl, lt1 - lt0, lt2 - lt1, lt3 - lt2, (unsigned long long)(unsigned)nc);
}

// ---- camera lists: per 8x8-pixel tile of the chunk, a frontier of the reference's instance
// tree for packet_first's list mode. The tile's rays start at the camera origin O and run
// through its pixels' rectangle [i0, i1 + 1] x [j0, j1 + 1] of the image plane (the samples lie
// strictly inside it, raytrace.cpp:236-239), so they lie in the cone from O through the
// rectangle's four corners; a box that lies outside a cone plane by more than a margin above
// the slab test's rounding fails every such ray's exact test (intersect_check_bbox,
// scene.cpp:371-382) at any tmax.
//
// The list is a frontier: disjoint subtrees of the reference's tree (inner nodes or leaves)
// that together hold every leaf the cone reaches, in the reference's DFS order (child start+1
// before start, scene.cpp:446-479). One wave per tile grows it from the root, a round per tree
// level, lane q holding entry q: an inner entry whose children the cone reaches one or none of
// is replaced by that child (or dropped) -- that never lengthens the list --, and one whose
// children both stay is replaced by them while the list has room (camera_list_max entries, the
// earlier entries first), so a small frontier ends as the tile's leaf list and a large one
// keeps subtrees where the cone splits. Entries are the first 32 bytes of the node's
// camera-relative spine record (trel: {lo - o, child record offset or first slot}
// {hi - o, count | leaf}), exactly what the walk reads for that node.
__global__ __launch_bounds__(256) void k_camera_lists(dev_scene_view S, dev_render_args A, chunk_args C, wf_buffers B) {
    constexpr int K = camera_list_max;
    static_assert(K <= 64, "one list entry per lane");
    __shared__ float4 fr[4][2][K][2];  // per wave: the frontier, double-buffered
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ntiles = C.npix / (TILE * TILE);
    const int t = blockIdx.x * 4 + w;
    if (t >= ntiles) return;  // (whole waves)
    YRT_LT_STAMP(lt0);
    const long long T = C.pix0 / (TILE * TILE) + t;
    const int lx0 = (int)(T % C.tiles_x) * TILE, ly0 = (int)(T / C.tiles_x) * TILE;
    // the tile's image columns and rows (bands interleave the rows: take their range)
    const int i0 = A.x0 + lx0, i1 = A.x0 + lx0 + TILE - 1;
    int jr;
    {
        const int ly = ly0 + (lane < TILE ? lane : 0);
        const int b = ly / A.band, r = ly % A.band;
        jr = A.y0 + (b * A.band_stride + A.band_offset) * A.band + r;
    }
    int j0 = jr, j1 = jr;
    for (int off = 1; off < 64; off <<= 1) j0 = min(j0, __shfl_xor(j0, off, 64)), j1 = max(j1, __shfl_xor(j1, off, 64));
    j0 = uniform(j0), j1 = uniform(j1);
    const float u0 = (float)i0 / (float)A.width, u1 = (float)(i1 + 1) / (float)A.width;
    const float v0 = (float)j0 / (float)A.height, v1 = (float)(j1 + 1) / (float)A.height;
    const dev_camera& Kc = A.cam;
    auto dir = [&](float u, float v) {
        return vec3f{(u - 0.5f) * Kc.w * Kc.xx + (v - 0.5f) * Kc.h * Kc.yx - Kc.focus * Kc.zx,
                     (u - 0.5f) * Kc.w * Kc.xy + (v - 0.5f) * Kc.h * Kc.yy - Kc.focus * Kc.zy,
                     (u - 0.5f) * Kc.w * Kc.xz + (v - 0.5f) * Kc.h * Kc.yz - Kc.focus * Kc.zz};
    };
    const vec3f O = {Kc.ox, Kc.oy, Kc.oz};
    // the margin of a box: 1e-3 + 3e-5 x the magnitude of its coordinates and the origin's, far
    // above the slab test's rounding at that magnitude. Per box, not the scene's: the root box's
    // magnitude made it huge for every box once one instance was (an instance of an empty shape
    // is bounded by +-FLT_MAX), and every list became the whole tree.
    const float Om = fmaxf(fmaxf(fabsf(O.x), fabsf(O.y)), fabsf(O.z));
    // cone plane k (through O and corners k, k + 1; the cone on its negative side), computed by
    // lane k < 4 and read by every lane
    vec3f n = {0, 0, 0};
    if (lane < 4) {
        const float cu[4] = {u0, u1, u1, u0}, cv[4] = {v0, v0, v1, v1};
        const vec3f a = dir(cu[lane], cv[lane]), b = dir(cu[(lane + 1) & 3], cv[(lane + 1) & 3]);
        n = cross(a, b);
        const vec3f c = dir(0.5f * (u0 + u1), 0.5f * (v0 + v1));
        if (dot(n, c) > 0.0f) n = n * -1.0f;
    }
    float pn[4][3], pl1[4];
    for (int k = 0; k < 4; k++) {
        pn[k][0] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(n.x), k));
        pn[k][1] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(n.y), k));
        pn[k][2] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(n.z), k));
        pl1[k] = fabsf(pn[k][0]) + fabsf(pn[k][1]) + fabsf(pn[k][2]);
    }
    // a camera-relative box outside some cone plane by more than its margin (a NaN bound never
    // separates; neither does an infinite one, whose margin is infinite)
    auto outside = [&](float4 lo, float4 hi) {
        const float Mb = Om + fmaxf(fmaxf(fmaxf(fabsf(lo.x), fabsf(lo.y)), fmaxf(fabsf(lo.z), fabsf(hi.x))),
                                    fmaxf(fabsf(hi.y), fabsf(hi.z)));
        const float eps = 1e-3f + 3e-5f * Mb;
        bool o = false;
        for (int k = 0; k < 4; k++) {
            const float mn = pn[k][0] * (pn[k][0] > 0.0f ? lo.x : hi.x) + pn[k][1] * (pn[k][1] > 0.0f ? lo.y : hi.y) +
                             pn[k][2] * (pn[k][2] > 0.0f ? lo.z : hi.z);
            o = o || mn > pl1[k] * eps;
        }
        return o;
    };
    const f4* trel = B.trel;
    const unsigned long long below = (1ull << lane) - 1ull;
    // the frontier starts as the tree's top cut (S.tcut: the nodes at depth camera_cut_depth
    // and the leaves above it, in DFS order) less the nodes the cone excludes -- one round of
    // parallel loads instead of camera_cut_depth dependent ones from the root. A node whose
    // ancestor the cone excludes is excluded too (its box lies inside the ancestor's), and an
    // entry kept needlessly only costs its box test in the walk: the list stays exact.
    static_assert((1 << camera_cut_depth) <= K, "the top cut fits one list");
    int nf, cur = 0;
    {
        float4 rl = {0, 0, 0, 0}, rh = {0, 0, 0, 0};
        bool in = false;
        if (lane < S.ntcut) {
            const f4* r = trel + (size_t)((unsigned)S.tcut[lane] / 16u);
            rl = ld4(r), rh = ld4(r + 1);
            in = !outside(rl, rh);
        }
        const unsigned long long km0 = ballot(in);
        if (in) {
            const int q = __popcll(km0 & below);
            fr[w][0][q][0] = rl, fr[w][0][q][1] = rh;
        }
        nf = __popcll(km0);
    }
#ifdef YRT_LIST_TIMING
    int nrounds = 0;
#endif
    YRT_LT_STAMP(lt1);
    for (int round = 0; round < 64 && nf > 0; round++) {
#ifdef YRT_LIST_TIMING
        nrounds++;
#endif
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        float4 lo = {0, 0, 0, 0}, hi = {0, 0, 0, 0}, alo = lo, ahi = lo, blo = lo, bhi = lo;
        bool inner = false, ka = false, kb = false;
        if (lane < nf) {
            lo = fr[w][cur][lane][0], hi = fr[w][cur][lane][1];
            inner = !(ubits(hi.w) & leaf_bit);
            if (inner) {
                // children start (B) and start + 1 (A): adjacent records, start's at byte offset lo.w
                const f4* rb = trel + (size_t)((unsigned)ibits(lo.w) / 16u);
                blo = ld4(rb), bhi = ld4(rb + 1), alo = ld4(rb + spine_record_f4), ahi = ld4(rb + spine_record_f4 + 1);
                ka = !outside(alo, ahi), kb = !outside(blo, bhi);
            }
        }
        const int c = (int)ka + (int)kb;
        const bool both = inner && c == 2;  // expanding it lengthens the list by one
        const bool shrink = inner && c < 2;
        // the list's length with no two-child expansion, then the two-child ones that fit, in order
        const int size0 = lane < nf ? (shrink ? c : 1) : 0;
        const unsigned long long b1 = ballot(size0 & 1), b2 = ballot(size0 & 2);
        const int len0 = __popcll(b1) + 2 * __popcll(b2);
        const unsigned long long bb = ballot(both);
        const bool grow = both && __popcll(bb & below) < K - len0;
        if (!ballot(shrink || grow)) break;
        const int size = grow ? 2 : size0;
        const unsigned long long s1 = ballot(size & 1), s2 = ballot(size & 2);
        const int pos = __popcll(s1 & below) + 2 * __popcll(s2 & below);
        float4(*dst)[2] = fr[w][cur ^ 1];
        if (shrink || grow) {
            int q = pos;
            if (ka) dst[q][0] = alo, dst[q][1] = ahi, q++;  // the reference visits start+1 first
            if (kb) dst[q][0] = blo, dst[q][1] = bhi;
        } else if (lane < nf) {
            dst[pos][0] = lo, dst[pos][1] = hi;
        }
        nf = __popcll(s1) + 2 * __popcll(s2);
        cur ^= 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    YRT_LT_STAMP(lt2);
    float4 elo = {0, 0, 0, 0}, ehi = {0, 0, 0, 0};
    bool keep = false;
    int nskip = 0;  // this lane's entry: the instances the cone excludes
    if (lane < nf) {
        const float4 lo = fr[w][cur][lane][0];
        float4 hi = fr[w][cur][lane][1];
        // a listed leaf's instances that the cone excludes (their world boxes, dev_scene_view
        // ibox, relative to O and outside a cone plane by more than the margin: every ray of
        // the tile fails their root box test in the instance's space): skip bits 16-30 of the
        // entry's count word, which packet_first's list mode honours (a tree leaf's are 0)
        const uint32_t cw = ubits(hi.w);
        const int count = (int)(cw & 0xffffu);
        if (YRT_INSTANCE_MASKS && S.ibox && (cw & leaf_bit) && count > 1 && count <= 15) {
            const int first = ibits(lo.w);
            uint32_t skip = 0;
            for (int i = 0; i < count; i++) {
                const float4 a = ld4(S.ibox + 2 * (first + i)), b = ld4(S.ibox + 2 * (first + i) + 1);
                const float4 ar = {a.x - O.x, a.y - O.y, a.z - O.z, 0.0f}, br = {b.x - O.x, b.y - O.y, b.z - O.z, 0.0f};
                if (outside(ar, br)) skip |= 1u << i;
            }
            hi.w = __uint_as_float(cw | skip << 16);
            nskip = __popc(skip);
            // a leaf whose every instance is excluded leaves the list
            keep = skip != (1u << count) - 1u;
        } else {
            keep = true;
        }
        elo = lo, ehi = hi;
    }
    // the kept entries, in order
    const unsigned long long km = ballot(keep);
    if (keep) {
        f4* out = B.clist + ((size_t)t * camera_list_max + __popcll(km & below)) * 2;
        out[0] = {elo.x, elo.y, elo.z, elo.w};
        out[1] = {ehi.x, ehi.y, ehi.z, ehi.w};
    }
    nf = __popcll(km);
    nskip = (int)wave_sum((unsigned long long)nskip);
    if (lane == 0) B.ccount[t] = nf, B.cskip[t] = nskip;
    YRT_LT_STAMP(lt3);
    YRT_LT_WRITE(0, t, lt1 - lt0, lt2 - lt1, lt3 - lt2, (unsigned long long)nrounds << 32 | (unsigned)nf);
}

// the sums of one chunk's list lengths into B.lstats (a list that fell back to the tree counts
// as camera_list_max + 1 / bundle_max + 1 entries) and of the instances the lists' masks
// exclude, added to the render's totals: a grid-stride sum per block, list_sums atomics per block
__global__ __launch_bounds__(256) void k_list_stats(wf_buffers B, int ntiles, int nlists) {
    __shared__ unsigned long long part[list_sums][256 / 64];
    unsigned long long v[list_sums] = {};
    const int stride = gridDim.x * 256;
    if (B.cam_lists)
        for (int i = blockIdx.x * 256 + (int)threadIdx.x; i < ntiles; i += stride) {
            const int n = B.ccount[i];
            v[0] += n < 0 ? camera_list_max + 1 : n, v[1]++, v[4] += (unsigned)B.cskip[i];
        }
    if (B.bundles)
        for (int i = blockIdx.x * 256 + (int)threadIdx.x; i < nlists; i += stride) {
            const int n = B.lcount[i];
            v[2] += n < 0 ? bundle_max + 1 : n, v[3]++, v[5] += (unsigned)B.lskip[i];
        }
    for (int q = 0; q < list_sums; q++) {
        const unsigned long long t = wave_sum(v[q]);
        if ((threadIdx.x & 63) == 0) part[q][threadIdx.x >> 6] = t;
    }
    __syncthreads();
    if (threadIdx.x < list_sums) {
        const unsigned long long t = part[threadIdx.x][0] + part[threadIdx.x][1] + part[threadIdx.x][2] + part[threadIdx.x][3];
        if (t) atomicAdd(B.lstats + threadIdx.x, t);
    }
}

// ---- shadow rays, persistent: a grid of SP_BLOCK-thread blocks that fills the chip once;
// every wave walks its own share of the (64-sample block, light) items, so no block
// launch, block retirement or per-block counter flush happens per item (level 0 with
// enough items; the kernel also takes a mirror level's sample count from the device). LDSN > 0: each block first stages the first LDSN 4-wide records --
// the breadth-first top of the instance tree (device_scene.cpp emit_bfs) -- in LDS, and
// the walk reads those with ds_read_b128 instead of through the scalar cache (the
// north_star's "hot node tiles staged in LDS").
//
// Item order: item = bx * nlights + light (the light index minor, as k_shadow). The
// hardware deals workgroup b to XCD b % 8; XCD x takes runs x, x + 8, x + 16, ... of C
// consecutive items (k_shadow's XCD runs), its blocks taking chunks of them in order, so
// all eight XCDs sweep the image together while each traces neighbouring pixels. Items
// past the last whole super-run are dealt round-robin to the XCDs.
#ifndef YRT_SHADOW_PERSIST_MIN_ITEMS
// the persistent grid saves the hardware dealing's per-block cost and, with block chunks,
// keeps a CU's waves on neighbouring items; it needs enough items per wave to amortise its
// start and tail (A/B against k_shadow, items = 64-sample blocks x lights: 6.2 M (a c4
// frame) -6 % before block chunks, which take another 2.7 % off; 1.55 M (rank 0 of 4) -10 %; 1.04 M (c3's level 0) -9 %; 0.78 M (rank 0 of
// 8) -9.5 %; 43 K (instance10000 at 720p, 1 spp) +1 %; 29 K (c2) +20 %)
#define YRT_SHADOW_PERSIST_MIN_ITEMS 262144
#endif
#ifndef YRT_SHADOW_ITEM_LIGHTS
// an item is a 64-sample block with all its lights, looped inside the item, instead of one
// (block, light) pair: one queue position, item split, index arithmetic and bundle-list
// prologue per block (A/B, one process: c4 shadow 8.14 -> 7.79 ms, instance100k 4.69 -> 3.01,
// instance1k 5.30 -> 4.77, c3 1.54 -> 1.46, rank 0 of 8 equal)
#define YRT_SHADOW_ITEM_LIGHTS 1
#endif
#ifndef YRT_SHADOW_ITEM_RUN
#define YRT_SHADOW_ITEM_RUN 48  // (YRT_SHADOW_ITEM_LIGHTS) XCD run length in 64-sample blocks (12 / 24 / 48: within 1 %)
#endif
#ifndef YRT_SHADOW_LDS_RECORDS
// k_shadow_persist with LDS staging on (yrt_scene_set_lds_staging): the 4-wide records staged
// in LDS per block (A/B: 21 / 85 / 341 records +2 / +2 / +3 %; the handle's default is off)
#define YRT_SHADOW_LDS_RECORDS 85
#endif

template <int LDSN>
__global__ __launch_bounds__(SP_BLOCK, YRT_SHADOW_WAVES) void k_shadow_persist(dev_scene_view S, int nsamp,
                                                                                int nx, wf_buffers B,
                                                                                unsigned long long* counters,
                                                                                float4 cam4) {
    const vec3f cam_o = xyz(cam4);  // the camera rays' origin: the view point of level 0's shading
    constexpr int WPB = SP_BLOCK / 64;  // waves per block
    constexpr unsigned C = (YRT_SHADOW_ITEM_LIGHTS && LDSN == 0) ? YRT_SHADOW_ITEM_RUN : YRT_SHADOW_LIGHT_MINOR;
    __shared__ float4 lds_nodes[LDSN > 0 ? LDSN * 8 : 1];
    if constexpr (LDSN > 0) {
        const int nrec = LDSN * 8;
        const float4* src = reinterpret_cast<const float4*>(S.wnodes);
        for (int i = threadIdx.x; i < nrec; i += SP_BLOCK) lds_nodes[i] = src[i];
        __syncthreads();
    }
    const int nl = S.nlights;
    // YRT_SHADOW_ITEM_LIGHTS: an item is a 64-sample block with every light (the lights looped
    // inside it: one queue position, one item split, per block instead of per (block, light))
    // (not with LDS-staged records: that copy keeps its registers for the staged walk)
    constexpr bool IL = YRT_SHADOW_ITEM_LIGHTS && LDSN == 0;
    const unsigned n_items = IL ? (unsigned)nx : (unsigned)nx * (unsigned)nl;
    const unsigned lane = threadIdx.x & 63;
    const unsigned xcd = blockIdx.x % 8u;
    unsigned rays = 0;  // wave-uniform (an SGPR): shadow rays of this wave (the reference's count)
    // per lane (a VGPR: one more SGPR would spill): this lane's rays answered without a walk
    unsigned culled_l = 0;
    // positions from the block's chunk ring (chunk_ring_next), YRT_SHADOW_BLOCK_CHUNK at a time
    constexpr unsigned CS = YRT_SHADOW_BLOCK_CHUNK;
    __shared__ chunk_ring ring;
    const unsigned head = head_items<C, CS>(n_items);
    chunk_ring_init<CS>(ring, B.queue + xcd, B.queue + 8, head / 8u);
#ifdef YRT_TAIL_STATS
    const unsigned long long tail_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned tail_items = 0;
#endif
    for (;;) {
        const unsigned q = chunk_ring_next<CS>(ring, B.queue + xcd, lane, B.queue + 8, head / 8u);
        const unsigned it = split_item<C>(q, xcd, n_items, head);
        if (it >= n_items) break;
#ifdef YRT_TAIL_STATS
        tail_items++;
#endif
        const int bx = IL ? (int)it : (int)(it / (unsigned)nl);
        for (int lq = 0; lq < (IL ? nl : 1); lq++) {
        const int li = IL ? lq : (int)(it % (unsigned)nl);
        // the light's frame and position: one wave-uniform record, through the scalar cache
        float4 lrec[6];
        ld_records_at<6>(S.lights, (unsigned)(6 * li), lrec);
        const frame3f lf = {xyz(lrec[0]), xyz(lrec[1]), xyz(lrec[2]), xyz(lrec[3])};
        const vec3f lp0 = xyz(lrec[4]);
        const int idx = bx * 64 + (int)lane;
        bool valid = false;
        int info = -1;
        float r = 1.0f;
        float4 s1 = {0, 0, 0, 0};
        ray3 sr = {{0, 0, 0}, {0, 0, 1}, 0.01f, 1.0f};
        if (idx < nsamp) {
            // (every light of the item reads the sample's surface again: cached loads, not the
            // streaming ones; holding it across the walks instead spills 5 VGPRs: +0.5 %)
            float4 s0 = IL ? ld4(B.surf0 + idx) : ld4s(B.surf0 + idx);
            if (YRT_SHADOW_CULL && !YRT_HIT16) s1 = IL ? ld4(B.surf1 + idx) : ld4s(B.surf1 + idx);  // n, for light_term_zero
            info = sample_state(s0);
            if (info >= 0) {
                const vec3f p = YRT_HIT16 ? hit16_surface(S, s0).p : xyz(s0);
                vec3f tp = transform_point(lf, lp0 - p);
                vec3f l;
                normalize_len(tp, l, r);
                sr = {p, l, 0.01f, r - 0.01f};
                valid = true;
            }
        }
        rays += (unsigned)__popcll(ballot(valid));
        // the rays whose light term is zero (light_term_zero, called by every lane in uniform
        // control flow: its loads and ballots see the whole wave; it is false on a lane that is
        // not a hit, info < 0, so it implies valid) start the walk as done -- recorded as
        // occluded -- and a wave whose every ray is culled skips it. (Taking them out of `valid`
        // instead trips the compiler inside this loop: "illegal VGPR to SGPR copy".)
        const bool zero_term =
            YRT_SHADOW_CULL && !YRT_HIT16 && light_term_zero(info, xyz(s1), sr.o, cam_o, sr.d, r, xyz(lrec[5]));
        const unsigned long long culled = ballot(zero_term);
        culled_l += zero_term ? 1u : 0u;
        const bool all_culled = YRT_SHADOW_CULL && !YRT_HIT16 && culled == ballot(valid);
        bool occ;
        int lc = -1;  // the bundle's list: its leaf count, -1 = walk the tree
        if (YRT_SHADOW_BUNDLES && LDSN == 0 && B.bundles) {
            const int gl = (bx / bundle_g) * nl + li;
            lc = __builtin_amdgcn_readfirstlane(B.lcount[gl]);
        }
        const f4* tbase = S.wnodes;
        uint32_t troot = (uint32_t)S.wtop_root;
        if (lc > 0) {  // (the host turns bundles off with LDS-staged records: LDSN == 0 here)
            tbase = B.lists;
            troot = (uint32_t)(((bx / bundle_g) * nl + li) * bundle_recs * wide_record_bytes);
        }
        // lc == 0: no leaf can be passed by these rays, none is occluded; all_culled: recorded
        // as occluded, k_shade skips the light
        occ = all_culled ? true
                         : lc == 0 ? ((culled >> lane) & 1ull) != 0
                                   : packet_occluded_wide2<LDSN, true>(S, sr, valid, lds_nodes, tbase, troot, culled);
        if (valid) stb(B.occl + (size_t)li * B.capacity + idx, occ ? 1 : 0);
        }
    }
#ifdef YRT_TAIL_STATS
    tail_record(1, tail_t0, tail_items);
#endif
    const unsigned long long mine = lane == 0 ? (unsigned long long)rays : 0ull;
    flush_block<2, SP_BLOCK>(counters, {cnt_shadow_rays, cnt_shadow_culled}, {mine, (unsigned long long)culled_l});
}

// ---- shade() after the queries (raytrace.cpp:99-206) ----
// FUSE (level 0 of a scene without mirrors, s*s dividing the block): the block's
// samples are whole pixels, so the ordered per-pixel sum of k_accumulate is done here
// from LDS and the per-sample radiance never goes to HBM.
#ifndef YRT_SHADE_WAVES
#define YRT_SHADE_WAVES 7  // k_shade register budget: 65-73 VGPRs with the f64 pow called (A/B at c4: 5 -> 7 waves -4 %; with the pow inlined it needed 96)
#endif
// OCC4 (scenes with at most four lights): the occlusion bytes are loaded together with the
// surface, one memory round trip instead of one per light inside the light loop.
#ifndef YRT_SHADE_LDS_SRGB
// textured scenes: the srgb table (1 KiB) is copied into LDS per block, so the last
// link of a texture lookup's chain of dependent loads (material -> texel -> table) is
// an LDS read
#define YRT_SHADE_LDS_SRGB 1
#endif
#ifndef YRT_FOLD_PREFETCH
// mirror levels: the parent's fold records (D, la and its material's kr) are loaded at the
// top of k_shade, beside the sample's own surface, instead of after the shading, so their
// latency overlaps the light loop rather than following it
#define YRT_FOLD_PREFETCH 0
#endif
#ifndef YRT_SHADE_LEVEL_WAVES
// the same for the unfused k_shade (reflective scenes: per-level shading, mirror-ray
// compaction, the fold). Its waits are dependent loads (SQ_WAIT_ANY 76 % at 7 waves); more
// registers per wave shorten them (A/B at c3: shade 1.55 -> 1.35 / 1.34 ms at 6 / 5 waves)
#define YRT_SHADE_LEVEL_WAVES 5
#endif
template <bool COUNT, bool FUSE, int SB = WF_BLOCK, bool OCC4 = false>
__global__ __launch_bounds__(SB, FUSE ? YRT_SHADE_WAVES : YRT_SHADE_LEVEL_WAVES) void k_shade(dev_scene_view S, dev_render_args A, int level, int nsamp_level0,
                                                    int max_depth, wf_buffers B, unsigned long long* counters,
                                                    chunk_args C, float4* __restrict__ out) {
    __shared__ float4 fused_rad[FUSE ? SB : 1];
    __shared__ int cmp_count[SB / 64], cmp_base[SB / 64];
    __shared__ float srgb_lds[YRT_SHADE_LDS_SRGB ? 256 : 1];
    // (a scene without textures never looks the table up: it is not staged)
    const float* lut = YRT_SHADE_LDS_SRGB ? srgb_lds : S.srgb;
    if (YRT_SHADE_LDS_SRGB && S.ntextures > 0) {  // uniform over the grid
        for (int q = (int)threadIdx.x; q < 256; q += SB) srgb_lds[q] = S.srgb[q];
        __syncthreads();
    }
    work_counts wc;
    unsigned long long truncated = 0;
    const vec3f amb = {A.amb[0], A.amb[1], A.amb[2]};
    const vec3f cam_o = {A.cam.ox, A.cam.oy, A.cam.oz};
    // the loop bounds are uniform per block so every lane reaches the ballot and the
    // barriers below
    const int stride = gridDim.x * SB;
    // this block's mirror rays go to segment blockIdx.x % level_segments of the next level
    const int gout = (int)(blockIdx.x % (unsigned)level_segments);
    // (FUSE runs level 0 only: one segment, no loop)
    const int nseg = FUSE ? 1 : level ? level_segments : 1;
    for (int g = 0; g < nseg; g++) {
    const int n = (!FUSE && level) ? *seg_counter(B.count, level, g) : nsamp_level0;
    const int nround = (n + stride - 1) / stride;
    for (int round = 0; round < nround; round++) {
        const int j = round * stride + blockIdx.x * SB + threadIdx.x;
        const int idx = FUSE ? j : g * B.seg + j;
        bool spawn = false;
        vec3f p = {0, 0, 0}, dr = {0, 0, 0}, rec_d = {0, 0, 0}, rec_la = {0, 0, 0};
        int rec_mat = 0;
        if (j < n) {
            float4 s0 = ld4s(B.surf0 + idx);
            uint32_t occ_bits = 0;
            if constexpr (OCC4) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int lq = q < S.nlights ? q : 0;  // an unconditional load, masked after
                    const uint32_t ob = ldb(B.occl + (size_t)lq * B.capacity + idx);
                    occ_bits |= (q < S.nlights && ob != 0u) ? 1u << q : 0u;
                }
            }
            const int info = sample_state(s0);
            vec3f R = {0, 0, 0};
            bool write_r = info != -2;
            // level >= 1: this sample's ray record {origin, parent index}; with
            // YRT_FOLD_PREFETCH the parent's fold records are requested now
            const float4 ro4 = (!FUSE && level) ? ld4(B.ray_o(level) + idx) : make_float4(cam_o.x, cam_o.y, cam_o.z, 0.0f);
            float4 pd = {0, 0, 0, 0}, pla = {0, 0, 0, 0}, pkr = {0, 0, 0, 0};
            if (YRT_FOLD_PREFETCH && !FUSE && level) {
                const int parent = ibits(ro4.w);
                pd = ld4(B.rec0(level - 1) + parent), pla = ld4(B.rec1(level - 1) + parent);
                pkr = ld4(S.mats + 4 * ibits(pd.w) + 2);
            }
            if (info >= 0) {
                vec3f nrm;
                vec2f uv;
                int mat, kind;
                if (YRT_HIT16) {
                    const surface sf = hit16_surface(S, s0);
                    p = sf.p, nrm = sf.n, uv = sf.uv, mat = sf.mat, kind = sf.kind;
                } else {
                    const float4 s1 = ld4s(B.surf1 + idx);
                    p = xyz(s0), nrm = xyz(s1), uv = {s1.w, (!YRT_SKIP_UNUSED_V || B.need_v) ? lds1(B.surfv + idx) : 0.0f};
                    mat = info_mat(info), kind = info & 3;
                }
                const vec3f ro = xyz(ro4);
                float4 m0, m1, m2, m3;
                {
                    m0 = ld4(S.mats + 4 * mat), m1 = ld4(S.mats + 4 * mat + 1);
                    m2 = ld4(S.mats + 4 * mat + 2), m3 = ld4(S.mats + 4 * mat + 3);
                }
                const vec3f kd0 = xyz(m0), ks0 = xyz(m1), kr = xyz(m2);
                const float ns = m0.w;
                const int kd_txt = ibits(m1.w), ks_txt = ibits(m2.w);
                const bool reflective = ibits(m3.w) & mat_reflective;
                vec3f la = amb * kd0;
                vec3f tkd = {1, 1, 1}, tks = {1, 1, 1};
                if (kd_txt >= 0) {
                    tkd = eval_texture<COUNT>(S, kd_txt, uv, wc, lut);
                    la = la * tkd;
                }
                if (ks_txt >= 0) tks = eval_texture<COUNT>(S, ks_txt, uv, wc, lut);
                vec3f c = {0.0f, 0.0f, 0.0f};
                // raytrace.cpp:147 (per light) and :196 (mirror): the same value each time
                vec3f v;
                float vlen;
                normalize_len(ro - p, v, vlen);
                for (int li = 0; li < S.nlights; li++) {
                    if (OCC4 ? ((occ_bits >> li) & 1u) != 0u : ldb(B.occl + (size_t)li * B.capacity + idx) != 0) continue;
                    const f4* lr = S.lights + 6 * li;
                    // the light record is the same for every lane (li is the loop index):
                    // one scalar fetch instead of six 64-lane vector loads of one address
                    float4 lrec[6];
                    ld_scalar<6>(lr, lrec);
                    frame3f lf = {xyz(lrec[0]), xyz(lrec[1]), xyz(lrec[2]), xyz(lrec[3])};
                    vec3f lp0 = xyz(lrec[4]), ke = xyz(lrec[5]);
                    vec3f tp = transform_point(lf, lp0 - p);
                    vec3f l, h;
                    float r, hlen;
                    normalize_len(tp, l, r);
                    normalize_len(v + l, h, hlen);
                    vec3f kd = kd0, ks = ks0;
                    if (kd_txt >= 0) kd = kd * tkd;
                    if (ks_txt >= 0) ks = ks * tks;
                    const vec3f ker = div3(ke, r * r);
                    vec3f ld = kd * ker;
                    vec3f ls = ks * ker;
                    if (kind == kind_lines) {
                        float prodnl = dot(nrm, l);
                        float prodnh = dot(nrm, h);
                        if (prodnl < 0.0f) prodnl *= -1;
                        if (prodnh < 0.0f) prodnh *= -1;
                        float sinnl = __builtin_sqrtf(1.0f - prodnl);
                        float sinnh = __builtin_sqrtf(1.0f - prodnh);
                        ld = ld * sinnl;
                        ls = ls * spec_pow(sinnh, ns, ls);
                    } else {
                        ld = ld * smax(0.0f, dot(nrm, l));
                        ls = ls * spec_pow(smax(0.0f, dot(nrm, h)), ns, ls);
                    }
                    c = c + (ld + ls);
                }
                if (!reflective) {
                    R = c + la;
                } else if (FUSE || level + 1 >= max_depth || level + 1 >= B.nlevels) {
                    // (FUSE runs one-level renders: B.nlevels == 1, no mirror ray is spawned)
                    // depth cap: the reflected contribution counts as a miss (col = 0)
                    truncated++;
                    vec3f t = {0.0f * kr.x, 0.0f * kr.y, 0.0f * kr.z};
                    R = (c + t) + la;
                } else {
                    spawn = true;
                    dr = (nrm * 2.0f * dot(nrm, v)) - v;
                    rec_d = c;
                    rec_la = la;
                    rec_mat = mat;
                    write_r = false;
                }
                if (COUNT) wc.hits++;
            }
            if (FUSE) {
                fused_rad[threadIdx.x] = make_float4(R.x, R.y, R.z, 1.0f);
            } else if (write_r) {
                // a final value at level k >= 1 folds straight up its chain of parents
                // (raytrace.cpp:201-206, R_k-1 = (D + R_k * kr) + la, in that order) to
                // the camera sample; each parent has this one child, so its value is
                // final now too
                vec3f col = R;
                int lev = level, node = idx;
                while (lev > 0) {
                    const bool pre = YRT_FOLD_PREFETCH && lev == level;
                    const int parent = pre ? ibits(ro4.w) : ibits(B.ray_o(lev)[node].w);
                    const float4 d = pre ? pd : ld4(B.rec0(lev - 1) + parent);
                    const float4 la = pre ? pla : ld4(B.rec1(lev - 1) + parent);
                    const float4 kr = pre ? pkr : ld4(S.mats + 4 * ibits(d.w) + 2);  // the parent's material kr
                    vec3f cc = {d.x, d.y, d.z};
                    cc = cc + vec3f{col.x * kr.x, col.y * kr.y, col.z * kr.z};
                    cc = cc + xyz(la);
                    col = cc, node = parent, lev--;
                }
                B.rad[node] = {col.x, col.y, col.z, 1.0f};
            }
        }
        // compaction of the mirror rays (the fold follows parent indices, so the order is
        // free): a sample's own fold records go out at once; the block's mirror rays take
        // consecutive slots of its segment (waves in wave order, lanes in lane order)
        // behind one atomic per block. (One atomic per wave: c3 shade 1.99 -> 5.81 ms.)
        if constexpr (FUSE) continue;  // one level: no mirror rays
        const unsigned long long mask = __ballot(spawn);
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (spawn) {
            B.rec0(level)[idx] = {rec_d.x, rec_d.y, rec_d.z, __int_as_float(rec_mat)};
            B.rec1(level)[idx] = {rec_la.x, rec_la.y, rec_la.z, 0};
        }
        if (lane == 0) cmp_count[w] = __popcll(mask);
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int q = 0; q < SB / 64; q++) tot += cmp_count[q];
            int acc = tot ? atomicAdd(seg_counter(B.count, level + 1, gout), tot) : 0;
            for (int q = 0; q < SB / 64; q++) cmp_base[q] = acc, acc += cmp_count[q];
        }
        __syncthreads();
        if (spawn) {
            const int slot = gout * B.seg + cmp_base[w] + __popcll(mask & ((1ull << lane) - 1));
            B.ray_o(level + 1)[slot] = {p.x, p.y, p.z, __int_as_float(idx)};
            B.ray_d(level + 1)[slot] = {dr.x, dr.y, dr.z, 0};
        }
    }
    }
    if (FUSE) {
        // raytrace.cpp:232-249: s*s samples of a pixel summed in jj/ii order, then / s*s
        __syncthreads();
        const int ppb = SB / C.spp;
        // one lane per (pixel, colour component): each lane's sum is the reference's ordered
        // chain of adds (raytrace.cpp:232-249) for that component, so a pixel's three
        // dependent chains run side by side (A/B: c4 shade 2.00 -> 1.96 ms)
        for (int t = (int)threadIdx.x; t < 3 * ppb; t += SB) {
            const int px = t / 3, comp = t - 3 * px;
            const int pl = (int)(blockIdx.x * SB / C.spp) + px;
            int lx, ly, i, j;
            const bool valid = pl < C.npix && pixel_of(A, C.tiles_x, C.pix0 + pl, lx, ly, i, j);
            if (pl < C.npix && lx < A.tile_w && ly < A.tile_h) {
                float v = 0.0f;
                if (valid) {
                    const float* r = reinterpret_cast<const float*>(fused_rad + px * C.spp) + comp;
                    float acc = 0.0f;
                    for (int q = 0; q < C.spp; q++) acc = acc + r[4 * q];
                    v = acc / float(C.spp);
                }
                float* o = reinterpret_cast<float*>(out + (size_t)ly * A.out_stride + lx);
                o[comp] = v;
                if (comp == 0) o[3] = valid ? 1.0f : 0.0f;
            }
        }
    }
    flush(counters, cnt_depth_truncated, truncated);
    if (COUNT) flush_work(counters, wc);
}

// ---- ordered per-pixel sum (raytrace.cpp:232-249) ----
// A wave sums 64 pixels. Their samples are consecutive in memory (spp per pixel), so the
// wave stages them through LDS AQ samples of every pixel at a time with loads in which
// neighbouring lanes read neighbouring samples (a pixel's AQ samples are one contiguous
// run), then each lane adds its own pixel's samples in the reference's order.
constexpr int AQ = 8;
__global__ __launch_bounds__(WF_BLOCK) void k_accumulate(dev_render_args A, chunk_args C, wf_buffers B,
                                                         float4* __restrict__ out) {
    __shared__ float4 stage[WF_BLOCK / 64][64 * (AQ + 1)];  // rows padded against bank conflicts
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int pl0 = blockIdx.x * WF_BLOCK + w * 64;
    const int np = max(0, min(64, C.npix - pl0));  // pixels of this wave
    float4* S = stage[w];
    const f4* base = B.rad + (size_t)pl0 * C.spp;
    vec4f acc = {0, 0, 0, 0};
    for (int q0 = 0; q0 < C.spp; q0 += AQ) {  // the same trip count in every wave of the block
        const int qn = min(AQ, C.spp - q0);
        for (int e = lane; e < np * qn; e += 64) {
            const int px = e / qn, q = e % qn;
            S[px * (AQ + 1) + q] = ld4(base + (size_t)px * C.spp + q0 + q);
        }
        __syncthreads();
        if (lane < np)
            for (int q = 0; q < qn; q++) {
                const float4 c = S[lane * (AQ + 1) + q];
                acc = {acc.x + c.x, acc.y + c.y, acc.z + c.z, acc.w + 1.0f};
            }
        __syncthreads();
    }
    if (lane >= np) return;
    const int pl = pl0 + lane;
    int lx, ly, i, j;
    const bool valid = pixel_of(A, C.tiles_x, C.pix0 + pl, lx, ly, i, j);
    if (lx >= A.tile_w || ly >= A.tile_h) return;
    const float d = float(C.spp);
    out[(size_t)ly * A.out_stride + lx] =
        valid ? make_float4(acc.x / d, acc.y / d, acc.z / d, 1.0f) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// the per-level, per-segment mirror-ray counters (seg_counter)
size_t count_bytes(int nlevels) { return sizeof(int) * ((size_t)nlevels + 1) * level_segments * count_stride; }

// shadow bundles: items (64-sample blocks) and bundles of a chunk of cap samples
size_t bundle_items(int cap) { return ((size_t)cap + 63) / 64; }
size_t bundle_count(int cap) { return (bundle_items(cap) + bundle_g - 1) / bundle_g; }
int bundle_lights(int nlights) { return nlights <= bundle_max_lights ? nlights : 0; }
size_t super_count(int cap) { return (bundle_count(cap) + super_bundles - 1) / super_bundles; }

// camera lists: 8x8-pixel tiles of a chunk of cap samples at spp samples per pixel
size_t camera_tiles(int cap, int spp) { return ((size_t)cap / (size_t)spp + TILE * TILE - 1) / (TILE * TILE); }

size_t workspace_bytes(int cap, int spp, int nlights, int nlevels) {
    size_t c = (size_t)cap;
    size_t b = align_up(count_bytes(nlevels)) + align_up(32 * sizeof(unsigned)) +
               align_up(list_sums * sizeof(unsigned long long));
    b += align_up(16 * c) * 2 + align_up(4 * c) + align_up(c * std::max(nlights, 1)) + align_up(16 * c);
    if (YRT_SHADOW_BUNDLES) {
        const size_t gl = bundle_count(cap) * bundle_lights(nlights);
        b += align_up(32 * bundle_items(cap)) + 2 * align_up(4 * gl) +
             align_up((size_t)bundle_recs * wide_record_bytes * gl);
        if (YRT_BUNDLE_SUPER) b += align_up(super_count(cap) * bundle_lights(nlights) * super_list_f4 * 16);
    }
    if (YRT_CAMERA_LISTS) {
        const size_t nt = camera_tiles(cap, spp);
        b += 2 * align_up(4 * nt) + align_up(nt * camera_list_max * 32);
    }
    // levels >= 1: ray_o, ray_d; levels < last: rec0, rec1 (one slab each)
    if (nlevels > 1) b += 4 * align_up((size_t)(nlevels - 1) * 16 * c);
    return b;
}

wf_buffers carve(void* base, int cap, int spp, int nlights, int nlevels) {
    wf_buffers B = {};
    char* p = (char*)base;
    size_t c = (size_t)cap;
    auto take = [&](size_t bytes) {
        char* q = p;
        p += align_up(bytes);
        return (void*)q;
    };
    B.count = (int*)take(count_bytes(nlevels));
    B.queue = (unsigned*)take(32 * sizeof(unsigned));
    B.lstats = (unsigned long long*)take(list_sums * sizeof(unsigned long long));
    B.surf0 = (f4*)take(16 * c);
    B.surf1 = (f4*)take(16 * c);
    B.surfv = (float*)take(4 * c);
    B.occl = (unsigned char*)take(c * std::max(nlights, 1));
    B.rad = (f4*)take(16 * c);
    if (YRT_SHADOW_BUNDLES) {
        const size_t gl = bundle_count(cap) * bundle_lights(nlights);
        B.pbox = (f4*)take(32 * bundle_items(cap));
        B.lcount = (int*)take(4 * gl);
        B.lskip = (int*)take(4 * gl);
        B.lists = (f4*)take((size_t)bundle_recs * wide_record_bytes * gl);
        if (YRT_BUNDLE_SUPER) B.slists = (f4*)take(super_count(cap) * bundle_lights(nlights) * super_list_f4 * 16);
    }
    if (YRT_CAMERA_LISTS) {
        const size_t nt = camera_tiles(cap, spp);
        B.ccount = (int*)take(4 * nt);
        B.cskip = (int*)take(4 * nt);
        B.clist = (f4*)take(nt * camera_list_max * 32);
    }
    if (nlevels > 1) {
        const size_t slab = (size_t)(nlevels - 1) * 16 * c;
        B.ray_o_ = (f4*)take(slab);
        B.ray_d_ = (f4*)take(slab);
        B.rec0_ = (f4*)take(slab);
        B.rec1_ = (f4*)take(slab);
    }
    B.capacity = cap;
    B.nlevels = nlevels;
    return B;
}

template <bool COUNT, bool PACKET, typename SE>
hipError_t run(device_scene& ds, const dev_render_args& A, float4* out, unsigned long long* counters,
               hipStream_t stream) {
    const int spp = A.samples * A.samples;
    const int tiles_x = (A.tile_w + TILE - 1) / TILE;
    const int tiles_y = (A.tile_h + TILE - 1) / TILE;
    const long long npix_total = (long long)tiles_x * tiles_y * TILE * TILE;
    // one level per trace_first call a camera sample may make (A.max_depth; the reference
    // recursion is unbounded, so the caller's depth is kept as given)
    const int nlevels = ds.reflective ? std::max(A.max_depth, 1) : 1;
    // samples per chunk: a whole frame at c3/c4, 15 chunks at c5. A reflective scene keeps
    // per-level records for every level (64 B per sample and level). The chunk is halved
    // until the workspace takes at most half of the free HBM (deep mirror recursions run
    // as more, smaller chunks); a depth whose smallest chunk (2^16 samples) still does not
    // fit is refused.
    long long target = ds.reflective ? (1ll << 25) : (1ll << CHUNK_LOG2);
    auto cap_for = [&](long long tgt) {
        int pix = (int)std::max<long long>(1, std::min<long long>(npix_total, tgt / spp));
        pix = ((pix + TILE * TILE - 1) / (TILE * TILE)) * TILE * TILE;
        return pix;
    };
    // slots per sample record: a chunk's samples, and with mirror levels a slack so that
    // every segment of a level holds whatever k_shade's blocks of that segment spawn: at
    // level 0 one round of 256-sample blocks puts at most cap / 8 + 256 rays into a
    // segment, at later levels (a grid-stride grid of 2048 blocks over up to 8 input
    // segments) at most cap / 8 + 8 * 256
    auto seg_of = [&](int pix) { return pix * spp / level_segments + level_segments * WF_BLOCK; };
    auto cap_of = [&](int pix) { return nlevels > 1 ? level_segments * seg_of(pix) : pix * spp; };
    auto bytes_of = [&](long long tgt) { return workspace_bytes(cap_of(cap_for(tgt)), spp, ds.nlights, nlevels); };
    // the free-memory query (a driver round trip) only when the workspace must grow: a
    // steady frame loop reuses the workspace it already has
    if (bytes_of(target) > ds.work_bytes) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
        free_b += ds.work_bytes;  // the current workspace is given back if it is regrown
        while (target > (1ll << 16) && bytes_of(target) > free_b / 2) target /= 2;
        if (bytes_of(target) > free_b)
            throw unsupported_error("max_depth " + std::to_string(A.max_depth) + " needs " +
                                    std::to_string(bytes_of(target) >> 20) + " MiB of mirror-level records for its " +
                                    "smallest chunk; " + std::to_string(free_b >> 20) + " MiB of HBM are free");
    }
    const int pix_per_chunk = cap_for(target);
    const int seg = seg_of(pix_per_chunk);
    const int cap = cap_of(pix_per_chunk);
    const size_t need = workspace_bytes(cap, spp, ds.nlights, nlevels);
    if (need > ds.work_bytes) {
        if (ds.work) (void)hipFree(ds.work);
        ds.work = nullptr;
        ds.work_bytes = 0;
        hipError_t e = hipMalloc(&ds.work, need);
        if (e != hipSuccess) return e;
        ds.work_bytes = need;
    }
    wf_buffers B = carve(ds.work, cap, spp, ds.nlights, nlevels);
    B.trel = ds.trel;
    B.seg = seg;
    B.need_v = ds.view.ntextures > 0;
    bool list_stats = false;
    ds.last_camera_lists = ds.last_bundles = false;
    if (!ds.list_stats_host) {
        // the sums of the last render that built lists (behind list_stats_ev)
        hipError_t e =
            hipHostMalloc((void**)&ds.list_stats_host, list_sums * sizeof(unsigned long long), hipHostMallocDefault);
        if (e != hipSuccess) return e;
        memset(ds.list_stats_host, 0, list_sums * sizeof(unsigned long long));
    }
    if (!ds.list_stats_ev) {
        hipError_t e = hipEventCreateWithFlags(&ds.list_stats_ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    if (nlevels > 1 && !ds.level_count_host) {
        hipError_t e = hipHostMalloc((void**)&ds.level_count_host, sizeof(int) * level_segments * count_stride,
                                     hipHostMallocDefault);
        if (e != hipSuccess) return e;
    }
    if (nlevels > 1 && !ds.level_count_ev) {
        hipError_t e = hipEventCreateWithFlags(&ds.level_count_ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    phase_timer& T = ds.timer;
    // LDS staging of the instance tree's top (yrt_scene_set_lds_staging): the persistent walks
    // read it from LDS; the tile lists, whose walks start below it, are not built
    const bool stage = ds.lds_staging != 0 && !COUNT && PACKET;
    ds.last_lds_staging = 0;
    const float4 cam4 = make_float4(A.cam.ox, A.cam.oy, A.cam.oz, 0.0f);
    const int stride_grid = 2048;  // grid-stride kernels: 8 blocks of 256 per CU
    // one level and whole pixels per block: shade sums the pixels itself (k_shade FUSE;
    // one-wave fused blocks lose: +9 %)
    const bool fuse = nlevels == 1 && WF_BLOCK % spp == 0;
    if (npix_total == 0 && counters) {  // (no chunk, so no k_chunk_setup: the counters still start at 0)
        hipError_t e = hipMemsetAsync(counters, 0, (size_t)cnt_slots * cnt_count * sizeof(unsigned long long), stream);
        if (e != hipSuccess) return e;
    }
    for (long long pix0 = 0; pix0 < npix_total; pix0 += pix_per_chunk) {
        chunk_args C = {pix0, (int)std::min<long long>(pix_per_chunk, npix_total - pix0), spp, tiles_x};
        const int nsamp = C.npix * spp;
        const int grid = (nsamp + WF_BLOCK - 1) / WF_BLOCK;
        constexpr int TB = shadow_block<PACKET>();
        const int tgrid = (nsamp + TB - 1) / TB;
        // level 0's shadow rays run on the persistent any-hit grid (k_shadow_persist) -- on
        // any frame size when the caller forces the lists on (the bundles live there)
        const bool shadow_persist = !COUNT && PACKET && ds.wide_ok && TB == 64 && ds.nlights > 0 &&
                                    ((long long)tgrid * ds.nlights >= YRT_SHADOW_PERSIST_MIN_ITEMS ||
                                     ds.lists_mode == 1 || stage);
        // ... and walk the bundles' candidate lists (k_bundle_lists) instead of the tree
        const bool bundles_possible = YRT_SHADOW_BUNDLES && !stage && shadow_persist &&
                                      bundle_lights(ds.nlights) > 0 && ds.view.nwtop >= YRT_BUNDLE_MIN_TOP;
        // the camera rays walk their tiles' leaf lists (k_camera_lists)
        const bool cam_lists_possible = YRT_CAMERA_LISTS && YRT_PRIMARY_REL && !stage && !COUNT && PACKET && ds.wide_ok &&
                                        ds.view.nwtop >= YRT_BUNDLE_MIN_TOP;
        // YRT_LISTS_ON: whenever the scene allows; YRT_LISTS_AUTO: the same from
        // YRT_LISTS_MIN_SPP samples per pixel; _OFF: never (yrt_scene_set_tile_lists)
        const bool lists = ds.lists_mode == 1 || (ds.lists_mode == 0 && spp >= YRT_LISTS_MIN_SPP);
        B.cam_lists = cam_lists_possible && lists;
        B.bundles = bundles_possible && lists;
        ds.last_camera_lists |= B.cam_lists != 0, ds.last_bundles |= B.bundles != 0;
        const bool zero_lstats = (B.cam_lists || B.bundles) && !list_stats;
        list_stats |= zero_lstats;
        int t = T.begin(phase_lists, stream);
        {
            // the chunk's setup (k_chunk_setup): the camera-relative instance-level records of
            // this render (the first chunk of a packet render; timed in the lists phase,
            // YRT_PHASE_LISTS, with the camera lists built from them) and the chunk's zeroed
            // counters
            const int nrec = (PACKET && pix0 == 0) ? (int)ds.ntnodes * 2 * spine_len : 0;
            const int count_ints = nlevels > 1 ? (int)(count_bytes(nlevels) / sizeof(int)) : 0;
            const int counter_words = pix0 == 0 && counters ? cnt_slots * cnt_count : 0;
            const int work = std::max(std::max(nrec, count_ints), std::max(counter_words, 32));
            const int nb = std::min((work + WF_BLOCK - 1) / WF_BLOCK, 1024);
            hipLaunchKernelGGL(k_chunk_setup, dim3(nb), dim3(WF_BLOCK), 0, stream, nrec ? ds.view.tpair : nullptr,
                               nrec, A.cam.ox, A.cam.oy, A.cam.oz, ds.trel, B.queue,
                               zero_lstats ? B.lstats : nullptr, B.count, count_ints, counters, counter_words);
        }
        if (B.cam_lists) {
            const int nt = C.npix / (TILE * TILE);
            hipLaunchKernelGGL(k_camera_lists, dim3((nt + 3) / 4), dim3(256), 0, stream, ds.view, A, C, B);
        }
        T.end(t, stream);
        t = T.begin(phase_primary, stream);
        bool persist = false;
        if constexpr (!COUNT && PACKET) {
            persist = ((long long)nsamp + 63) / 64 >= (long long)YRT_PRIMARY_PERSIST_MIN_ITEMS;
            if (persist) {  // (its work counters B.queue[16, 25) were zeroed by k_chunk_setup)
                const int nb = ds.num_cus * (YRT_PRIMARY_WAVES * 4 * 64 / YRT_PRIMARY_SP_BLOCK);
                if (B.cam_lists)
                    hipLaunchKernelGGL((k_primary_persist<SE, 0, true>), dim3(nb), dim3(YRT_PRIMARY_SP_BLOCK), 0,
                                       stream, ds.view, A, C, B, counters);
                else if (stage && YRT_PRIMARY_REL) {
                    hipLaunchKernelGGL((k_primary_persist<SE, YRT_PRIMARY_LDS_RECORDS, false>), dim3(nb),
                                       dim3(YRT_PRIMARY_SP_BLOCK), 0, stream, ds.view, A, C, B, counters);
                    ds.last_lds_staging |= 1;
                } else
                    hipLaunchKernelGGL((k_primary_persist<SE, 0, false>), dim3(nb), dim3(YRT_PRIMARY_SP_BLOCK), 0,
                                       stream, ds.view, A, C, B, counters);
            }
        }
        if (!persist) {
            const dim3 pg((nsamp + YRT_PRIMARY_BLOCK - 1) / YRT_PRIMARY_BLOCK);
            if (B.cam_lists)
                hipLaunchKernelGGL((k_primary<COUNT, PACKET, SE, true>), pg, dim3(YRT_PRIMARY_BLOCK), 0, stream, ds.view,
                                   A, C, B, counters);
            else
                hipLaunchKernelGGL((k_primary<COUNT, PACKET, SE, false>), pg, dim3(YRT_PRIMARY_BLOCK), 0, stream,
                                   ds.view, A, C, B, counters);
        }
        T.end(t, stream);
        // levels run: a level with no mirror rays ends the chunk's recursion. The host
        // reads each level's ray count (written by the previous level's k_shade) without
        // draining the stream: the level's k_bounce, which takes its count on the device,
        // is queued first, so the GPU works on it while the count comes back; only a
        // level that turns out empty costs a launch (one k_bounce of no rays)
        for (int level = 0; level < nlevels; level++) {
            if (level > 0) {
                t = T.begin(phase_bounce, stream);
                hipLaunchKernelGGL((k_bounce<COUNT, PACKET, SE>), dim3(stride_grid), dim3(WF_BLOCK), 0, stream, ds.view,
                                   level, B, counters);
                T.end(t, stream);
                hipError_t e = hipEventSynchronize(ds.level_count_ev);
                if (e != hipSuccess) return e;
                bool any = false;
                for (int g = 0; g < level_segments; g++) any |= ds.level_count_host[g * count_stride] != 0;
                if (!any) break;
            }
            if (ds.nlights > 0) {
                dim3 sg(level ? stride_grid * WF_BLOCK / TB : tgrid, ds.nlights);
                if (level == 0 && shadow_persist && B.bundles) {  // the bundles' candidate lists
                    t = T.begin(phase_lists, stream);
                    if (YRT_BUNDLE_FUSED && YRT_BUNDLE_SUPER && bundle_g * super_bundles <= 256) {
                        const long long ns = (long long)super_count(nsamp) * ds.nlights;
                        hipLaunchKernelGGL(k_bundle_lists<true>, dim3((unsigned)ns), dim3(256), 0, stream, ds.view, B,
                                           tgrid);
                    } else {
                        if (YRT_BUNDLE_SUPER) {
                            const long long ns = (long long)super_count(nsamp) * ds.nlights;
                            hipLaunchKernelGGL(k_bundle_super, dim3((unsigned)((ns + 3) / 4)), dim3(256), 0, stream,
                                               ds.view, B, tgrid);
                        }
                        const long long nw = (long long)bundle_count(nsamp) * ds.nlights;
                        hipLaunchKernelGGL(k_bundle_lists<false>, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, stream,
                                           ds.view, B, tgrid);
                    }
                    T.end(t, stream);
                }
                t = T.begin(phase_shadow, stream);
                // level 0 only: at c3 the mirror levels' compacted samples trace faster with the
                // hardware's dealing (shadow 1.64 -> 1.72 ms with them persistent)
                if (level == 0 && shadow_persist) {
                    // one resident grid: two 1024-thread blocks per CU (8 waves per SIMD)
                    // (its work counters B.queue[0, 9) were zeroed by k_chunk_setup)
                    const int nb = ds.num_cus * (YRT_SHADOW_WAVES * 4 * 64 / SP_BLOCK);
                    constexpr int L = YRT_SHADOW_LDS_RECORDS;
                    if (stage && L > 0 && ds.view.nwtop >= L) {  // (the copy reads L whole records)
                        hipLaunchKernelGGL((k_shadow_persist<L>), dim3(nb), dim3(SP_BLOCK), 0, stream, ds.view,
                                           nsamp, tgrid, B, counters, cam4);
                        ds.last_lds_staging |= 2;
                    } else
                        hipLaunchKernelGGL((k_shadow_persist<0>), dim3(nb), dim3(SP_BLOCK), 0, stream, ds.view,
                                           nsamp, tgrid, B, counters, cam4);
                } else if (!COUNT && PACKET && ds.wide_ok)
                    hipLaunchKernelGGL((k_shadow<COUNT, PACKET, SE, true>), sg, dim3(TB), 0,
                                       stream, ds.view, level, nsamp, B, counters, cam4);
                else
                    hipLaunchKernelGGL((k_shadow<COUNT, PACKET, SE, false>), sg, dim3(TB), 0,
                                       stream, ds.view, level, nsamp, B, counters, cam4);
                T.end(t, stream);
            }
            t = T.begin(phase_shade, stream);
            const bool occ4 = ds.nlights <= 4;
#define YRT_SHADE_LAUNCH(FU, SBV, GRID)                                                                          \
    do {                                                                                                        \
        if (occ4)                                                                                               \
            hipLaunchKernelGGL((k_shade<COUNT, FU, SBV, true>), GRID, dim3(SBV), 0, stream, ds.view, A, level, nsamp, \
                               A.max_depth, B, counters, C, out);                                               \
        else                                                                                                    \
            hipLaunchKernelGGL((k_shade<COUNT, FU, SBV, false>), GRID, dim3(SBV), 0, stream, ds.view, A, level,      \
                               nsamp, A.max_depth, B, counters, C, out);                                        \
    } while (0)
            if (fuse) {
                YRT_SHADE_LAUNCH(true, WF_BLOCK, dim3(grid));
            } else {
                YRT_SHADE_LAUNCH(false, WF_BLOCK, dim3(level ? stride_grid : grid));
            }
#undef YRT_SHADE_LAUNCH
            T.end(t, stream);
            if (level + 1 < nlevels) {
                hipError_t e = hipMemcpyAsync(ds.level_count_host,
                                              B.count + (size_t)(level + 1) * level_segments * count_stride,
                                              sizeof(int) * level_segments * count_stride, hipMemcpyDeviceToHost,
                                              stream);
                if (e == hipSuccess) e = hipEventRecord(ds.level_count_ev, stream);
                if (e != hipSuccess) return e;
            }
        }
        if (!fuse) {
            t = T.begin(phase_accumulate, stream);
            hipLaunchKernelGGL(k_accumulate, dim3((C.npix + WF_BLOCK - 1) / WF_BLOCK), dim3(WF_BLOCK), 0, stream, A,
                               C, B, out);
            T.end(t, stream);
        }
        if (B.cam_lists || B.bundles) {
            t = T.begin(phase_lists, stream);
            hipLaunchKernelGGL(k_list_stats, dim3(64), dim3(256), 0, stream, B, C.npix / (TILE * TILE),
                               (int)(bundle_count(nsamp) * (size_t)ds.nlights));
            T.end(t, stream);
        }
    }
    if (list_stats) {
        hipError_t e = hipMemcpyAsync(ds.list_stats_host, B.lstats, list_sums * sizeof(unsigned long long),
                                      hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipEventRecord(ds.list_stats_ev, stream);
        if (e != hipSuccess) return e;
        ds.list_stats_recorded = true;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_render_wavefront(device_scene& ds, const dev_render_args& args, void* out_rgba,
                                   unsigned long long* counters, bool count_work, bool packet, hipStream_t stream) {
    if (args.tile_w <= 0 || args.tile_h <= 0) return hipSuccess;
    float4* out = (float4*)out_rgba;
    if (packet) {
        // the per-wave stack holds 32-bit node indices: no narrow/wide split needed
        return count_work ? run<true, true, uint32_t>(ds, args, out, counters, stream)
                          : run<false, true, uint32_t>(ds, args, out, counters, stream);
    }
    if (ds.narrow_stack)
        return count_work ? run<true, false, uint16_t>(ds, args, out, counters, stream)
                          : run<false, false, uint16_t>(ds, args, out, counters, stream);
    return count_work ? run<true, false, uint32_t>(ds, args, out, counters, stream)
                      : run<false, false, uint32_t>(ds, args, out, counters, stream);
}

}  // namespace yrt

#ifdef YRT_WIDE_STATS
extern "C" int yrt_debug_wide_stats(unsigned long long* out16, int reset) {
    static unsigned long long h[1024 * 16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(yrt::g_wide_stats), sizeof h) != hipSuccess) return -1;
    for (int i = 0; i < 16; i++) {
        out16[i] = 0;
        for (int k = 0; k < 1024; k++) out16[i] += h[16 * k + i];
    }
    if (reset) {
        static const unsigned long long z[1024 * 16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(yrt::g_wide_stats), z, sizeof z);
    }
    return 0;
}
#endif

#ifdef YRT_WIDE_STATS
extern "C" int yrt_debug_first_stats(unsigned long long* out16, int reset) {
    static unsigned long long h[1024 * 16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(yrt::g_first_stats), sizeof h) != hipSuccess) return -1;
    for (int i = 0; i < 16; i++) {
        out16[i] = 0;
        for (int k = 0; k < 1024; k++) out16[i] += h[16 * k + i];
    }
    if (reset) {
        static const unsigned long long z[1024 * 16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(yrt::g_first_stats), z, sizeof z);
    }
    return 0;
}
#endif

#ifdef YRT_LIST_TIMING
// out: n x {phase times..., size} of list builder k (0 k_camera_lists, 1 k_bundle_super,
// 2 k_bundle_lists), n <= 65536; reset: zero them afterwards
extern "C" int yrt_debug_list_time(unsigned long long* out, int k, int n, int reset) {
    if (k < 0 || k > 2 || n < 0 || n > 65536) return -1;
    const size_t off = (size_t)k * sizeof(yrt::g_list_time[0]);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(yrt::g_list_time), (size_t)n * 32, off) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long z[65536 * 4];
        (void)hipMemcpyToSymbol(HIP_SYMBOL(yrt::g_list_time), z, sizeof z, off);
    }
    return 0;
}
#endif

#ifdef YRT_TAIL_STATS
// out: 8192 x {start, end, items, xcd} for kernel k (0 k_primary_persist, 1 k_shadow_persist)
extern "C" int yrt_debug_tail(unsigned long long* out, int k) {
    if (k < 0 || k > 1) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(yrt::g_tail), sizeof(yrt::g_tail[0]), k * sizeof(yrt::g_tail[0])) ==
                   hipSuccess
               ? 0
               : -1;
}
#endif

#ifdef YRT_DEBUG_BOUNDS
extern "C" int yrt_debug_bounds(unsigned* out8, int reset) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(yrt::g_dbg_bounds), 8 * sizeof(unsigned)) != hipSuccess) return -1;
    if (reset) {
        unsigned z[8] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(yrt::g_dbg_bounds), z, sizeof z);
    }
    return 0;
}
#endif

