// packet_trace.h -- wave-coherent ("packet") traversal of the reference's two-level
// BVH: the 64 rays of a wave walk the tree together.
//
// Each stack entry is a node plus the mask of lanes that reached it (the lanes
// whose parent box test passed). Popping an entry, every lane of its mask tests
// the node's box with ITS OWN ray and current tmax; the lanes that pass continue
// into the node. The order of the walk is the reference's DFS order (pop; slab
// test; inner node pushes start then start+1, so start+1 is visited first;
// instance leaves enter their instances in slot order; shape leaves test their
// primitives in slot order), so every lane sees exactly the node tests, in exactly
// the order and with exactly the tmax, of intersect_bvh for its ray
// (src/scene.cpp:386-479) -- closest-hit tie-breaking included. Lanes only idle on
// nodes that other lanes of the wave need.
//
// One tmax per lane: the reference copies the world tmax into the local ray on
// instance entry and writes the shape's hit distance back when the shape returns
// (scene.cpp:468-471); nothing reads the world value in between, so keeping a
// single value is the same computation. A lane whose tmax became NaN (a NaN hit
// distance passes both range checks, and only a later hit in the SAME leaf can
// replace it) fails every later slab test in the reference: it leaves the walk when
// the leaf is done.
//
// Shaped for CDNA4's issue model (one scalar unit per CU, 64-wide VALU):
//  * everything that steers the walk is wave-uniform and lives in SGPRs: node
//    index, lane masks, stack pointer, instance range, shape root/kind;
//  * the stack lives in three VGPRs used as 64 lane-indexed slots (slot s = lane s):
//    a push is three v_writelane (packet_any: a compare + three selects), a pop three
//    v_readlane with the stack pointer as the lane index -- no LDS round trip, no
//    exec-masked store;
//  * every branch is on an SGPR value (no exec-mask divergence in the walk) and the
//    primitive tests are branchless (the reference's early returns become one
//    predicate);
//  * an instance record carries its shape's root node and primitive kind, so
//    entering an instance costs the four frame fetches and no dependent fetch.
// Rays of a wave are 64 samples of one pixel (or an 8x8 pixel tile), so the union
// of their paths is barely larger than one path.
//
// Contract: called by every lane of the wave in uniform control flow; lanes with
// valid == false take no part (they report no hit). Stack depth <= 64 (the host
// rejects scenes whose instance + shape BVH depth exceeds traversal_stack_cap).
#pragma once

#include "descent_asm.h"
#include "fast_div.h"
#include "wide_asm.h"
#include "trace_common.h"

namespace yrt {

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
// this lane's index, computed where it is used (two v_mbcnt) instead of being held in
// a VGPR across the walk -- under register pressure the compiler otherwise spills it
__device__ __forceinline__ int lane_now() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n v_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
// v_writelane_b32 (the LLVM intrinsic; clang has no builtin for it): value -> lane `lane`
// of `old`, every other lane kept; exec is ignored
extern "C" __device__ int yrt_llvm_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ int writelane(int old, int value, int lane) { return yrt_llvm_writelane(value, lane, old); }

// N consecutive 16-byte records at a wave-uniform address through the scalar data
// cache into SGPRs (s_load_dwordx4/x8/x16; the scene is read-only for the whole
// launch). The VALU reads them as scalar operands; nothing occupies the vector memory
// pipe, which a 64-lane load of one shared address would (1 KiB returned per record).
// Where one asm block issues two loads its outputs are early-clobber ("=&s"): the
// first load's destination must not share registers with the address the second one
// reads, or a quickly returning first load overwrites it (an intermittent fault).
typedef int sgpr4 __attribute__((ext_vector_type(4)));
typedef int sgpr8 __attribute__((ext_vector_type(8)));
typedef int sgpr16 __attribute__((ext_vector_type(16)));
template <typename V>
__device__ __forceinline__ float4 rec_of(const V& v, int k) {
    return {__int_as_float(v[4 * k]), __int_as_float(v[4 * k + 1]), __int_as_float(v[4 * k + 2]),
            __int_as_float(v[4 * k + 3])};
}
// the address as SGPRs (a no-op when the compiler already holds it there; where its
// uniformity analysis lost track, one v_readfirstlane per half)
__device__ __forceinline__ const f4* sgpr_ptr(const f4* p) {
    const unsigned long long a = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    return (const f4*)((unsigned long long)hi << 32 | lo);
}

template <int N>
__device__ __forceinline__ void ld_scalar(const f4* p_, float4 (&out)[N]) {
    static_assert(N == 3 || N == 4 || N == 6, "record count");
    const f4* p = sgpr_ptr(p_);
    if constexpr (N == 3) {
        sgpr8 a;
        sgpr4 b;
        asm volatile("s_load_dwordx8 %0, %2, 0x0\n s_load_dwordx4 %1, %2, 0x20\n s_waitcnt lgkmcnt(0)"
                     : "=&s"(a), "=&s"(b)
                     : "s"(p));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1), out[2] = rec_of(b, 0);
    } else if constexpr (N == 4) {
        sgpr16 a;
        asm volatile("s_load_dwordx16 %0, %1, 0x0\n s_waitcnt lgkmcnt(0)" : "=s"(a) : "s"(p));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1), out[2] = rec_of(a, 2), out[3] = rec_of(a, 3);
    } else {
        sgpr16 a;
        sgpr8 b;
        asm volatile("s_load_dwordx16 %0, %2, 0x0\n s_load_dwordx8 %1, %2, 0x40\n s_waitcnt lgkmcnt(0)"
                     : "=&s"(a), "=&s"(b)
                     : "s"(p));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1), out[2] = rec_of(a, 2), out[3] = rec_of(a, 3);
        out[4] = rec_of(b, 0), out[5] = rec_of(b, 1);
    }
}

// the same with the record index applied as an SGPR byte offset of the load itself
// (s_load ... sbase, soffset): one s_lshl instead of a 64-bit address computation
template <int N>
__device__ __forceinline__ void ld_scalar_at(const f4* base_, unsigned index, float4 (&out)[N]) {
    static_assert(N == 2 || N == 3 || N == 4 || N == 5 || N == 6, "record count");
    const f4* base = sgpr_ptr(base_);
    const unsigned off = (unsigned)__builtin_amdgcn_readfirstlane((int)(index * 16u));
    if constexpr (N == 2) {
        sgpr8 a;
        asm volatile("s_load_dwordx8 %0, %1, %2\n s_waitcnt lgkmcnt(0)" : "=s"(a) : "s"(base), "s"(off));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1);
    } else if constexpr (N == 3) {
        sgpr8 a;
        sgpr4 b;
        asm volatile("s_load_dwordx8 %0, %2, %3\n s_load_dwordx4 %1, %2, %3 offset:0x20\n s_waitcnt lgkmcnt(0)"
                     : "=&s"(a), "=&s"(b)
                     : "s"(base), "s"(off));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1), out[2] = rec_of(b, 0);
    } else if constexpr (N == 4) {
        sgpr16 a;
        asm volatile("s_load_dwordx16 %0, %1, %2\n s_waitcnt lgkmcnt(0)" : "=s"(a) : "s"(base), "s"(off));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1), out[2] = rec_of(a, 2), out[3] = rec_of(a, 3);
    } else if constexpr (N == 5) {
        sgpr16 a;
        sgpr4 b;
        asm volatile("s_load_dwordx16 %0, %2, %3\n s_load_dwordx4 %1, %2, %3 offset:0x40\n s_waitcnt lgkmcnt(0)"
                     : "=&s"(a), "=&s"(b)
                     : "s"(base), "s"(off));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1), out[2] = rec_of(a, 2), out[3] = rec_of(a, 3);
        out[4] = rec_of(b, 0);
    } else {
        sgpr16 a;
        sgpr8 b;
        asm volatile("s_load_dwordx16 %0, %2, %3\n s_load_dwordx8 %1, %2, %3 offset:0x40\n s_waitcnt lgkmcnt(0)"
                     : "=&s"(a), "=&s"(b)
                     : "s"(base), "s"(off));
        out[0] = rec_of(a, 0), out[1] = rec_of(a, 1), out[2] = rec_of(a, 2), out[3] = rec_of(a, 3);
        out[4] = rec_of(b, 0), out[5] = rec_of(b, 1);
    }
}

// N records at base + index (16-byte units)
template <int N>
__device__ __forceinline__ void ld_records_at(const f4* base, unsigned index, float4 (&out)[N]) {
    ld_scalar_at<N>(base, index, out);
}


// intersect_triangle (scene.cpp:229-263) without branches: the same values in the
// same order; the early returns become one predicate (a NaN w1/w2/t passes its
// range checks exactly as it does in the reference).
//
// `in`: the lanes whose result is used; `inm`: the same lanes as a wave mask. 1/den is the
// reference's IEEE division; with RCP, when every such lane has den and 1/den normal (a
// wave-uniform check), fast_div.h's rcp_nr gives the same bits in three instructions
// instead of ten. The test leaves early, wave-wide, after the first and after the second
// barycentric test when no lane that counts passes them (A/B: shadow -1.1 %, primary
// -0.8 % for the second exit). The exits use one ballot per compare -- the compare's own
// SGPR result -- and AND them on the scalar unit (a ballot of an AND of compares is
// materialised in a VGPR and compared back: v_cndmask + v_cmp per exit).
template <bool RCP = false>
__device__ __forceinline__ bool tri_hit_nb(vec3f o, vec3f d, float tmin, float tmax, vec3f v0, vec3f e1, vec3f e2,
                                           float& t, float& w1, float& w2, bool in, unsigned long long inm) {
    vec3f r = cross(d, e2);
    float den = dot(r, e1);
    float inv_den;
    if (!RCP || (ballot(!rcp_nr_ok(den)) & inm) != 0)
        inv_den = 1.0f / den;
    else
        inv_den = rcp_nr(den);
    vec3f c = o - v0;
    w1 = dot(r, c) * inv_den;
    // !(w1 < 0 || w1 > 1) == !(w1 < 0) && !(w1 > 1): a NaN passes both, as in the reference
    const unsigned long long m1 = inm & ballot(den != 0) & ballot(!(w1 < 0)) & ballot(!(w1 > 1));
    // no lane that counts passes the first barycentric test: the rest of the test (half of
    // it) cannot make any of them hit
    if (m1 == 0) {
        t = w2 = 0.0f;
        return false;
    }
    vec3f s = cross(c, e1);
    w2 = dot(s, d) * inv_den;
    if ((m1 & ballot(!(w2 < 0.0f)) & ballot(!(w1 + w2 > 1.0f))) == 0) {
        t = 0.0f;
        return false;
    }
    t = dot(s, e2) * inv_den;
    return (den != 0) & !(w1 < 0 || w1 > 1) & !(w2 < 0.0f || w1 + w2 > 1.0f) & !(t < tmin || t > tmax);
}

// tri_hit_nb as a wave mask: the lanes of `inm` whose ray hits, one ballot per compare ANDed
// on the scalar unit (no predicate materialised in a VGPR and compared back), 0 -- wave-
// uniform -- at the early exits. The caller turns the mask back into a per-lane condition with
// inverse_ballot (the mask used as the select's lane mask, no VALU).
template <bool RCP = false>
__device__ __forceinline__ unsigned long long tri_hit_mask(vec3f o, vec3f d, float tmin, float tmax, vec3f v0,
                                                           vec3f e1, vec3f e2, float& t, float& w1, float& w2,
                                                           unsigned long long inm) {
    vec3f r = cross(d, e2);
    float den = dot(r, e1);
    float inv_den;
    if (!RCP || (ballot(!rcp_nr_ok(den)) & inm) != 0)
        inv_den = 1.0f / den;
    else
        inv_den = rcp_nr(den);
    vec3f c = o - v0;
    w1 = dot(r, c) * inv_den;
    const unsigned long long m1 = inm & ballot(den != 0) & ballot(!(w1 < 0)) & ballot(!(w1 > 1));
    if (m1 == 0) {
        t = w2 = 0.0f;
        return 0;
    }
    vec3f s = cross(c, e1);
    w2 = dot(s, d) * inv_den;
    const unsigned long long m2 = m1 & ballot(!(w2 < 0.0f)) & ballot(!(w1 + w2 > 1.0f));
    if (m2 == 0) {
        t = 0.0f;
        return 0;
    }
    t = dot(s, e2) * inv_den;
    return m2 & ballot(!(t < tmin)) & ballot(!(t > tmax));
}
__device__ __forceinline__ bool lane_in(unsigned long long m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

// 1 / d per component (the slab test's invd, scene.cpp:372) as fast_div.h's rcp_nr when
// every lane of `lanes` has all three components in its range (bit-identical there), else
// the IEEE divisions
__device__ __forceinline__ vec3f rcp3(vec3f d, unsigned long long lanes) {
    if (!(ballot(!(rcp_nr_ok(d.x) && rcp_nr_ok(d.y) && rcp_nr_ok(d.z))) & lanes))
        return {rcp_nr(d.x), rcp_nr(d.y), rcp_nr(d.z)};
    return {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
}

// ---- any hit on the reference's binary BVH ----
// intersect_any (scene.cpp:489) as a packet walk: the instrumented (COUNT) pass, which
// counts the reference's own box/instance/primitive tests, and scenes too deep for the
// 4-wide walk's stack (device_scene wide_ok). The timed path is packet_occluded_wide2.
template <bool COUNT>
__device__ __forceinline__ bool packet_any(const dev_scene_view& S, const ray3& wray, bool valid, work_counts& wc) {
    const int lane = __lane_id();
    const unsigned long long me = 1ull << lane;
    // a NaN tmin/tmax fails every slab test of the reference: such a ray never enters a node
    const unsigned long long live = ballot(valid && !is_nan(wray.tmin) && !is_nan(wray.tmax));
    if (!live) return false;
    const vec3f wo = wray.o, wd = wray.d;
    const float tmin = wray.tmin, tmax = wray.tmax;
    // ray of the current level (local inside an instance); the world inverse direction
    // is recomputed when the walk leaves an instance leaf rather than kept live
    vec3f co = wo, cd = wd, ci = {1.0f / wd.x, 1.0f / wd.y, 1.0f / wd.z};
    // per-lane flags are kept as ints (VGPRs): a bool carried around the loop becomes
    // a 64-bit lane mask merged with exec on every back edge (scalar work per step)
    int hit = 0;
    // the stack: slot s of each of these VGPRs is lane s
    int stk_node = 0, stk_mlo = 0, stk_mhi = 0;
    unsigned long long done = 0;       // lanes out of the walk (a hit found)
    unsigned long long inst_mask = 0;  // lanes entering the current instance leaf
    int level = 0, sp = 0, base = 0, root = 0, kind = 0, inst_next = 0, inst_end = 0;
    int node = 0;
    // spine records of the current level (yrt_device.h tpair/spair): node X's record and
    // its child start+1's -- the nodes the reference tests back to back (test X; push
    // start; pop start+1 and test it) with no primitive test in between
    const f4* pbase = S.tpair;
    unsigned long long mask = live;
    for (;;) {
        node = uniform(node);  // keep the node index (and the address math) scalar
        float4 rec[2 * spine_len];
        ld_records_at<2 * spine_len>(pbase, (unsigned)(spine_record_f4 * node), rec);
        bool pass[spine_len];
#pragma unroll
        for (int j = 0; j < spine_len; j++) pass[j] = box_hit(co, ci, tmin, tmax, rec[2 * j], rec[2 * j + 1]);
        if (COUNT && lane == 0) wc.wnode++;
        // walk down the spine: node j is tested by the lanes that passed node j-1
        int lstart = 0;          // the leaf to process after this step, if any:
        uint32_t lcl = 0;        //   first slot, count | leaf_bit,
        unsigned long long lmask = 0;  //   lanes
        bool descend = false;
        unsigned long long mj = mask;
#pragma unroll
        for (int j = 0; j < spine_len; j++) {
            if (COUNT && (mj & me)) wc.box++;
            const unsigned long long pm = ballot(pass[j]) & mj;
            if (!pm) break;
            const int sw = uniform(ibits(rec[2 * j].w));
            const uint32_t cl = (uint32_t)uniform((int)ubits(rec[2 * j + 1].w));
            if (cl & leaf_bit) {
                lstart = sw, lcl = cl, lmask = pm;
                break;
            }
            const int start = sw / spine_record_bytes;  // inner: a record byte offset
            // push start (slot sp of the stack VGPRs := {start, pm}); the reference pops
            // start+1 next and tests it: that is spine node j+1
            const bool at = lane_now() == sp;
            stk_node = at ? start : stk_node;
            stk_mlo = at ? (int)(uint32_t)pm : stk_mlo;
            stk_mhi = at ? (int)(uint32_t)(pm >> 32) : stk_mhi;
            sp++;
            mj = pm;
            if (j == spine_len - 1) {
                node = start + 1;
                mask = pm;
                descend = true;
            }
        }
        if (descend) continue;
        if (lmask) {
            const int start = lstart;
            const int count = (int)(lcl & 0xffffu);
            if (level == 0) {
                inst_next = start;
                inst_end = start + count;
                inst_mask = lmask;
                level = 1;
                base = sp;
            } else {
                const bool in = (lmask >> lane) & 1;
                int leaf_hit = 0;
                for (int i = start; i < start + count; i++) {
                    float4 pv[3];
                    ld_scalar<3>(S.sprims + 3 * i, pv);
                    const float4 a = pv[0], b = pv[1], c = pv[2];
                    if (COUNT && in && !leaf_hit) wc.prim++;
                    if (COUNT && lane == 0) wc.wprim++;
                    float t, w1, w2;
                    bool h;
                    if (kind == kind_triangles) {
                        h = tri_hit_nb(co, cd, tmin, tmax, xyz(a), xyz(b), xyz(c), t, w1, w2, in, ballot(in));
                    } else {
                        vec4f ew;
                        const ray3 lr = {co, cd, tmin, tmax};
                        h = kind == kind_lines ? line_hit(lr, xyz(a), xyz(b), b.w, c.x, t, ew)
                                               : point_hit(lr, xyz(a), b.x, t, ew);
                    }
                    h = h && in;
                    leaf_hit |= h ? 1 : 0;
                }
                hit |= leaf_hit;
                // lanes with a hit are finished
                done |= ballot(leaf_hit);
                if (!(live & ~done)) return hit;
            }
        }
        // ---- next: the next instance of the current leaf, or pop ----
        for (;;) {
            if (level == 1 && sp == base) {
                if (inst_next < inst_end) {
                    // enter instance k: transform_ray_inverse (vmath.h:275-278), every lane
                    const int k = inst_next++;
                    float4 fr[4];
                    ld_scalar<4>(S.tinst + 4 * k, fr);
                    const float4 fx = fr[0], fy = fr[1], fz = fr[2], fo = fr[3];
                    const frame3f f = {xyz(fx), xyz(fy), xyz(fz), xyz(fo)};
                    co = transform_point_inverse(f, wo);
                    cd = transform_direction_inverse(f, wd);
                    ci = {1.0f / cd.x, 1.0f / cd.y, 1.0f / cd.z};
                    const uint32_t rk = (uint32_t)uniform(ibits(fo.w));
                    root = (int)(rk & 0x3fffffffu);
                    kind = (int)(rk >> 30);
                    pbase = S.spair + spine_record_f4 * root;
                    node = 0;  // the shape root, tested like any popped node
                    mask = inst_mask & ~done;
                    if (COUNT && (mask & me)) wc.inst++;
                    if (mask) break;
                    continue;
                }
                level = 0;
                pbase = S.tpair;
                co = wo;
                cd = wd;
                ci = {1.0f / wd.x, 1.0f / wd.y, 1.0f / wd.z};
            }
            if (sp == 0) return hit;
            sp--;
            node = __builtin_amdgcn_readlane(stk_node, sp);
            const uint32_t mlo = (uint32_t)__builtin_amdgcn_readlane(stk_mlo, sp);
            const uint32_t mhi = (uint32_t)__builtin_amdgcn_readlane(stk_mhi, sp);
            mask = ((unsigned long long)mhi << 32 | mlo) & ~done;
            if (mask) break;
        }
    }
}


#ifdef YRT_DEBUG_BOUNDS
// diagnostic build: the first out-of-range walk state is recorded here (no fault; the
// walk gives up): {code, a, b, c, d, e}
static __device__ unsigned g_dbg_bounds[8];
__device__ __forceinline__ bool dbg_fail(unsigned code, int a, int b, int c, int d, int e) {
    if ((__lane_id() == 0) && atomicCAS(&g_dbg_bounds[0], 0u, code) == 0u) {
        g_dbg_bounds[1] = a, g_dbg_bounds[2] = b, g_dbg_bounds[3] = c, g_dbg_bounds[4] = d, g_dbg_bounds[5] = e;
    }
    return true;
}
#define DBG_CHECK(cond, code, a, b, c, d, e) \
    if (!(cond) && dbg_fail(code, a, b, c, d, e)) return false
#else
#define DBG_CHECK(cond, code, a, b, c, d, e)
#endif

#ifdef YRT_WIDE_STATS
// diagnostic build: per-wave work of the wide any-hit walk, summed over 1024 spread
// lines of 16 counters: {walks, steps at the instance level, steps in shapes, instance
// entries, leaves reached in shapes, primitive tests, pops, empty pops, live lanes,
// occluded lanes, walks that end with every live lane occluded, their steps}
static __device__ unsigned long long g_wide_stats[1024 * 16];
// the closest-hit walk's (packet_first, timed instantiations): per walk {walks, list
// entries tested, spine records, instance entries, entries whose root record no lane passes,
// shape leaves, primitive tests, pops, live lanes, hit lanes}
static __device__ unsigned long long g_first_stats[1024 * 16];
#define WSTAT(i, v) (ws[i] += (v))
#else
#define WSTAT(i, v) ((void)0)
#endif

// the instance-local direction and its inverse on instance entry (transform_ray_inverse,
// vmath.h:275-278: the direction renormalized, invd = 1/d as intersect_check_bbox
// computes it).
//
// The four reciprocals (normalize's 1/l, vmath.h:118-122, and invd) are exact IEEE
// divisions in the reference. Here they are rcp_nr (fast_div.h: v_rcp_f32
// plus one Newton step, bit-identical to 1.0f / x on every input it admits -- checked on
// all 2^32 floats) whenever every live lane's l and cd components are in the normal range;
// otherwise (a zero, subnormal, huge, infinite or NaN value in some lane) the wave takes
// the division.
__device__ __forceinline__ void enter_direction(const frame3f& f, vec3f wd, unsigned long long lanes, vec3f& cd,
                                                vec3f& ci) {
    {
        const vec3f v = {dot(f.x, wd), dot(f.y, wd), dot(f.z, wd)};
        const float l2 = dot(v, v);  // length(v) = sqrt(dot(v, v))
        const float l = sqrt_nr(l2);  // normalize's sqrt; exact where sqrt_nr_ok (fast_div.h)
        const float y = rcp_nr(l);
        const vec3f c = v * y;
        const float lo = fminf(fminf(l, fabsf(c.x)), fminf(fabsf(c.y), fabsf(c.z)));
        const float hi = fmaxf(fmaxf(l, fabsf(c.x)), fmaxf(fabsf(c.y), fabsf(c.z)));
        // l == l: a NaN component makes l NaN (fminf/fmaxf would drop it)
        const bool fast = (l == l) && lo >= 0x1p-126f && hi < 0x1p126f && sqrt_nr_ok(l2);
        if (!(ballot(!fast) & lanes)) {
            cd = c;
            ci = {rcp_nr(c.x), rcp_nr(c.y), rcp_nr(c.z)};
            return;
        }
    }
    cd = transform_direction_inverse(f, wd);
    ci = {1.0f / cd.x, 1.0f / cd.y, 1.0f / cd.z};
}

// intersect_check_bbox (scene.cpp:371-382) with the per-axis swap decided at compile
// time: OCT bit a set = this lane's invd component a is < 0 (the reference's swap
// condition). The same two products per axis are computed -- (lo - o) * invd and
// (hi - o) * invd -- and each lands where the reference's swap puts it, so the values
// are bit-identical; OCT 8 is the run-time select of box_hit6.
template <int OCT>
__device__ __forceinline__ bool box_oct(vec3f o, vec3f invd, float tmin_r, float tmax_r, float lx, float ly, float lz,
                                        float hx, float hy, float hz) {
    if constexpr (OCT == 8) {
        float tn;
        return box_hit6(o, invd, tmin_r, tmax_r, lx, ly, lz, hx, hy, hz, tn);
    } else {
        const float nx = (OCT & 1) ? hx : lx, fx = (OCT & 1) ? lx : hx;
        const float ny = (OCT & 2) ? hy : ly, fy = (OCT & 2) ? ly : hy;
        const float nz = (OCT & 4) ? hz : lz, fz = (OCT & 4) ? lz : hz;
        const float t0x = (nx - o.x) * invd.x, t0y = (ny - o.y) * invd.y, t0z = (nz - o.z) * invd.z;
        const float t1x = (fx - o.x) * invd.x, t1y = (fy - o.y) * invd.y, t1z = (fz - o.z) * invd.z;
        float tmin = fmaxf(fmaxf(fmaxf(t0x, t0y), t0z), tmin_r);
        float tmax = fminf(fminf(fminf(t1x, t1y), t1z), tmax_r);
        tmax *= 1.00000024f;
        return tmin <= tmax;
    }
}

// the octant shared by every lane of `lanes` (bit a: invd component a < 0), or 8
__device__ __forceinline__ int wave_octant(vec3f invd, unsigned long long lanes) {
    const unsigned long long nx = ballot(invd.x < 0) & lanes, ny = ballot(invd.y < 0) & lanes,
                             nz = ballot(invd.z < 0) & lanes;
    if ((nx && nx != lanes) || (ny && ny != lanes) || (nz && nz != lanes)) return 8;
    return (nx ? 1 : 0) | (ny ? 2 : 0) | (nz ? 4 : 0);
}

#ifndef YRT_POP_ONE_EXIT
#define YRT_POP_ONE_EXIT 1
#endif
// pop inside a descent: entries above `floor` until one with live lanes (true), or down
// to the floor (false, mask 0) -- the level boundary is the caller's
__device__ __forceinline__ bool inner_pop(int floor, unsigned long long done, int& node, unsigned long long& mask,
                                          int& sp, int stk_node, int stk_mlo, int stk_mhi) {
#if YRT_POP_ONE_EXIT
    // one exit block: the loop leaves through the same edge whether it found live lanes or
    // reached the floor, and the empty asm hides m from the optimiser so that it cannot thread
    // the caller's test back into the loop (two exit blocks make the structurizer's
    // loop-exit unification route every descent step through a state variable)
    unsigned long long m = 0;
    while (sp > floor) {
        sp--;
        node = __builtin_amdgcn_readlane(stk_node, sp);
        m = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(stk_mhi, sp) << 32 |
             (uint32_t)__builtin_amdgcn_readlane(stk_mlo, sp)) &
            ~done;
        if (m) break;
    }
    m = (unsigned long long)(uint32_t)uniform((int)(m >> 32)) << 32 | (uint32_t)uniform((int)(uint32_t)m);
    asm volatile("" : "+s"(m));
    mask = m;
    return m != 0;
#else
    while (sp > floor) {
        sp--;
        node = __builtin_amdgcn_readlane(stk_node, sp);
        mask = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(stk_mhi, sp) << 32 |
                (uint32_t)__builtin_amdgcn_readlane(stk_mlo, sp)) &
               ~done;
        if (mask) return true;
    }
    mask = 0;
    return false;
#endif
}

// The closest hit's stack without lane masks (YRT_STACK_MASKS 0): an entry is the node
// alone, and a popped node is tested by every lane still walking this level (`avail`: the
// level's lanes -- the walk's live lanes at the instance level, the instance leaf's lanes
// in a shape -- less the done ones). A lane outside the entry's mask failed the box of an
// ancestor of that node in the same tree and space (or of the list entry above it), at a
// tmax no smaller than its current one; the node's box lies inside that ancestor's box,
// and a box test is monotone in the box and in tmax (NaN slabs included, trace_common.h
// box_hit6), so the lane fails the node too: the ballot, and with it the walk, is the
// same bit for bit. Per push one v_writelane instead of three, per pop one v_readlane
// instead of three and no mask AND; the counting pass (COUNT) keeps the masks, since it
// counts each lane's box tests. Inside a descent `avail` is never 0: the descent starts with
// a mask inside it (and done does not change until the leaf), so an entry above the floor
// always has lanes.
#ifndef YRT_STACK_MASKS
#define YRT_STACK_MASKS 0
#endif
// the any-hit walk's 4-wide descent as generated assembly (wide_asm.h); 0: the compiled loop
#ifndef YRT_WIDE_ASM
#define YRT_WIDE_ASM 1
#endif
// the maskless descent as generated assembly (descent_asm.h) in the camera rays' list-mode
// walk; 0: the compiled loop everywhere; 2: the assembly in every packet closest hit (equal
// time in the tree-mode kernels, more spills there)
#ifndef YRT_DESCENT_ASM
#define YRT_DESCENT_ASM 1
#endif
__device__ __forceinline__ bool inner_pop_avail(int floor, unsigned long long avail, int& node,
                                                unsigned long long& mask, int& sp, int stk_node) {
    // (one exit, the result hidden behind an empty asm: inner_pop's reason)
    unsigned long long m = 0;
    if (sp > floor) {
        sp--;
        node = __builtin_amdgcn_readlane(stk_node, sp);
        m = avail;
    }
    asm volatile("" : "+s"(m));
    mask = m;
    return m != 0;
}

constexpr int packet_block = 256;
#ifndef YRT_R5_LANE
#define YRT_R5_LANE 1
#endif
#ifndef YRT_R5_UORIG
#define YRT_R5_UORIG 1
#endif  // >= threads per block of every kernel that runs packet_first


// one descent of the closest-hit walk from the spine record at byte offset `node` of
// pbase: returns with mask = 0 when no lane passes, or with a leaf reached (mask: its
// lanes, node: its first slot, cl: count | leaf_bit). Per spine node: one ballot &
// mask, one leaf test, one push (v_writelane of the record offset and lane mask). A
// node no lane passes pops inside the descent (no re-dispatch of the octant copy).
//
// REL: the records' bounds are relative to the rays' common origin (every lane's ray starts
// at the one point the records were rewritten for, k_relative_records): the box test's
// (bound - o) is the record itself -- the same fp32 value, computed once per frame instead
// of once per test -- so the slab test is the three products per plane pair and the
// reference's min/max chains (x - 0.0f folds to x, bit for bit)
//
// LDSN > 0 (REL only): the first LDSN records of pbase are also in `lds` (staged per block by
// k_primary_persist, YRT_PRIMARY_LDS_RECORDS); a record below that offset is read with
// ds_read_b128 at a wave-uniform address instead of through the scalar cache
#ifndef YRT_DESCENT_ONE_EXIT
#define YRT_DESCENT_ONE_EXIT 1
#endif
#if YRT_DESCENT_ONE_EXIT
#define YRT_DESCENT_EXIT break
#else
#define YRT_DESCENT_EXIT return
#endif
//
// SM: the stack holds lane masks (`done`: the lanes that left the walk); without them
// (inner_pop_avail) `done` is the level's available lanes instead
template <int OCT, bool COUNT, bool REL = false, int LDSN = 0, bool SM = true, bool ASM = false>
__device__ __forceinline__ void first_descend(const f4* pbase, vec3f co, vec3f ci, float tmin, float tmax,
                                              unsigned long long me, int& node, unsigned long long& mask, int& sp,
                                              int& stk_node, int& stk_mlo, int& stk_mhi, uint32_t& cl,
                                              work_counts& wc, int floor, unsigned long long done,
                                              const float4* lds = nullptr) {
#if YRT_DESCENT_ASM && !defined(YRT_WIDE_STATS)
    // the same loop as one asm block (descent_asm.h, tools/gen_descent_asm.py). ASM: the camera
    // rays' list-mode walk only -- in the tree-mode kernels (k_bounce, the lists-off primary)
    // its fixed registers cost spills: c3 bounce 0.76 -> 0.82 ms, primary 1.04 -> 1.07
    if constexpr (ASM && !COUNT && !SM && LDSN == 0 && OCT < 8) {
        // (the "s" operands made wave-uniform first: folded away where the compiler knows them
        // to be in SGPRs, needed where its uniformity analysis lost track, as in YRT_DEBUG_BOUNDS)
        auto u64 = [](unsigned long long v) {
            return (unsigned long long)(uint32_t)uniform((int)(v >> 32)) << 32 | (uint32_t)uniform((int)(uint32_t)v);
        };
        node = uniform(node), sp = uniform(sp), mask = u64(mask), cl = (uint32_t)uniform((int)cl);
        descent_asm<OCT, REL>::run(sgpr_ptr(pbase), co, ci, tmin, tmax, uniform(floor), u64(done), node, mask, sp,
                                   stk_node, cl);
        sp = uniform(sp);
        mask = (unsigned long long)(uint32_t)uniform((int)(mask >> 32)) << 32 | (uint32_t)uniform((int)(uint32_t)mask);
        node = uniform(node);
        cl = (uint32_t)uniform((int)cl);
        asm volatile("" : "+s"(mask), "+s"(node), "+s"(cl));
        return;
    }
#endif
#define YRT_POP (SM ? inner_pop(floor, done, node, mask, sp, stk_node, stk_mlo, stk_mhi) \
                    : inner_pop_avail(floor, done, node, mask, sp, stk_node))
    const f4* pb = sgpr_ptr(pbase);  // once per descent, not per record (the compiler kept pbase in VGPRs)
    for (;;) {
        float4 rec[4];
        if (LDSN > 0 && (unsigned)node < (unsigned)(LDSN * spine_record_bytes)) {
            const float4* p = lds + ((unsigned)uniform(node) >> 4);
            rec[0] = p[0], rec[1] = p[1], rec[2] = p[2], rec[3] = p[3];
        } else {
            sgpr16 a;
            asm volatile("s_load_dwordx16 %0, %1, %2\n s_waitcnt lgkmcnt(0)"
                         : "=s"(a)
                         : "s"(pb), "s"(uniform(node)));
            rec[0] = rec_of(a, 0), rec[1] = rec_of(a, 1), rec[2] = rec_of(a, 2), rec[3] = rec_of(a, 3);
        }
        const vec3f bo = REL ? vec3f{0.0f, 0.0f, 0.0f} : co;
        const bool p0 = box_oct<OCT>(bo, ci, tmin, tmax, rec[0].x, rec[0].y, rec[0].z, rec[1].x, rec[1].y, rec[1].z);
        const bool p1 = box_oct<OCT>(bo, ci, tmin, tmax, rec[2].x, rec[2].y, rec[2].z, rec[3].x, rec[3].y, rec[3].z);
        if (COUNT && (me & 1)) wc.wnode++;
#ifdef YRT_WIDE_STATS
        if (!COUNT) {
            wc.wnode++;
            if (!REL && node == 0 && !(ballot(p0) & mask)) wc.wprim++;  // (a shape's root record, REL callers)
        }
#endif
        if (COUNT && (mask & me)) wc.box++;
        const unsigned long long pm0 = ballot(p0) & mask;
        mask = pm0;
        if (!pm0) {
            if (YRT_POP) continue;
            YRT_DESCENT_EXIT;
        }
        const int s0 = uniform(ibits(rec[0].w));
        const uint32_t c0 = (uint32_t)uniform(ibits(rec[1].w));
        if (c0 & leaf_bit) {
            node = s0, cl = c0;
            YRT_DESCENT_EXIT;
        }
        // push L (X's child start) for the lanes that passed X
        stk_node = writelane(stk_node, s0, sp);
        if constexpr (SM) {
            stk_mlo = writelane(stk_mlo, (int)(uint32_t)pm0, sp);
            stk_mhi = writelane(stk_mhi, (int)(uint32_t)(pm0 >> 32), sp);
        }
        sp++;
        if (COUNT && (pm0 & me)) wc.box++;
        const unsigned long long pm1 = ballot(p1) & pm0;
        mask = pm1;
        if (!pm1) {
            if (YRT_POP) continue;
            YRT_DESCENT_EXIT;
        }
        const int s1 = uniform(ibits(rec[2].w));
        const uint32_t c1 = (uint32_t)uniform(ibits(rec[3].w));
        if (c1 & leaf_bit) {
            node = s1, cl = c1;
            YRT_DESCENT_EXIT;
        }
        // push RL (R's child start)
        stk_node = writelane(stk_node, s1, sp);
        if constexpr (SM) {
            stk_mlo = writelane(stk_mlo, (int)(uint32_t)pm1, sp);
            stk_mhi = writelane(stk_mhi, (int)(uint32_t)(pm1 >> 32), sp);
        }
        sp++;
        node = s1 + spine_record_bytes;
    }
#undef YRT_POP
#if YRT_DESCENT_ONE_EXIT
    // every exit of the loop above arrives here; the empty asm makes the exit state opaque so
    // that the caller's tests on it (leaf reached or not) are not threaded back into the loop
    // as separate exit blocks
    // (readfirstlane first: folded away where the compiler knows the values are in SGPRs, and
    // the "s" constraints need them there where its uniformity analysis lost track, as in the
    // YRT_DEBUG_BOUNDS build)
    mask = (unsigned long long)(uint32_t)uniform((int)(mask >> 32)) << 32 | (uint32_t)uniform((int)(uint32_t)mask);
    node = uniform(node);
    cl = (uint32_t)uniform((int)cl);
    asm volatile("" : "+s"(mask), "+s"(node), "+s"(cl));
#endif
}
#undef YRT_DESCENT_EXIT

// ---- closest hit, laid out for the scalar unit ----
// The packet discipline of packet_any (same node tests, in the reference's order, with
// the same tmax per lane), with the control flow written so that the hot descent path
// carries no merged loop state: per spine node
// one s_and (ballot & mask, SCC = any lane), one leaf test and one stack push. The
// push is three v_writelane of the SGPR values into lane sp of the stack VGPRs (no
// lane-index compare, no selects). SALU issue -- one scalar unit per CU shared by
// its four SIMDs -- is what bounds the closest-hit kernels (SQ_INSTS_SALU per CU
// against the kernel's cycles), so every scalar instruction on the descent counts.
// BS: threads per block of the calling kernel (one LDS slot per thread for the parked 1/d)
// trel (REL): the instance-level spine records relative to the origin that every lane's
// ray shares (the camera's, for primary rays); the instance level is walked on them.
// LDSN/lds (REL): the first LDSN records of trel staged in LDS by the caller (first_descend).
//
// List mode (REL, ln >= 0): instead of walking the instance tree, the walk takes the ln
// leaves at lbase (wavefront.hip k_camera_lists: every instance-level leaf whose box a camera
// ray of this pixel tile can pass, boxes relative to the camera origin, in the reference's
// DFS order -- descending first slot, since the reference visits child start+1 before start
// and the builder gives start the lower half) and tests each leaf's box with every live lane
// at the lane's current tmax. That is the reference's computation: a leaf whose box passes
// at the current tmax has every ancestor pass at the earlier (larger) tmax the reference
// tested it with -- a box test is monotone in the box and in tmax -- so the reference reaches
// it and tests it with this same tmax (the hits before it in DFS order being the same); a
// leaf that fails, it either never reaches or tests and fails. Entries {lo - o, first}
// {hi - o, count} (32 bytes).
template <int OCT>
__device__ __forceinline__ unsigned long long list_entry_test(vec3f ci, float tmin, float tmax, const float4 (&e)[2],
                                                             unsigned long long lanes) {
    return ballot(box_oct<OCT>(vec3f{0.0f, 0.0f, 0.0f}, ci, tmin, tmax, e[0].x, e[0].y, e[0].z, e[1].x, e[1].y,
                               e[1].z)) &
           lanes;
}
// (LIST: the list mode is compiled in; without it the walk is the tree walk alone)
template <bool COUNT, int BS = packet_block, bool REL = false, int LDSN = 0, bool LIST = false>
__device__ __forceinline__ bool packet_first(const dev_scene_view& S, const ray3& wray, bool valid, hit_record& hr,
                                             work_counts& wc, const f4* trel = nullptr,
                                             const float4* lds = nullptr, const f4* lbase = nullptr,
                                             int ln = -1) {
    static_assert(spine_len == 2, "packet_first walks two-node spine records");
    // (this lane's bit, wave-relative LDS slot: recomputed where used -- lane_now() is not
    // hoisted out of a persistent caller's item loop, where a held copy would be spilled)
    const unsigned long long me = (COUNT || !YRT_R5_LANE) ? 1ull << __lane_id() : 0ull;
    const unsigned long long live = ballot(valid && !is_nan(wray.tmin) && !is_nan(wray.tmax));
    if (!live) return false;
    // REL: every live lane's ray starts at the one origin the records were made relative to
    // (the camera's): it is read from the first live lane into SGPRs, so the walk holds no
    // VGPRs for it
    const int fl = __builtin_ctzll(live);
    const vec3f wo = (REL && YRT_R5_UORIG) ? vec3f{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(wray.o.x), fl)),
                                 __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wray.o.y), fl)),
                                 __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wray.o.z), fl))}
                         : wray.o;
    const vec3f wd = wray.d;
    const float tmin = wray.tmin;
    float tmax = wray.tmax;
    vec3f co = wo, cd = wd, ci = rcp3(wd, live);
    // the world inverse direction, parked in LDS for the returns from instance leaves
    // (three ds_read instead of three IEEE divisions; three VGPRs stay free)
    __shared__ float wi_lds[3][BS];
    const int wave = uniform((int)threadIdx.x >> 6);
    {
        const int t = YRT_R5_LANE ? wave * 64 + lane_now() : (int)threadIdx.x;
        wi_lds[0][t] = ci.x, wi_lds[1][t] = ci.y, wi_lds[2][t] = ci.z;
    }
    float hw1 = 0, hw2 = 0;
    int hslot = -1, hei = -1;
    int stk_node = 0, stk_mlo = 0, stk_mhi = 0;
    // avail: the lanes still walking the current level -- the walk's live lanes at the
    // instance level, the instance leaf's lanes inside its instances -- less the done ones
    // (the lanes a popped node is tested with when the stack holds no masks, inner_pop_avail)
    unsigned long long done = 0, avail = live, mask = live;
    int level = 0, sp = 0, base = 0, kind = 0, inst_next = 0, inst_end = 0, cur_slot = -1;
    int node = 0;  // byte offset of the current spine record from pbase
    const f4* const ptop = REL ? trel : S.tpair;
    const f4* pbase = ptop;
    // the octant of the current level's rays when the whole wave shares it (8: mixed):
    // the descent runs the copy with its slab swaps resolved at compile time (box_oct)
    const int woct = wave_octant(ci, live);
    int oct = woct;
    // the instance-local direction of the instances with an identity rotation, once per
    // walk (packet_occluded_wide2 does the same)
    vec3f icd, ici;
    enter_direction(frame3f{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}}, wd, live, icd, ici);
    const int ioct = wave_octant(ici, live);
    // list mode (LIST, REL): level 0 is driven by the tile's frontier list (k_camera_lists):
    // its address, length and next entry are parked in this wave's LDS slot between list
    // steps, so they hold no registers through the walk; a wave without a list (ln < 0) walks
    // the tree from its root as the list's one virtual entry
    constexpr bool LM = LIST && REL && !COUNT;
    constexpr bool SM = COUNT || YRT_STACK_MASKS;  // the stack keeps lane masks (inner_pop_avail)
    __shared__ int list_lds[BS / 64][4];
    int* const lst = list_lds[wave];
    if constexpr (LM) {
        lst[0] = (int)(unsigned)(unsigned long long)lbase, lst[1] = (int)((unsigned long long)lbase >> 32);
        lst[2] = ln, lst[3] = 0;
    }
    bool lstep = LM;  // the next step takes the next list entry (the walk's first step, in list mode)
    for (;;) {
        uint32_t lcl = 0;
        bool descend = true;
        if (LM && lstep) {
            // ---- list step: the next entry some live lane passes, or the end of the walk ----
            lstep = false;
            mask = 0;
            asm volatile("" ::: "memory");
            const int lend = uniform(lst[2]);
            int lnext = uniform(lst[3]);
            if (lend < 0) {
                if (lnext == 0) node = 0, mask = live & ~done, lnext = 1;  // the root's record
            } else {
                const f4* lb =
                    (const f4*)((unsigned long long)(unsigned)uniform(lst[1]) << 32 | (unsigned)uniform(lst[0]));
                while (lnext < lend) {
                    float4 e[2];
                    ld_records_at<2>(lb, (unsigned)(2 * lnext), e);
                    lnext++;
#ifdef YRT_WIDE_STATS
                    wc.tex++;  // (stats build: list entries tested)
#endif
                    const unsigned long long lanes = live & ~done;
                    unsigned long long m;
                    switch (oct) {
                        case 0: m = list_entry_test<0>(ci, tmin, tmax, e, lanes); break;
                        case 1: m = list_entry_test<1>(ci, tmin, tmax, e, lanes); break;
                        case 2: m = list_entry_test<2>(ci, tmin, tmax, e, lanes); break;
                        case 3: m = list_entry_test<3>(ci, tmin, tmax, e, lanes); break;
                        case 4: m = list_entry_test<4>(ci, tmin, tmax, e, lanes); break;
                        case 5: m = list_entry_test<5>(ci, tmin, tmax, e, lanes); break;
                        case 6: m = list_entry_test<6>(ci, tmin, tmax, e, lanes); break;
                        case 7: m = list_entry_test<7>(ci, tmin, tmax, e, lanes); break;
                        default: m = list_entry_test<8>(ci, tmin, tmax, e, lanes); break;
                    }
                    if (m) {
                        const int w0 = uniform(ibits(e[0].w));
                        const uint32_t w1 = (uint32_t)uniform(ibits(e[1].w));
                        mask = m;
                        if (w1 & leaf_bit) {  // an instance-level leaf: its instances next
                            node = w0, lcl = w1;
                            descend = false;
                        } else {
                            // a subtree root X that the lanes of m pass: what first_descend does
                            // once X passes -- push X's child start (record w0) for them and go on
                            // at child start+1, whose record follows start's
                            stk_node = writelane(stk_node, w0, sp);
                            if constexpr (SM) {
                                stk_mlo = writelane(stk_mlo, (int)(uint32_t)m, sp);
                                stk_mhi = writelane(stk_mhi, (int)(uint32_t)(m >> 32), sp);
                            }
                            sp++;
                            node = w0 + spine_record_bytes;
                        }
                        break;
                    }
                }
            }
            if (!mask) break;
            lst[3] = lnext;
            asm volatile("" ::: "memory");
        }
        if (descend) {
        // ---- descent: one spine record per step, until a leaf or no passing lane ----
        DBG_CHECK(node >= 0 && (node % spine_record_bytes) == 0 && sp >= 0 && sp < 63 &&
                      (level == 0 ? node / spine_record_bytes < S.ntnodes
                                  : (int)((pbase - S.spair) / 4) + node / spine_record_bytes < S.nsnodes),
                  1, node, sp, level, (int)((pbase - S.spair) / 4), base);
        const int floor = level ? base : 0;
        // (without stack masks: the lanes a popped node is tested with, inner_pop_avail)
        const unsigned long long pop_arg = SM ? done : avail;
#define YRT_FD(o, R)                                                                                          \
    first_descend<o, COUNT, R, R ? LDSN : 0, SM, LM || YRT_DESCENT_ASM >= 2>(pbase, co, ci, tmin, tmax, me, node,  \
                                                                           mask, sp, stk_node,                 \
                                                stk_mlo, stk_mhi, lcl, wc, floor, pop_arg, lds)
        if (REL && level == 0) {
            switch (oct) {
                case 0: YRT_FD(0, REL); break;
                case 1: YRT_FD(1, REL); break;
                case 2: YRT_FD(2, REL); break;
                case 3: YRT_FD(3, REL); break;
                case 4: YRT_FD(4, REL); break;
                case 5: YRT_FD(5, REL); break;
                case 6: YRT_FD(6, REL); break;
                case 7: YRT_FD(7, REL); break;
                default: YRT_FD(8, REL); break;
            }
        } else {
            switch (oct) {
                case 0: YRT_FD(0, false); break;
                case 1: YRT_FD(1, false); break;
                case 2: YRT_FD(2, false); break;
                case 3: YRT_FD(3, false); break;
                case 4: YRT_FD(4, false); break;
                case 5: YRT_FD(5, false); break;
                case 6: YRT_FD(6, false); break;
                case 7: YRT_FD(7, false); break;
                default: YRT_FD(8, false); break;
            }
        }
#undef YRT_FD
        }
        const unsigned long long lmask = mask;
        const int lstart = node, lcount = (int)(lcl & 0xffffu);
        // ---- the leaf reached, if any ----
        if (lmask) {
            if (level == 0) {
                inst_next = lstart;
                inst_end = lstart + lcount;
                avail = lmask;
                if (LM) {
                    // a camera list's leaf: the instances its tile's cone excludes (bits 16-30
                    // of the count word, wavefront.hip k_camera_lists; a tree leaf's are 0).
                    // The runs of them at either end of the leaf are dropped here, once per
                    // leaf; one between kept instances is entered as before (its root box
                    // test fails for every lane). (Skipping those too, per entry, cost the
                    // closest hit more scalar work than it saved: c4 primary 9.42 -> 9.62 ms
                    // with a keep mask, instance100k +1 ms.)
                    const uint32_t skip = (lcl >> 16) & 0x7fffu;
                    if (skip) {
                        const uint32_t keep = ~skip & ((1u << lcount) - 1u);  // (count <= 15 when skip != 0)
                        if (!keep) {
                            inst_end = inst_next;
                        } else {
                            inst_next = lstart + __builtin_ctz(keep);
                            inst_end = lstart + 32 - __builtin_clz(keep);
                        }
                    }
                }
                level = 1;
                base = sp;
            } else {
                const bool in = lane_in(lmask);
                unsigned long long leaf_hits = 0;  // the lanes that hit a primitive of this leaf
                DBG_CHECK(lstart >= 0 && lstart + lcount <= S.nsprims, 2, lstart, lcount, level, kind, sp);
#ifdef YRT_WIDE_STATS
                if (!COUNT) wc.box++, wc.prim += (unsigned)lcount;  // (stats build: shape leaves, primitive tests)
#endif
                if (kind == kind_triangles) {
                    for (int i = lstart; i < lstart + lcount; i++) {
                        float4 pv[3];
                        ld_records_at<3>(S.sprims, (unsigned)(3 * i), pv);
                        if (COUNT && in) wc.prim++;
                        if (COUNT && (me & 1)) wc.wprim++;
                        float t, w1, w2;
                        const unsigned long long hm =
                            tri_hit_mask<true>(co, cd, tmin, tmax, xyz(pv[0]), xyz(pv[1]), xyz(pv[2]), t, w1, w2, lmask);
                        // most triangles hit no lane: their record-keeping selects are skipped
                        if (hm) {
                            const bool h = lane_in(hm);
                            tmax = h ? t : tmax;
                            hslot = h ? cur_slot : hslot;
                            hei = h ? ibits(pv[0].w) : hei;
                            hw1 = h ? w1 : hw1;
                            hw2 = h ? w2 : hw2;
                            leaf_hits |= hm;
                        }
                    }
                } else {
                    for (int i = lstart; i < lstart + lcount; i++) {
                        float4 pv[3];
                        ld_records_at<3>(S.sprims, (unsigned)(3 * i), pv);
                        if (COUNT && in) wc.prim++;
                        if (COUNT && (me & 1)) wc.wprim++;
                        // lines: ew = {1-s, s, 0, 0}; points: {1, 0, 0, 0} -- both are
                        // {1-w1-w2, w1, w2, 0} with w1 = ew.y, w2 = ew.z
                        float t;
                        vec4f ew;
                        const ray3 lr = {co, cd, tmin, tmax};
                        bool h = kind == kind_lines ? line_hit(lr, xyz(pv[0]), xyz(pv[1]), pv[1].w, pv[2].x, t, ew)
                                                    : point_hit(lr, xyz(pv[0]), pv[1].x, t, ew);
                        h = h && in;
                        tmax = h ? t : tmax;
                        hslot = h ? cur_slot : hslot;
                        hei = h ? ibits(pv[0].w) : hei;
                        hw1 = h ? ew.y : hw1;
                        hw2 = h ? ew.z : hw2;
                        leaf_hits |= ballot(h);
                    }
                }
                // a NaN tmax fails every later slab test: such a lane leaves the walk
                done |= leaf_hits & ballot(is_nan(tmax));
                avail &= ~done;
            }
        }
        // ---- the next node: the next instance of the current leaf, or a pop ----
        bool finished = false;
        for (;;) {
            if (level == 1 && sp == base) {
                if (inst_next < inst_end) {
                    // enter instance k: transform_ray_inverse (vmath.h:275-278), every lane
                    const int k = inst_next++;
                    DBG_CHECK(k >= 0 && k < S.ninst, 3, k, inst_end, sp, base, 0);
#ifdef YRT_WIDE_STATS
                    if (!COUNT) wc.inst++;
#endif
                    float4 fr[4];
                    ld_records_at<4>(S.tinst, (unsigned)(4 * k), fr);
                    const frame3f f = {xyz(fr[0]), xyz(fr[1]), xyz(fr[2]), xyz(fr[3])};
                    co = transform_point_inverse(f, wo);
                    const bool ident = (uniform(ibits(fr[0].w)) & (int)inst_identity_bit) != 0;
                    if (ident)
                        cd = icd, ci = ici;
                    else
                        enter_direction(f, wd, live & ~done, cd, ci);
                    const uint32_t rk = (uint32_t)uniform(ibits(fr[3].w));
                    pbase = S.spair + spine_record_f4 * (rk & 0x3fffffffu);
                    kind = (int)(rk >> 30);
                    cur_slot = k;
                    mask = avail;
                    if (COUNT && (mask & me)) wc.inst++;
                    node = 0;  // the shape root, tested like any popped node
                    oct = ident ? ioct : wave_octant(ci, live & ~done);
                    if (mask) break;
                    continue;
                }
                level = 0;
                avail = live & ~done;
                pbase = ptop;
                co = wo;
                cd = wd;
                {
                    const int t = YRT_R5_LANE ? wave * 64 + lane_now() : (int)threadIdx.x;
                    ci = {wi_lds[0][t], wi_lds[1][t], wi_lds[2][t]};
                }
                oct = woct;
            }
            if (sp == 0) {
                finished = true;
                break;
            }
            if constexpr (SM) {
                sp--;
                node = __builtin_amdgcn_readlane(stk_node, sp);
                mask = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(stk_mhi, sp) << 32 |
                        (uint32_t)__builtin_amdgcn_readlane(stk_mlo, sp)) &
                       ~done;
                if (mask) break;
            } else {
                // the level's available lanes (inner_pop_avail); none: its entries are all skipped
                mask = avail;
                if (!mask) {
                    sp = level ? base : 0;
                    continue;
                }
                sp--;
                node = __builtin_amdgcn_readlane(stk_node, sp);
                break;
            }
        }
        if (finished) {
            if (!LM) break;
            lstep = true;  // this list entry is done: the next one
        }
    }
#ifdef YRT_WIDE_STATS
    if (!COUNT) {
        const unsigned long long hitl = ballot(hslot >= 0) & live;
        if ((threadIdx.x & 63) == 0) {
            unsigned long long* line = g_first_stats + 16 * ((blockIdx.x * 7u + threadIdx.x / 64u) & 1023u);
            const unsigned long long v[10] = {1, wc.tex, wc.wnode, wc.inst, wc.wprim, wc.box, wc.prim, 0,
                                              (unsigned long long)__popcll(live), (unsigned long long)__popcll(hitl)};
            for (int i = 0; i < 10; i++) atomicAdd(line + i, v[i]);
        }
        wc = work_counts{};  // (a persistent caller keeps one wc across its items)
    }
#endif
    if (hslot < 0) return false;
    hr.slot = hslot;
    hr.ei = hei;
    hr.ew = {1 - hw1 - hw2, hw1, hw2, 0};
    hr.dist = tmax;
    return true;
}

// A wide record through the scalar cache: its first 112 bytes (bounds and child words:
// x16 + x8 + x4, 28 SGPRs instead of 32) -- the slot count in the last row is implied by
// the child words, an empty slot's word being wide_leaf exactly (a leaf of no
// primitives: skipping one changes nothing). A/B: shadow -1.1 to -1.7 %.
__device__ __forceinline__ void ld_wide_record(const f4* wbase, uint32_t off, float4 (&r)[7]) {
    sgpr16 a;
    sgpr8 b;
    sgpr4 c;
    asm volatile(
        "s_load_dwordx16 %0, %3, %4\n s_load_dwordx8 %1, %3, %4 offset:0x40\n s_load_dwordx4 %2, %3, %4 offset:0x60\n"
        " s_waitcnt lgkmcnt(0)"
        : "=&s"(a), "=&s"(b), "=&s"(c)
        : "s"(wbase), "s"(uniform((int)off)));
#pragma unroll
    for (int k = 0; k < 4; k++) r[k] = rec_of(a, k);
    r[4] = rec_of(b, 0), r[5] = rec_of(b, 1), r[6] = rec_of(c, 0);
}

// ---- a cheaper slab test for the any-hit walk's inner slots ----
// Any hit does not depend on the order of the walk, only on which leaves are reached, and
// the reference reaches a leaf exactly when the leaf's own box passes intersect_check_bbox
// (scene.cpp:371-382): its ancestors' boxes contain it and the test is monotone in the box
// (the argument of the 4-wide collapse, packet_occluded_wide2). So an inner slot may use
// any test that passes at least every ray the exact one passes; leaf slots keep the exact
// test, and the set of leaves reached -- and so the answer -- stays the reference's.
//
// The inner test computes each plane distance as one FMA, fma(b, invd, -(o * invd)), instead
// of (b - o) * invd (a subtraction and a product), and widens the comparison by the error
// of that form. Per plane, with u = 2^-24, T = (b - o) * invd the real value, e the exact
// test's value and c the FMA's: |e - T| <= 2.0001u|T|, |c - T| <= u|T| + 1.0001uM, where
// M = max_a |o_a * invd_a| (the rounding of the per-lane product), so
// |c - e| <= 3.001u|c| + 1.001uM. Carried through the max/min chains (lo >= tmin > 0 on a
// passing exact test) and the reference's tmax * 1.00000024, an exact pass implies
//     lo_c <= hi_c * (1 + 11.1u) + 2.1uM,
// which the inner test admits with room: lo_c <= fma(hi_c, 1 + 16u, max(16uM, 2^-100))
// (the floor covers underflow). The inner test is 12 VALU against the exact test's 18.
// It is taken only when every live lane has a finite invd and M <= 2^100 (a zero direction
// component or a huge offset makes the wave use the exact test everywhere), and only for
// single-octant waves (OCT < 8), on nodes whose four slots are all inner (one scalar branch
// per node). Compile-time switch YRT_ANY_CONSERVATIVE, off: it loses (DESIGN.md §5 round 5:
// c4 shadow 11.63 -> 12.49 ms per node, 12.91 with a branch per inner slot -- the walk is
// co-bound by the scalar unit, which the branches load, and the planes cost 6 VGPRs and 6
// SGPR spills).
#ifndef YRT_ANY_CONSERVATIVE
#define YRT_ANY_CONSERVATIVE 0
#endif
struct inner_planes {
    vec3f noci;  // -(o * invd), per lane
    float marg;  // max(16uM, 2^-100), per lane
    bool on;     // wave-uniform: the inner slots use the conservative test
};

__device__ __forceinline__ inner_planes make_inner_planes(vec3f o, vec3f ci, unsigned long long lanes) {
    inner_planes p;
    p.noci = {-(o.x * ci.x), -(o.y * ci.y), -(o.z * ci.z)};
    const float M = fmaxf(fmaxf(fabsf(p.noci.x), fabsf(p.noci.y)), fabsf(p.noci.z));
    p.marg = fmaxf(M * 0x1p-20f, 0x1p-100f);
    // (a NaN fails every comparison: that lane turns the test off for the wave)
    const bool ok = M <= 0x1p100f && fabsf(ci.x) <= 0x1p100f && fabsf(ci.y) <= 0x1p100f && fabsf(ci.z) <= 0x1p100f;
    p.on = YRT_ANY_CONSERVATIVE && !(ballot(!ok) & lanes);
    return p;
}

template <int OCT>
__device__ __forceinline__ bool box_oct_inner(const inner_planes& P, vec3f invd, float tmin_r, float tmax_r, float lx,
                                              float ly, float lz, float hx, float hy, float hz) {
    const float nx = (OCT & 1) ? hx : lx, fx = (OCT & 1) ? lx : hx;
    const float ny = (OCT & 2) ? hy : ly, fy = (OCT & 2) ? ly : hy;
    const float nz = (OCT & 4) ? hz : lz, fz = (OCT & 4) ? lz : hz;
    const float t0x = fmaf(nx, invd.x, P.noci.x), t0y = fmaf(ny, invd.y, P.noci.y), t0z = fmaf(nz, invd.z, P.noci.z);
    const float t1x = fmaf(fx, invd.x, P.noci.x), t1y = fmaf(fy, invd.y, P.noci.y), t1z = fmaf(fz, invd.z, P.noci.z);
    const float lo = fmaxf(fmaxf(fmaxf(t0x, t0y), t0z), tmin_r);
    const float hi = fminf(fminf(fminf(t1x, t1y), t1z), tmax_r);
    return lo <= fmaf(hi, 1.00000095367431640625f, P.marg);  // 1 + 2^-20
}

// the slab tests of a wide step on the record r: m[k] = the lanes of `mask` that pass
// slot k's box (0 for a slot the node does not have: a scalar branch around it), w[k] =
// slot k's child word. A node of four inner slots takes box_oct_inner when P.on.
template <int OCT>
__device__ __forceinline__ void wide_tests(const float4 (&r)[7], vec3f co, vec3f ci, float tmin, float tmax,
                                           const inner_planes& P, unsigned long long mask, uint32_t (&w)[4],
                                           unsigned long long (&m)[4]) {
    const float lx[4] = {r[0].x, r[0].y, r[0].z, r[0].w}, ly[4] = {r[1].x, r[1].y, r[1].z, r[1].w},
                lz[4] = {r[2].x, r[2].y, r[2].z, r[2].w}, hx[4] = {r[3].x, r[3].y, r[3].z, r[3].w},
                hy[4] = {r[4].x, r[4].y, r[4].z, r[4].w}, hz[4] = {r[5].x, r[5].y, r[5].z, r[5].w};
    w[0] = (uint32_t)uniform(ibits(r[6].x)), w[1] = (uint32_t)uniform(ibits(r[6].y));
    w[2] = (uint32_t)uniform(ibits(r[6].z)), w[3] = (uint32_t)uniform(ibits(r[6].w));
    if (YRT_ANY_CONSERVATIVE && OCT < 8 && P.on && !((w[0] | w[1] | w[2] | w[3]) & wide_leaf)) {
        // a node of four inner slots: all four take the inner test, one branch per node
#pragma unroll
        for (int k = 0; k < 4; k++)
            m[k] = ballot(box_oct_inner<OCT < 8 ? OCT : 0>(P, ci, tmin, tmax, lx[k], ly[k], lz[k], hx[k], hy[k], hz[k])) &
                   mask;
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < 2 || w[k] != wide_leaf) {  // every wide node has >= 2 slots but a leaf root's 1
            m[k] = ballot(box_oct<OCT>(co, ci, tmin, tmax, lx[k], ly[k], lz[k], hx[k], hy[k], hz[k])) & mask;
        } else
            m[k] = 0;
    }
}

// one step of the 4-wide any-hit descent on the record r (in SGPRs when it came through
// the scalar cache, in VGPRs -- the same value in every lane -- when it came from LDS):
// the four slab tests, then the first passing child becomes current and the other
// passing ones are pushed last-to-first (three v_writelane each: word, mask halves), so
// they pop in slot order. Returns true to continue the descent from `cur`.
template <int OCT>
__device__ __forceinline__ bool wide_step(const float4 (&r)[7], vec3f co, vec3f ci, float tmin, float tmax,
                                          const inner_planes& P,
                                          uint32_t& cur, unsigned long long& mask, int& sp, int& stk_word,
                                          int& stk_mlo, int& stk_mhi, int floor, unsigned long long done) {
    uint32_t w[4];
    unsigned long long m[4];
    wide_tests<OCT>(r, co, ci, tmin, tmax, P, mask, w, m);
    unsigned long long cm = 0;
    uint32_t cw = 0;
    // the select chain as written for the scalar unit. Chain A tests the slots from the
    // highest while none has passed; the first passing slot j becomes the candidate and
    // control moves to the blocks that know it: B(j,k) tests slot k < j and, when it
    // passes, pushes slot j's word and mask halves straight from the record/ballot
    // registers (three v_writelane at lane sp) and continues in B(k, k-1). FIN(j) hands
    // back slot j. Per slot one s_cmp_lg_u64 and one branch; no materialised conditions
    // and no copies of the candidate. cm = 0 when no slot passed.
    {
        uint32_t ow;
        unsigned long long om;
        // (wave-uniform first: folded away where the compiler holds sp in an SGPR; needed where
        // its uniformity analysis lost track of it)
        sp = uniform(sp);
        asm volatile(
            "s_cmp_lg_u64 %[m3], 0\n"
            "s_cbranch_scc1 .Lyb32_%=\n"
            "s_cmp_lg_u64 %[m2], 0\n"
            "s_cbranch_scc1 .Lyb21_%=\n"
            "s_cmp_lg_u64 %[m1], 0\n"
            "s_cbranch_scc1 .Lyb10_%=\n"
            "s_cmp_lg_u64 %[m0], 0\n"
            "s_cbranch_scc1 .Lyfin0_%=\n"
            "s_mov_b64 %[cm], 0\n"
            "s_mov_b32 %[cw], 0\n"
            "s_branch .Lyend_%=\n"
            ".Lyb32_%=:\n"
            "s_cmp_lg_u64 %[m2], 0\n"
            "s_cbranch_scc0 .Lyb31_%=\n"
            "s_mov_b32 m0, %[sp]\n"
            "v_writelane_b32 %[sw], %[w3], m0\n"
            "v_writelane_b32 %[sl], %[l3], m0\n"
            "v_writelane_b32 %[sh], %[h3], m0\n"
            "s_add_u32 %[sp], %[sp], 1\n"
            "s_branch .Lyb21_%=\n"
            ".Lyb31_%=:\n"
            "s_cmp_lg_u64 %[m1], 0\n"
            "s_cbranch_scc0 .Lyb30_%=\n"
            "s_mov_b32 m0, %[sp]\n"
            "v_writelane_b32 %[sw], %[w3], m0\n"
            "v_writelane_b32 %[sl], %[l3], m0\n"
            "v_writelane_b32 %[sh], %[h3], m0\n"
            "s_add_u32 %[sp], %[sp], 1\n"
            "s_branch .Lyb10_%=\n"
            ".Lyb30_%=:\n"
            "s_cmp_lg_u64 %[m0], 0\n"
            "s_cbranch_scc0 .Lyfin3_%=\n"
            "s_mov_b32 m0, %[sp]\n"
            "v_writelane_b32 %[sw], %[w3], m0\n"
            "v_writelane_b32 %[sl], %[l3], m0\n"
            "v_writelane_b32 %[sh], %[h3], m0\n"
            "s_add_u32 %[sp], %[sp], 1\n"
            "s_branch .Lyfin0_%=\n"
            ".Lyb21_%=:\n"
            "s_cmp_lg_u64 %[m1], 0\n"
            "s_cbranch_scc0 .Lyb20_%=\n"
            "s_mov_b32 m0, %[sp]\n"
            "v_writelane_b32 %[sw], %[w2], m0\n"
            "v_writelane_b32 %[sl], %[l2], m0\n"
            "v_writelane_b32 %[sh], %[h2], m0\n"
            "s_add_u32 %[sp], %[sp], 1\n"
            "s_branch .Lyb10_%=\n"
            ".Lyb20_%=:\n"
            "s_cmp_lg_u64 %[m0], 0\n"
            "s_cbranch_scc0 .Lyfin2_%=\n"
            "s_mov_b32 m0, %[sp]\n"
            "v_writelane_b32 %[sw], %[w2], m0\n"
            "v_writelane_b32 %[sl], %[l2], m0\n"
            "v_writelane_b32 %[sh], %[h2], m0\n"
            "s_add_u32 %[sp], %[sp], 1\n"
            "s_branch .Lyfin0_%=\n"
            ".Lyb10_%=:\n"
            "s_cmp_lg_u64 %[m0], 0\n"
            "s_cbranch_scc0 .Lyfin1_%=\n"
            "s_mov_b32 m0, %[sp]\n"
            "v_writelane_b32 %[sw], %[w1], m0\n"
            "v_writelane_b32 %[sl], %[l1], m0\n"
            "v_writelane_b32 %[sh], %[h1], m0\n"
            "s_add_u32 %[sp], %[sp], 1\n"
            "s_branch .Lyfin0_%=\n"
            ".Lyfin3_%=:\n"
            "s_mov_b32 %[cw], %[w3]\n"
            "s_mov_b64 %[cm], %[m3]\n"
            "s_branch .Lyend_%=\n"
            ".Lyfin2_%=:\n"
            "s_mov_b32 %[cw], %[w2]\n"
            "s_mov_b64 %[cm], %[m2]\n"
            "s_branch .Lyend_%=\n"
            ".Lyfin1_%=:\n"
            "s_mov_b32 %[cw], %[w1]\n"
            "s_mov_b64 %[cm], %[m1]\n"
            "s_branch .Lyend_%=\n"
            ".Lyfin0_%=:\n"
            "s_mov_b32 %[cw], %[w0]\n"
            "s_mov_b64 %[cm], %[m0]\n"
            ".Lyend_%=:\n"
            : [cw] "=&s"(ow), [cm] "=&s"(om), [sp] "+s"(sp), [sw] "+v"(stk_word), [sl] "+v"(stk_mlo),
              [sh] "+v"(stk_mhi)
            : [w0] "s"(w[0]), [w1] "s"(w[1]), [w2] "s"(w[2]), [w3] "s"(w[3]), [m0] "s"(m[0]), [m1] "s"(m[1]),
              [m2] "s"(m[2]), [m3] "s"(m[3]), [l0] "s"((uint32_t)m[0]), [l1] "s"((uint32_t)m[1]),
              [l2] "s"((uint32_t)m[2]), [l3] "s"((uint32_t)m[3]), [h0] "s"((uint32_t)(m[0] >> 32)),
              [h1] "s"((uint32_t)(m[1] >> 32)), [h2] "s"((uint32_t)(m[2] >> 32)), [h3] "s"((uint32_t)(m[3] >> 32))
            : "m0", "scc");
        // asm results count as divergent to the compiler: readfirstlane (folded away on
        // SGPRs) keeps what follows on the scalar unit
        sp = uniform(sp);
        cw = (uint32_t)uniform((int)ow);
        cm = (unsigned long long)(uint32_t)uniform((int)(om >> 32)) << 32 | (uint32_t)uniform((int)(uint32_t)om);
    }
    mask = cm;
    cur = cw;
    if (cm) return !(cw & wide_leaf);
    {
        int n = 0;
        if (inner_pop(floor, done, n, mask, sp, stk_word, stk_mlo, stk_mhi)) {
            cur = (uint32_t)n;
            return !(cur & wide_leaf);
        }
    }
    return false;
}

// one descent of the 4-wide any-hit walk: from the wide node `cur` (a child word,
// yrt_device.h) through wide nodes until the current item is a leaf (mask != 0) or no
// child passes (mask = 0). LDSN > 0: the first LDSN records (the breadth-first top of
// the instance tree, staged by the persistent kernel) are read from `lds` with
// ds_read_b128 at a wave-uniform address; every other record through the scalar cache.
// `base`: the records `cur` is a byte offset into (S.wnodes, or a shadow bundle's list,
// packet_occluded_wide2)
template <int OCT, int LDSN, bool ASM = false>
__device__ __forceinline__ void wide_descend(const f4* base, const float4* lds, vec3f co, vec3f ci,
                                             const inner_planes& P,
                                             float tmin, float tmax, uint32_t& cur, unsigned long long& mask,
                                             int& sp, int& stk_word, int& stk_mlo, int& stk_mhi, int floor,
                                             unsigned long long done, unsigned& nsteps) {
#if YRT_WIDE_ASM && !defined(YRT_WIDE_STATS)
    // the same loop as one asm block (wide_asm.h, tools/gen_wide_asm.py) for the records read
    // through the scalar cache and the exact slab tests
    if constexpr (ASM && LDSN == 0 && OCT < 8 && !YRT_ANY_CONSERVATIVE) {
        auto u64 = [](unsigned long long v) {
            return (unsigned long long)(uint32_t)uniform((int)(v >> 32)) << 32 | (uint32_t)uniform((int)(uint32_t)v);
        };
        cur = (uint32_t)uniform((int)cur), sp = uniform(sp), mask = u64(mask);
        wide_asm<OCT>::run(sgpr_ptr(base), co, ci, tmin, tmax, uniform(floor), u64(done), cur, mask, sp, stk_word,
                           stk_mlo, stk_mhi);
        sp = uniform(sp);
        mask = u64(mask);
        cur = (uint32_t)uniform((int)cur);
        asm volatile("" : "+s"(mask), "+s"(cur), "+s"(sp));
        return;
    }
#endif
    const f4* wbase = sgpr_ptr(base);
    for (;;) {
        bool more;
#ifdef YRT_WIDE_STATS
        nsteps++;
#endif
        if (LDSN > 0 && cur < (uint32_t)(LDSN * wide_record_bytes)) {
            float4 r[7];
            const float4* p = lds + (cur >> 4);
#pragma unroll
            for (int k = 0; k < 7; k++) r[k] = p[k];
            more = wide_step<OCT>(r, co, ci, tmin, tmax, P, cur, mask, sp, stk_word, stk_mlo, stk_mhi, floor, done);
        } else {
            float4 r[7];
            ld_wide_record(wbase, cur, r);
            more = wide_step<OCT>(r, co, ci, tmin, tmax, P, cur, mask, sp, stk_word, stk_mlo, stk_mhi, floor, done);
        }
        if (!more) return;
    }
}

// ---- any hit on the 4-wide collapse, laid out for the scalar unit ----
// intersect_any (scene.cpp:489) over the 4-wide collapse of the reference BVH
// (device_scene.cpp wide_builder): the same packet discipline as packet_first (SGPR
// control, lane masks, a stack in VGPR lanes) over wide nodes. Results equal
// intersect_any's: every box of the collapse is one the reference tests, a box test is
// monotone in the box (NaN slabs included), so every leaf reached is one the reference
// reaches, and the any-hit answer does not depend on the order. The instrumented
// (COUNT) kernels use the binary walk instead, so work counts stay the reference's.
//
// tbase / troot: where the instance level's walk starts -- S.wnodes and the wide tree's root,
// or the wide records of a shadow bundle's candidate leaves (wavefront.hip k_bundle_lists:
// every instance-level leaf whose box a ray of the bundle can pass, so walking them instead
// of the tree reaches the same leaves; the leaves' boxes and words are the tree's own)
// ASM: the descent through the generated assembly (wide_asm.h; the persistent any-hit grid
// only -- its 36 fixed SGPRs are too many for the backend in some of the other kernels'
// diagnostic builds)
template <int LDSN = 0, bool ASM = false>
__device__ __forceinline__ bool packet_occluded_wide2(const dev_scene_view& S, const ray3& wray, bool valid,
                                                      const float4* lds = nullptr, const f4* tbase = nullptr,
                                                      uint32_t troot = 0, unsigned long long pre_done = 0) {
    const unsigned long long me = 1ull << __lane_id();
    const unsigned long long live = ballot(valid && !is_nan(wray.tmin) && !is_nan(wray.tmax));
    if (!live) return false;
    // pre_done: lanes answered already (their shadow ray is culled: reported occluded)
    if (!(live & ~pre_done)) return (pre_done & me) != 0;
    const vec3f wo = wray.o, wd = wray.d;
    const vec3f wi = rcp3(wd, live);
    const float tmin = wray.tmin, tmax = wray.tmax;
    vec3f co = wo, cd = wd, ci = wi;
    int stk_word = 0, stk_mlo = 0, stk_mhi = 0;
    unsigned long long done = pre_done & live, inst_mask = 0;
    int level = 0, sp = 0, base = 0, kind = 0, inst_first = 0;
    // the current leaf's instances still to enter: bit i = instance inst_first + i (a wide leaf
    // holds at most 7); the instances a bundle's hull excludes are not in it (its skip bits)
    uint32_t inst_keep = 0;
    if (!tbase) tbase = S.wnodes, troot = (uint32_t)S.wtop_root;
    // level 0 walks a shadow bundle's list in the bundle records' leaf format
    const bool blist = S.inst_masks && tbase != S.wnodes;
    // the current item: a child word (a wide node's byte offset, or a leaf)
    uint32_t cur = troot;
    unsigned long long mask = live & ~done;
    // the octant of the current level's rays when the whole wave shares it (8: mixed)
    const int woct = wave_octant(wi, live);
    int oct = woct;
    // the instance-local direction of every instance whose rotation is the identity:
    // enter_direction on the identity frame is what entering any of them computes, bit for
    // bit (the same dot products, normalisation and reciprocals), so it is done once here
    vec3f icd, ici;
    enter_direction(frame3f{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}}, wd, live, icd, ici);
    const int ioct = wave_octant(ici, live);
    // the inner slots' conservative planes of the current level (recomputed with co / ci)
    inner_planes ip = make_inner_planes(wo, wi, live);
    unsigned nsteps0 = 0, nsteps1 = 0;
#ifdef YRT_WIDE_STATS
    unsigned ws[16] = {1, 0, 0, 0, 0, 0, 0, 0};
#endif
    for (;;) {
        // ---- descent through wide nodes until a leaf or no passing child ----
        if (!(cur & wide_leaf)) {
            const int wfloor = level ? base : 0;
            DBG_CHECK(((level == 0 && tbase != S.wnodes) || cur < (uint32_t)S.nwnodes * wide_record_bytes) && sp >= 0 &&
                          sp < 61, 4, (int)cur, sp, level,
                      base, 0);
#define YRT_WD(o) wide_descend<o, LDSN, ASM>(level ? S.wnodes : tbase, lds, co, ci, ip, tmin, tmax, cur, mask, sp, stk_word, \
                                         stk_mlo, stk_mhi, wfloor, done, level ? nsteps1 : nsteps0)
            switch (oct) {
                case 0: YRT_WD(0); break;
                case 1: YRT_WD(1); break;
                case 2: YRT_WD(2); break;
                case 3: YRT_WD(3); break;
                case 4: YRT_WD(4); break;
                case 5: YRT_WD(5); break;
                case 6: YRT_WD(6); break;
                case 7: YRT_WD(7); break;
                default: YRT_WD(8); break;
            }
#undef YRT_WD
        }
        // ---- the leaf reached, if any ----
        if (mask) {
            const int first = (int)(cur & wide_index_mask);
            const int count = (int)((cur >> wide_count_shift) & 7u);
            if (level == 0) {
                // a shadow bundle's leaf (bundle_leaf_word): the instances its hull excludes
                // are skipped (wavefront.hip k_bundle_lists); a tree leaf: none
                inst_first = blist ? (int)(cur & bundle_first_mask) : first;
                inst_keep = ((1u << count) - 1u) & ~(blist ? (cur >> bundle_skip_shift) & 0x7fu : 0u);
                inst_mask = mask;
                level = 1;
                base = sp;
            } else {
                DBG_CHECK(first >= 0 && first + count <= S.nsprims, 5, first, count, level, kind, sp);
                const bool inl = (mask & me) != 0;
                int leaf_hit = 0;
                WSTAT(4, 1u);
                WSTAT(5, (unsigned)count);
                if (kind == kind_triangles) {
                    for (int i = first; i < first + count; i++) {
                        float t, w1, w2;
                        // v0, e1, e2 as 9 packed dwords (yrt_device.h aprims): 9 SGPRs, not 12
                        const f4* abase = sgpr_ptr(reinterpret_cast<const f4*>(S.aprims));
                        sgpr8 a;
                        int b;
                        asm volatile("s_load_dwordx8 %0, %2, %3\n s_load_dword %1, %2, %3 offset:0x20\n"
                                     " s_waitcnt lgkmcnt(0)"
                                     : "=&s"(a), "=&s"(b)
                                     : "s"(abase), "s"(uniform(i * 36)));
                        const vec3f tv0 = {__int_as_float(a[0]), __int_as_float(a[1]), __int_as_float(a[2])};
                        const vec3f te1 = {__int_as_float(a[3]), __int_as_float(a[4]), __int_as_float(a[5])};
                        const vec3f te2 = {__int_as_float(a[6]), __int_as_float(a[7]), __int_as_float(b)};
                        // (per lane, not tri_hit_mask: this kernel is bound by scalar issue, and the
                        // mask form -- with the leaf left once every lane hit -- moves VALU work to
                        // the scalar unit: shadow 8.13 -> 8.38 ms at c4)
                        const bool h = tri_hit_nb<true>(co, cd, tmin, tmax, tv0, te1, te2, t, w1, w2, inl, mask);
                        leaf_hit |= (h && inl) ? 1 : 0;
                    }
                } else {
                    for (int i = first; i < first + count; i++) {
                        float4 pv[3];
                        ld_records_at<3>(S.sprims, (unsigned)(3 * i), pv);
                        float t;
                        vec4f ew;
                        const ray3 lr = {co, cd, tmin, tmax};
                        const bool h = kind == kind_lines
                                           ? line_hit(lr, xyz(pv[0]), xyz(pv[1]), pv[1].w, pv[2].x, t, ew)
                                           : point_hit(lr, xyz(pv[0]), pv[1].x, t, ew);
                        leaf_hit |= (h && inl) ? 1 : 0;
                    }
                }
                done |= ballot(leaf_hit != 0);
                if (!(live & ~done)) break;
            }
        }
        // ---- the next item: the next instance of the current leaf, or a pop ----
        bool finished = false;
        for (;;) {
            if (level == 1 && sp == base) {
                if (inst_keep) {
                    const int k = inst_first + __builtin_ctz(inst_keep);
                    inst_keep &= inst_keep - 1u;
                    DBG_CHECK(k >= 0 && k < S.ninst, 6, k, inst_first, sp, base, 0);
                    float4 fr[winst_rows];
                    ld_records_at<winst_rows>(S.winst, (unsigned)(winst_rows * k), fr);
                    const frame3f f = {xyz(fr[0]), xyz(fr[1]), xyz(fr[2]), xyz(fr[3])};
                    co = transform_point_inverse(f, wo);
                    const bool ident = (uniform(ibits(fr[0].w)) & (int)inst_identity_bit) != 0;
                    if (ident)
                        cd = icd, ci = ici;
                    else
                        enter_direction(f, wd, live & ~done, cd, ci);
                    const uint32_t rk = (uint32_t)uniform(ibits(fr[1].w));
                    cur = rk & 0x3fffffffu;  // the shape's wide root (a record byte offset)
                    kind = (int)(rk >> 30);
                    mask = inst_mask & ~done;
                    {
                        // the shape root's own box, which the wide root (its children's
                        // children) skips: the reference tests it first, and a lane that
                        // fails it finds nothing in this instance (every box below is
                        // inside it)
                        float tn;
                        mask &= ballot(box_hit6(co, ci, tmin, tmax, fr[2].w, fr[3].w, fr[4].x, fr[4].y, fr[4].z,
                                                fr[4].w, tn));
                    }
                    WSTAT(3, 1u);
                    WSTAT(12, mask ? 0u : 1u);  // entries whose root box no lane passes
                    oct = ident ? ioct : wave_octant(ci, live & ~done);
                    ip = make_inner_planes(co, ci, mask);
                    if (mask) break;
                    continue;
                }
                level = 0;
                co = wo;
                cd = wd;
                ci = wi;
                oct = woct;
                ip = make_inner_planes(wo, wi, live & ~done);
            }
            if (sp == 0) {
                finished = true;
                break;
            }
            sp--;
            cur = (uint32_t)__builtin_amdgcn_readlane(stk_word, sp);
            mask = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(stk_mhi, sp) << 32 |
                    (uint32_t)__builtin_amdgcn_readlane(stk_mlo, sp)) &
                   ~done;
            WSTAT(6, 1u);
            WSTAT(7, mask ? 0u : 1u);
            if (mask) break;
        }
        if (finished) break;
    }
#ifdef YRT_WIDE_STATS
    ws[1] = nsteps0, ws[2] = nsteps1;
    ws[8] = (unsigned)__popcll(live), ws[9] = (unsigned)__popcll(done & live);
    ws[10] = (live & ~done) ? 0u : 1u, ws[11] = (live & ~done) ? 0u : nsteps0 + nsteps1;
    if (__lane_id() == 0) {
        unsigned long long* line = g_wide_stats + 16 * ((blockIdx.x * 7u + threadIdx.x / 64u) & 1023u);
        for (int i = 0; i < 13; i++) atomicAdd(line + i, (unsigned long long)ws[i]);
    }
#endif
    return (done & me) != 0;
}

}  // namespace yrt
