// packet_dual.h -- the 4-wide any-hit walk of packet_trace.h with TWO rays per lane.
//
// Lane l carries sample l of two neighbouring pixels' shadow rays to the same light
// (ray A and ray B). The wave-uniform control -- the record fetch, the stack, the
// branches -- is what bounds the one-ray walk (SALU 78 % busy at c4), and the
// union of two neighbouring pixels' walks is barely larger than one: sharing one walk
// between 128 rays spends that scalar work once for both, while the per-ray vector work
// (slab tests, triangle tests, instance transforms) stays what it was.
//
// Every ray sees exactly what packet_occluded_wide2 would give it: the set of (lane, ray)
// pairs that reach a node is a pair of lane masks; a child is entered or pushed when
// either mask is non-empty, and each ray's box and primitive tests use its own data and
// mask. The any-hit answer of a ray is the reference's for the same reasons as the
// one-ray walk (same boxes, monotone tests, order-free answer).
//
// Contract: every lane of the wave calls it in uniform control flow.
#pragma once

#include "packet_trace.h"

namespace yrt {

struct dual_ray {
    vec3f co, cd, ci;  // the current level's ray (instance-local inside an instance)
    vec3f wo, wd, wi;  // the world ray
    float tmax;
};

// the octant shared by every live lane of both rays, or 8
__device__ __forceinline__ int dual_octant(vec3f ciA, unsigned long long la, vec3f ciB, unsigned long long lb) {
    if (!la) return wave_octant(ciB, lb);
    if (!lb) return wave_octant(ciA, la);
    const int a = wave_octant(ciA, la), b = wave_octant(ciB, lb);
    return a == b ? a : 8;
}

template <int OCT>
__device__ __forceinline__ bool wide_step_dual(const float4 (&r)[8], const dual_ray& A, const dual_ray& B, float tmin,
                                               uint32_t& cur, unsigned long long& ma, unsigned long long& mb, int& sp,
                                               int& s_word, int& s_alo, int& s_ahi, int& s_blo, int& s_bhi, int floor,
                                               unsigned long long done_a, unsigned long long done_b) {
    const float lx[4] = {r[0].x, r[0].y, r[0].z, r[0].w}, ly[4] = {r[1].x, r[1].y, r[1].z, r[1].w},
                lz[4] = {r[2].x, r[2].y, r[2].z, r[2].w}, hx[4] = {r[3].x, r[3].y, r[3].z, r[3].w},
                hy[4] = {r[4].x, r[4].y, r[4].z, r[4].w}, hz[4] = {r[5].x, r[5].y, r[5].z, r[5].w};
    const uint32_t w[4] = {(uint32_t)uniform(ibits(r[6].x)), (uint32_t)uniform(ibits(r[6].y)),
                           (uint32_t)uniform(ibits(r[6].z)), (uint32_t)uniform(ibits(r[6].w))};
    const int nslots = uniform(ibits(r[7].x));
    unsigned long long pa[4], pb[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < 2 || k < nslots) {
            pa[k] = ballot(box_oct<OCT>(A.co, A.ci, tmin, A.tmax, lx[k], ly[k], lz[k], hx[k], hy[k], hz[k])) & ma;
            pb[k] = ballot(box_oct<OCT>(B.co, B.ci, tmin, B.tmax, lx[k], ly[k], lz[k], hx[k], hy[k], hz[k])) & mb;
        } else {
            pa[k] = pb[k] = 0;
        }
    }
    unsigned long long ca = 0, cb = 0;
    uint32_t cw = 0;
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        if (pa[k] | pb[k]) {
            if (ca | cb) {
                s_word = writelane(s_word, (int)cw, sp);
                s_alo = writelane(s_alo, (int)(uint32_t)ca, sp);
                s_ahi = writelane(s_ahi, (int)(uint32_t)(ca >> 32), sp);
                s_blo = writelane(s_blo, (int)(uint32_t)cb, sp);
                s_bhi = writelane(s_bhi, (int)(uint32_t)(cb >> 32), sp);
                sp++;
            }
            ca = pa[k];
            cb = pb[k];
            cw = w[k];
        }
    }
    ma = ca;
    mb = cb;
    cur = cw;
    if (ca | cb) return !(cw & wide_leaf);
    // pop inside the descent: entries above `floor` until one with a live lane
    while (sp > floor) {
        sp--;
        const uint32_t n = (uint32_t)__builtin_amdgcn_readlane(s_word, sp);
        ma = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(s_ahi, sp) << 32 |
              (uint32_t)__builtin_amdgcn_readlane(s_alo, sp)) &
             ~done_a;
        mb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(s_bhi, sp) << 32 |
              (uint32_t)__builtin_amdgcn_readlane(s_blo, sp)) &
             ~done_b;
        if (ma | mb) {
            cur = n;
            return !(cur & wide_leaf);
        }
    }
    ma = mb = 0;
    return false;
}

template <int OCT>
__device__ __forceinline__ void wide_descend_dual(const dev_scene_view& S, const dual_ray& A, const dual_ray& B,
                                                  float tmin, uint32_t& cur, unsigned long long& ma,
                                                  unsigned long long& mb, int& sp, int& s_word, int& s_alo,
                                                  int& s_ahi, int& s_blo, int& s_bhi, int floor,
                                                  unsigned long long done_a, unsigned long long done_b) {
    const f4* wbase = sgpr_ptr(S.wnodes);
    for (;;) {
        float4 r[8];
        sgpr16 a, b;
        asm volatile("s_load_dwordx16 %0, %2, %3\n s_load_dwordx16 %1, %2, %3 offset:0x40\n s_waitcnt lgkmcnt(0)"
                     : "=&s"(a), "=&s"(b)
                     : "s"(wbase), "s"(uniform((int)cur)));
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = rec_of(a, k), r[4 + k] = rec_of(b, k);
        if (!wide_step_dual<OCT>(r, A, B, tmin, cur, ma, mb, sp, s_word, s_alo, s_ahi, s_blo, s_bhi, floor, done_a,
                                 done_b))
            return;
    }
}

// the primitives of one shape leaf for one of the two rays: lanes in `lanes` that are hit
__device__ __forceinline__ unsigned long long dual_leaf_hits(const dev_scene_view& S, int kind, int first, int count,
                                                             const dual_ray& R, float tmin, unsigned long long lanes) {
    const bool in = (lanes >> __lane_id()) & 1;
    int leaf_hit = 0;
    if (kind == kind_triangles) {
        for (int i = first; i < first + count; i++) {
            float4 pv[3];
            ld_records<3>(S.sprims + 3 * i, pv);
            float t, w1, w2;
            const bool h = tri_hit_nb<YRT_TRI_RCP>(R.co, R.cd, tmin, R.tmax, xyz(pv[0]), xyz(pv[1]), xyz(pv[2]), t,
                                                   w1, w2, in, ballot(in));
            leaf_hit |= (h && in) ? 1 : 0;
        }
    } else {
        for (int i = first; i < first + count; i++) {
            float4 pv[3];
            ld_records<3>(S.sprims + 3 * i, pv);
            float t;
            vec4f ew;
            const ray3 lr = {R.co, R.cd, tmin, R.tmax};
            const bool h = kind == kind_lines ? line_hit(lr, xyz(pv[0]), xyz(pv[1]), pv[1].w, pv[2].x, t, ew)
                                              : point_hit(lr, xyz(pv[0]), pv[1].x, t, ew);
            leaf_hit |= (h && in) ? 1 : 0;
        }
    }
    return ballot(leaf_hit != 0);
}

// intersect_any (scene.cpp:489) for ray A and ray B of every lane; tmin is shared (the
// shadow rays' 0.01, raytrace.cpp:131). occ_a/occ_b: this lane's answers.
__device__ __forceinline__ void packet_occluded_dual(const dev_scene_view& S, const ray3& ra, bool valid_a,
                                                     const ray3& rb, bool valid_b, bool& occ_a, bool& occ_b) {
    const unsigned long long me = 1ull << __lane_id();
    const float tmin = ra.tmin;
    const unsigned long long live_a = ballot(valid_a && !is_nan(ra.tmin) && !is_nan(ra.tmax));
    const unsigned long long live_b = ballot(valid_b && !is_nan(rb.tmin) && !is_nan(rb.tmax));
    occ_a = occ_b = false;
    if (!(live_a | live_b)) return;
    dual_ray A, B;
    A.wo = ra.o, A.wd = ra.d, A.wi = {1.0f / ra.d.x, 1.0f / ra.d.y, 1.0f / ra.d.z}, A.tmax = ra.tmax;
    B.wo = rb.o, B.wd = rb.d, B.wi = {1.0f / rb.d.x, 1.0f / rb.d.y, 1.0f / rb.d.z}, B.tmax = rb.tmax;
    A.co = A.wo, A.cd = A.wd, A.ci = A.wi;
    B.co = B.wo, B.cd = B.wd, B.ci = B.wi;
    int s_word = 0, s_alo = 0, s_ahi = 0, s_blo = 0, s_bhi = 0;
    unsigned long long done_a = 0, done_b = 0, inst_a = 0, inst_b = 0;
    int level = 0, sp = 0, base = 0, kind = 0, inst_next = 0, inst_end = 0;
    uint32_t cur = (uint32_t)S.wtop_root;
    unsigned long long ma = live_a, mb = live_b;
    const int woct = YRT_WIDE_OCTANT ? dual_octant(A.wi, live_a, B.wi, live_b) : 8;
    int oct = woct;
    for (;;) {
        if (!(cur & wide_leaf)) {
            const int floor = level ? base : 0;
#define YRT_WDD(o) wide_descend_dual<o>(S, A, B, tmin, cur, ma, mb, sp, s_word, s_alo, s_ahi, s_blo, s_bhi, floor, done_a, done_b)
            switch (oct) {
                case 0: YRT_WDD(0); break;
                case 1: YRT_WDD(1); break;
                case 2: YRT_WDD(2); break;
                case 3: YRT_WDD(3); break;
                case 4: YRT_WDD(4); break;
                case 5: YRT_WDD(5); break;
                case 6: YRT_WDD(6); break;
                case 7: YRT_WDD(7); break;
                default: YRT_WDD(8); break;
            }
#undef YRT_WDD
        }
        if (ma | mb) {
            const int first = (int)(cur & wide_index_mask);
            const int count = (int)((cur >> wide_count_shift) & 7u);
            if (level == 0) {
                inst_next = first;
                inst_end = first + count;
                inst_a = ma;
                inst_b = mb;
                level = 1;
                base = sp;
            } else {
                if (ma) done_a |= dual_leaf_hits(S, kind, first, count, A, tmin, ma);
                if (mb) done_b |= dual_leaf_hits(S, kind, first, count, B, tmin, mb);
                if (!(live_a & ~done_a) && !(live_b & ~done_b)) break;
            }
        }
        // ---- the next item: the next instance of the current leaf, or a pop ----
        bool finished = false;
        for (;;) {
            if (level == 1 && sp == base) {
                if (inst_next < inst_end) {
                    const int k = inst_next++;
                    float4 fr[4];
                    ld_records_at<4>(S.tinst, (unsigned)(4 * k), fr);
                    const frame3f f = {xyz(fr[0]), xyz(fr[1]), xyz(fr[2]), xyz(fr[3])};
                    ma = inst_a & ~done_a;
                    mb = inst_b & ~done_b;
                    if (!(ma | mb)) continue;
                    A.co = transform_point_inverse(f, A.wo);
                    enter_direction(f, A.wd, live_a & ~done_a, A.cd, A.ci);
                    B.co = transform_point_inverse(f, B.wo);
                    enter_direction(f, B.wd, live_b & ~done_b, B.cd, B.ci);
                    const uint32_t rk = (uint32_t)uniform(ibits(fr[1].w));
                    cur = rk & 0x3fffffffu;
                    kind = (int)(rk >> 30);
                    if (YRT_WIDE_OCTANT) oct = dual_octant(A.ci, live_a & ~done_a, B.ci, live_b & ~done_b);
                    break;
                }
                level = 0;
                A.co = A.wo, A.cd = A.wd, A.ci = A.wi;
                B.co = B.wo, B.cd = B.wd, B.ci = B.wi;
                oct = woct;
            }
            if (sp == 0) {
                finished = true;
                break;
            }
            sp--;
            cur = (uint32_t)__builtin_amdgcn_readlane(s_word, sp);
            ma = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(s_ahi, sp) << 32 |
                  (uint32_t)__builtin_amdgcn_readlane(s_alo, sp)) &
                 ~done_a;
            mb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(s_bhi, sp) << 32 |
                  (uint32_t)__builtin_amdgcn_readlane(s_blo, sp)) &
                 ~done_b;
            if (ma | mb) break;
        }
        if (finished) break;
    }
    occ_a = (done_a & me) != 0;
    occ_b = (done_b & me) != 0;
}

}  // namespace yrt
