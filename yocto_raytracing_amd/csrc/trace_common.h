// trace_common.h -- device-side building blocks shared by the gfx950 kernels:
// the reference's intersection routines (src/scene.cpp:229-382), the two-level
// BVH traversal (src/scene.cpp:386-494) as one flat loop, texture and surface
// evaluation (src/raytrace.cpp:39-86, src/scene.h:159-218) and eval_camera
// (src/raytrace.cpp:6-37). Every floating-point operation is the reference's, in
// its order; this header is only ever compiled with -ffp-contract=off.
#pragma once

#include <hip/hip_runtime.h>

#include "fast_div.h"
#include "yrt_device.h"
#include "yrt_math.h"

namespace yrt {

struct ray3 {
    vec3f o, d;
    float tmin, tmax;
};

struct work_counts {
    unsigned long long box = 0, inst = 0, prim = 0, hits = 0, tex = 0;
    unsigned long long wnode = 0, wprim = 0;  // packet walk: steps of the wave (counted in lane 0)
};

__device__ __forceinline__ float4 ld4(const f4* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ int4 ld4(const i4* p) { return *reinterpret_cast<const int4*>(p); }
// a 16-byte record fetched whole, now: the empty asm consumes all four lanes at this
// point, so the compiler can neither narrow the load to its xyz part nor sink a
// separate load of .w into a later branch (which would put a second dependent memory
// round trip on a traversal step)
__device__ __forceinline__ float4 ld4_whole(const f4* p) {
    float4 v = *reinterpret_cast<const float4*>(p);
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    return v;
}
__device__ __forceinline__ vec3f xyz(float4 v) { return {v.x, v.y, v.z}; }
__device__ __forceinline__ int ibits(float f) { return __float_as_int(f); }
__device__ __forceinline__ uint32_t ubits(float f) { return __float_as_uint(f); }

// intersect_check_bbox (scene.cpp:371-382); invd = 1/ray.d is hoisted per traversal
// (the same value the reference recomputes per call).
// The reference's tmin/tmax are ?: select chains seeded with ray.tmin / ray.tmax:
// with a non-NaN seed such a chain is the maximum (minimum) over the non-NaN slab
// values -- a NaN slab (0*inf) is dropped -- which is exactly what the IEEE maxNum
// / minNum of v_max3_f32 / v_min3_f32 compute, up to the sign of a zero that the
// final <= cannot see. Callers guarantee non-NaN seeds (a NaN seed fails every test
// in the reference, and the traversals return "no hit" up front for it).
// The per-axis swap on invd < 0 stays a select: it must not drop NaNs.
__device__ __forceinline__ bool box_hit6(vec3f o, vec3f invd, float tmin_r, float tmax_r, float lx, float ly,
                                         float lz, float hx, float hy, float hz, float& tnear) {
    float t0x = (lx - o.x) * invd.x, t0y = (ly - o.y) * invd.y, t0z = (lz - o.z) * invd.z;
    float t1x = (hx - o.x) * invd.x, t1y = (hy - o.y) * invd.y, t1z = (hz - o.z) * invd.z;
    if (invd.x < 0) { float t = t0x; t0x = t1x; t1x = t; }
    if (invd.y < 0) { float t = t0y; t0y = t1y; t1y = t; }
    if (invd.z < 0) { float t = t0z; t0z = t1z; t1z = t; }
    float tmin = fmaxf(fmaxf(fmaxf(t0x, t0y), t0z), tmin_r);
    float tmax = fminf(fminf(fminf(t1x, t1y), t1z), tmax_r);
    tmax *= 1.00000024f;
    tnear = tmin;
    return tmin <= tmax;
}

__device__ __forceinline__ bool box_hit(vec3f o, vec3f invd, float tmin_r, float tmax_r, float4 lo, float4 hi,
                                        float& tnear) {
    return box_hit6(o, invd, tmin_r, tmax_r, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, tnear);
}

__device__ __forceinline__ bool box_hit(vec3f o, vec3f invd, float tmin_r, float tmax_r, float4 lo, float4 hi) {
    float tn;
    return box_hit(o, invd, tmin_r, tmax_r, lo, hi, tn);
}

__device__ __forceinline__ bool is_nan(float x) { return !(x == x); }

// intersect_triangle (scene.cpp:229-263) with e1 = v1-v0, e2 = v2-v0 precomputed on
// the host (the same single subtraction the reference performs)
__device__ __forceinline__ bool tri_hit(const ray3& ray, vec3f v0, vec3f e1, vec3f e2, float& dist,
                                        vec4f& ew) {
    vec3f r = cross(ray.d, e2);
    float den = dot(r, e1);
    if (den == 0) return false;
    float inv_den = 1.0f / den;
    vec3f c = ray.o - v0;
    float w1 = dot(r, c) * inv_den;
    if (w1 < 0 || w1 > 1) return false;
    vec3f s = cross(c, e1);
    float w2 = dot(s, ray.d) * inv_den;
    if (w2 < 0.0f || w1 + w2 > 1.0f) return false;
    float t = dot(s, e2) * inv_den;
    if (t < ray.tmin || t > ray.tmax) return false;
    dist = t;
    ew = {1 - w1 - w2, w1, w2, 0};
    return true;
}

// intersect_point (scene.cpp:267-281)
__device__ __forceinline__ bool point_hit(const ray3& ray, vec3f p, float r, float& dist, vec4f& ew) {
    vec3f w = p - ray.o;
    float t = dot(w, ray.d) / dot(ray.d, ray.d);
    if (t < ray.tmin || t > ray.tmax) return false;
    vec3f rp = ray.o + ray.d * t;
    vec3f prp = p - rp;
    if (dot(prp, prp) > r * r) return false;
    dist = t;
    ew = {1, 0, 0, 0};
    return true;
}

// intersect_line (scene.cpp:285-307)
__device__ __forceinline__ bool line_hit(const ray3& ray, vec3f v0, vec3f v1, float r0, float r1, float& dist,
                                         vec4f& ew) {
    vec3f u = ray.d, v = v1 - v0, w = ray.o - v0;
    float a = dot(u, u), b = dot(u, v), c = dot(v, v), d = dot(u, w), e = dot(v, w);
    float det = a * c - b * b;
    if (det == 0) return false;
    float t = (b * e - c * d) / det, s = (a * e - b * d) / det;
    if (t < ray.tmin || t > ray.tmax) return false;
    s = sclamp(s, 0.0f, 1.0f);
    vec3f p0 = ray.o + ray.d * t, p1 = v0 + (v1 - v0) * s;
    vec3f p01 = p0 - p1;
    float r = r0 * (1 - s) + r1 * s;
    if (dot(p01, p01) > r * r) return false;
    dist = t;
    ew = {1 - s, s, 0, 0};
    return true;
}

struct hit_record {
    int slot;  // instance-BVH leaf slot (tinst index), -1 on miss
    int ei;
    vec4f ew;
    float dist;
};

// Both levels of intersect_bvh (scene.cpp:386-479) as ONE loop over one per-lane
// stack, so that lanes at the instance level and lanes inside a shape execute the
// same node-test code together instead of serialising two nested loops.
// Order of work is exactly the reference's: pop; slab test; an inner node pushes
// start, start+1 (start+1 is visited first); an instance leaf visits its instances
// in slot order, each one's shape BVH completely before the next (instances are
// entered with the world tmax current at that moment); a shape leaf tests its
// primitives in slot order, shrinking tmax on every accepted hit.
//   stack: this lane's column in LDS (entry s at stk[s * STRIDE]); instance-level
//   entries are instance-BVH node indices, shape-level entries are node indices
//   relative to the shape's root. Entries above `base` belong to the current shape.
template <bool ANY, bool COUNT, int STRIDE, typename SE>
__device__ __forceinline__ bool traverse(const dev_scene_view& S, ray3 wray, hit_record& hr, SE* stk,
                                         work_counts& wc) {
    // a NaN tmin/tmax fails every slab test of the reference: no node is ever entered
    if (is_nan(wray.tmin) || is_nan(wray.tmax)) return false;
    const vec3f winvd = {1.0f / wray.d.x, 1.0f / wray.d.y, 1.0f / wray.d.z};
    vec3f lo_o = wray.o, linvd = winvd;  // local ray (valid while level == 1)
    vec3f ld = wray.d;
    float ltmax = wray.tmax;
    int level = 0, sp = 0, base = 0;
    int inst_next = 0, inst_end = 0, cur_slot = -1, root = 0, kind = 0;
    bool hit = false;
    stk[0] = (SE)0;
    sp = 1;
    for (;;) {
        if (level == 1 && sp == base) {
            if (inst_next < inst_end) {
                // enter instance `inst_next`: transform_ray_inverse (vmath.h:275-278)
                const int k = inst_next++;
                const f4* ti = S.tinst + 4 * k;
                float4 fx = ld4(ti), fy = ld4(ti + 1), fz = ld4(ti + 2), fo = ld4(ti + 3);
                if (COUNT) wc.inst++;
                frame3f f = {xyz(fx), xyz(fy), xyz(fz), xyz(fo)};
                lo_o = transform_point_inverse(f, wray.o);
                ld = transform_direction_inverse(f, wray.d);
                linvd = {1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z};
                ltmax = wray.tmax;
                int4 sh = ld4(S.shapes + (ibits(fx.w) & (int)inst_shape_mask));
                root = sh.x;
                kind = sh.y;
                cur_slot = k;
                stk[sp * STRIDE] = (SE)0;
                sp++;
                continue;
            }
            level = 0;
        }
        if (sp == 0) break;
        sp--;
        const int e = (int)stk[sp * STRIDE];
        const f4* nb = level ? S.snodes + 2 * (root + e) : S.tnodes + 2 * e;
        float4 lo = ld4(nb), hi = ld4(nb + 1);
        if (COUNT) wc.box++;
        vec3f o = level ? lo_o : wray.o;
        vec3f iv = level ? linvd : winvd;
        float tmax = level ? ltmax : wray.tmax;
        if (is_nan(tmax) || !box_hit(o, iv, wray.tmin, tmax, lo, hi)) continue;
        const int start = ibits(lo.w);
        const uint32_t cl = ubits(hi.w);
        const int count = (int)(cl & 0xffffu);
        if (!(cl & leaf_bit)) {
            // children are stored relative to the shape root at shape level
            for (int c = 0; c < count; c++) {
                stk[sp * STRIDE] = (SE)(start + c);
                sp++;
            }
        } else if (level == 0) {
            inst_next = start;
            inst_end = start + count;
            level = 1;
            base = sp;
        } else {
            ray3 tr = {lo_o, ld, wray.tmin, ltmax};
            bool leaf_hit = false;
            for (int i = start; i < start + count; i++) {
                const f4* pr = S.sprims + 3 * i;
                float4 a = ld4(pr), b = ld4(pr + 1);
                if (COUNT) wc.prim++;
                float t;
                vec4f ew;
                bool h;
                if (kind == kind_triangles) {
                    float4 c = ld4(pr + 2);
                    h = tri_hit(tr, xyz(a), xyz(b), xyz(c), t, ew);
                } else if (kind == kind_lines) {
                    float4 c = ld4(pr + 2);
                    h = line_hit(tr, xyz(a), xyz(b), b.w, c.x, t, ew);
                } else {
                    h = point_hit(tr, xyz(a), b.x, t, ew);
                }
                if (!h) continue;
                hit = leaf_hit = true;
                tr.tmax = t;
                hr.slot = cur_slot;
                hr.ei = ibits(a.w);
                hr.ew = ew;
                hr.dist = t;
                if (ANY) return true;
            }
            // the reference sets tray.tmax = dist after the shape returns a hit; nothing
            // reads the world tmax before that, so updating it here is equivalent
            ltmax = tr.tmax;
            if (leaf_hit) wray.tmax = tr.tmax;
        }
    }
    return hit;
}

// intersect_any (scene.cpp:489-493 -> 446-479 with any = true) on the reference's
// BVH. An any-hit query's answer does not depend on the order in which it visits
// nodes: tmax never shrinks before the first hit returns, so the set of (instance,
// primitive) pairs whose every ancestor box passes is fixed, and the result is
// whether any of them hits. That frees the schedule:
//   * a visited inner node tests BOTH children at once (their 64 B are adjacent),
//     descends into the nearer passing child and pushes the other, so every stack
//     entry is already known to pass and is never re-tested;
//   * shape roots are tested when their instance is entered.
// The boxes tested are exactly the reference's (children of visited nodes, roots).
template <bool COUNT, int STRIDE, typename SE>
__device__ __forceinline__ bool occluded(const dev_scene_view& S, const ray3& wray, SE* stk, work_counts& wc) {
    if (is_nan(wray.tmin) || is_nan(wray.tmax)) return false;
    const vec3f winvd = {1.0f / wray.d.x, 1.0f / wray.d.y, 1.0f / wray.d.z};
    const float tmin_r = wray.tmin, tmax_r = wray.tmax;
    vec3f co = wray.o, ci = winvd;  // ray of the current level
    vec3f ld = wray.d;
    int level = 0, sp = 0, base = 0, root = 0, kind = 0, inst_next = 0, inst_end = 0;
    // the instance-level root
    float4 lo = ld4(S.tnodes), hi = ld4(S.tnodes + 1);
    if (COUNT) wc.box++;
    if (!box_hit(co, ci, tmin_r, tmax_r, lo, hi)) return false;
    int start = ibits(lo.w);
    uint32_t cl = ubits(hi.w);
    for (;;) {
        bool have = false;
        if (!(cl & leaf_bit)) {
            // inner node: its two children are consecutive records
            const f4* nb = level ? S.snodes + 2 * (root + start) : S.tnodes + 2 * start;
            float4 alo = ld4(nb), ahi = ld4(nb + 1), blo = ld4(nb + 2), bhi = ld4(nb + 3);
            if (COUNT) wc.box += 2;
            float ta, tb;
            bool ha = box_hit(co, ci, tmin_r, tmax_r, alo, ahi, ta);
            bool hb = box_hit(co, ci, tmin_r, tmax_r, blo, bhi, tb);
            if (ha && hb) {
                bool a_first = ta <= tb;
                stk[sp * STRIDE] = (SE)(a_first ? start + 1 : start);
                sp++;
                lo = a_first ? alo : blo;
                hi = a_first ? ahi : bhi;
                have = true;
            } else if (ha || hb) {
                lo = ha ? alo : blo;
                hi = ha ? ahi : bhi;
                have = true;
            }
        } else if (level == 0) {
            inst_next = start;
            inst_end = start + (int)(cl & 0xffffu);
            level = 1;
            base = sp;
        } else {
            const int count = (int)(cl & 0xffffu);
            const ray3 lr = {co, ld, tmin_r, tmax_r};
            for (int i = start; i < start + count; i++) {
                const f4* pr = S.sprims + 3 * i;
                float4 a = ld4(pr), b = ld4(pr + 1);
                if (COUNT) wc.prim++;
                float t;
                vec4f ew;
                bool h;
                if (kind == kind_triangles) {
                    float4 c = ld4(pr + 2);
                    h = tri_hit(lr, xyz(a), xyz(b), xyz(c), t, ew);
                } else if (kind == kind_lines) {
                    float4 c = ld4(pr + 2);
                    h = line_hit(lr, xyz(a), xyz(b), b.w, c.x, t, ew);
                } else {
                    h = point_hit(lr, xyz(a), b.x, t, ew);
                }
                if (h) return true;
            }
        }
        while (!have) {
            if (level == 1 && sp == base) {
                if (inst_next < inst_end) {
                    // enter an instance: transform_ray_inverse (vmath.h:275-278), test its shape root
                    const f4* ti = S.tinst + 4 * inst_next++;
                    float4 fx = ld4(ti), fy = ld4(ti + 1), fz = ld4(ti + 2), fo = ld4(ti + 3);
                    if (COUNT) wc.inst++;
                    frame3f f = {xyz(fx), xyz(fy), xyz(fz), xyz(fo)};
                    co = transform_point_inverse(f, wray.o);
                    ld = transform_direction_inverse(f, wray.d);
                    ci = {1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z};
                    int4 sh = ld4(S.shapes + (ibits(fx.w) & (int)inst_shape_mask));
                    root = sh.x;
                    kind = sh.y;
                    lo = ld4(S.snodes + 2 * root);
                    hi = ld4(S.snodes + 2 * root + 1);
                    if (COUNT) wc.box++;
                    have = box_hit(co, ci, tmin_r, tmax_r, lo, hi);
                    continue;
                }
                level = 0;
                co = wray.o;
                ci = winvd;
            }
            if (sp == 0) return false;
            sp--;
            const int e = (int)stk[sp * STRIDE];
            const f4* nb = level ? S.snodes + 2 * (root + e) : S.tnodes + 2 * e;
            lo = ld4(nb);
            hi = ld4(nb + 1);
            have = true;  // tested when it was pushed
        }
        start = ibits(lo.w);
        cl = ubits(hi.w);
    }
}

// specular exponent: the reference calls powf; evaluate in f64 and round once.
// Bases here are >= 0 (max(0, n.h) or sqrt(1-|n.h|)) or NaN. exp2(y*log2(x)) in f64
// carries a relative error of about |y*log2 x| * 2^-52 (< 2^-44 until the result
// underflows f32), so the single rounding to f32 is the correctly rounded powf except
// within ~2^-20 ulp of a rounding boundary -- the same exposure as a full f64 pow at a
// fraction of its cost. pow(x, 0) = 1 for every x (log2(0) * 0 would be NaN).
// the f64 path of powf_cr. Called, not inlined: the f64 log2/exp2 need ~40 VGPRs, which
// inlined would count against the whole shading kernel's budget; as a call, the caller
// spills what it has live around it, and only on the (rare) path that needs it.
__device__ __attribute__((noinline)) float pow_f64_path(float x, float y) {
    return (float)exp2((double)y * log2((double)x));
}
__device__ __forceinline__ float powf_cr(float x, float y) {
    if (y == 0.0f) return 1.0f;
#ifdef YRT_DIAG_POW_F32
    // diagnostic build only (an A/B of what the f64 path costs): NOT the reference's values
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#endif
    // results below 2^-150 round to +0 (the f64 path gives exp2(-inf) = +0 for x = 0).
    // y * log2(x) < -151 by v_log_f32 (error ~2^-23 relative) puts the exact value below
    // -150 with a wide margin.
    if (y > 0.0f && (x == 0.0f || (x >= 0x1p-126f && x < 1.0f && y * __builtin_amdgcn_logf(x) < -151.0f)))
        return 0.0f;
    return pow_f64_path(x, y);
}

// the specular factor pow(x, y) as it multiplies ls = ks * (ke / r^2): when every
// component of ls is +-0 (a material without Ks) and pow(x, y) is finite and >= +0
// (x in [0, 1], y finite), ls * pow == ls * 1 bit for bit, and the pow is skipped.
__device__ __forceinline__ float spec_pow(float x, float y, vec3f ls) {
    if (ls.x == 0.0f && ls.y == 0.0f && ls.z == 0.0f && x >= 0.0f && x <= 1.0f && y >= 0.0f && y <= flt_max)
        return 1.0f;
    return powf_cr(x, y);
}

// lookup_texture + eval_texture (raytrace.cpp:39-86), srgb always on. fmod(u,1)*w in
// double equals the f32 product: the fmod is exact and the product of two floats is
// exact in double, so both round once to the same float. `lut`: the 256-entry srgb
// table (S.srgb, or a copy of it in LDS).
template <bool COUNT>
__device__ __forceinline__ vec3f eval_texture(const dev_scene_view& S, int tex, vec2f uv, work_counts& wc,
                                              const float* lut) {
    int4 ti = ld4(S.texinfo + tex);
    if (COUNT) wc.tex++;
    float w = (float)ti.y, h = (float)ti.z;
    float s = fmodf(uv.x, 1.0f) * w;
    float t = fmodf(uv.y, 1.0f) * h;
    int i = (int)floorf(s);
    int j = (int)floorf(t);
    int i1 = (int)fmodf((float)(i + 1), w);
    int j1 = (int)fmodf((float)(j + 1), h);
    float wi = s - i;
    float wj = t - j;
    int npix = ti.y * ti.z;
    auto texel = [&](int x, int y) -> vec3f {
        // the reference indexes pixels[y*width+x] unchecked (UB for negative uv); clamp
        // the linear index into the image so a bad uv cannot fault the GPU
        int idx = y * ti.y + x;
        idx = idx < 0 ? 0 : (idx >= npix ? npix - 1 : idx);
        uint32_t p = S.texels[ti.x + idx];
        return {lut[p & 0xff], lut[(p >> 8) & 0xff], lut[(p >> 16) & 0xff]};
    };
    vec3f cij = texel(i, j) * (1 - wi) * (1 - wj);
    vec3f ci1j = texel(i1, j) * wi * (1 - wj);
    vec3f cij1 = texel(i, j1) * (1 - wi) * wj;
    vec3f ci1j1 = texel(i1, j1) * wi * wj;
    return cij + ci1j + cij1 + ci1j1;
}

struct surface {
    vec3f p, n;
    vec2f uv;
    int mat, kind;
    int mcls;  // the material's shadow class (yrt_device.h mat_class_shift)
};

#ifndef YRT_FAST_NORMALIZE
#define YRT_FAST_NORMALIZE 1  // shadow-ray setup and shading: normalize / length / ke / r^2 through fast_div.h
#endif

// normalize(a) and length(a) (yrt_math.h, vmath.h:118-122) with fast_div.h's sqrt_nr and
// rcp_nr when every active lane's dot(a, a) is in sqrt_nr's range -- then l lies in
// [2^-48, 2^64), is not 0, and 1/l is normal, where both are bit-identical to sqrtf and
// 1.0f / l -- else the plain calls. Wave-uniform choice: called in any control flow.
__device__ __forceinline__ void normalize_len(vec3f a, vec3f& n, float& len) {
    const float d = dot(a, a);
    if (YRT_FAST_NORMALIZE && !__ballot(!sqrt_nr_ok(d))) {
        len = sqrt_nr(d);
        n = a * rcp_nr(len);
    } else {
        len = length(a);
        n = normalize(a);
    }
}

__device__ __forceinline__ vec3f normalize_w(vec3f a) {
    vec3f n;
    float len;
    normalize_len(a, n, len);
    return n;
}

// eval_pos / eval_norm / eval_texcoord (scene.h:159-218) for the hit (slot, ei, ew)
__device__ __forceinline__ surface eval_surface(const dev_scene_view& S, int slot, int ei, vec4f ew) {
    const f4* ti = S.tinst + 4 * slot;
    float4 fx = ld4(ti), fy = ld4(ti + 1), fz = ld4(ti + 2), fo = ld4(ti + 3);
    frame3f f = {xyz(fx), xyz(fy), xyz(fz), xyz(fo)};
    int4 sh = ld4(S.shapes + (ibits(fx.w) & (int)inst_shape_mask));
    int4 e = ld4(S.elems + sh.z + ei);
    surface sf;
    sf.mat = (int)((uint32_t)ibits(fz.w) & mat_index_mask);
    sf.mcls = (int)((uint32_t)ibits(fz.w) >> mat_class_shift);
    sf.kind = sh.y;
    vec3f lp, ln;
    vec2f luv;
    if (sh.y == kind_points) {
        lp = xyz(ld4(S.vpos + e.x));
        ln = xyz(ld4(S.vnorm + e.x));
        luv = {0, 0};  // points carry no texcoord: the reference reads an empty vector here
    } else if (sh.y == kind_lines) {
        lp = xyz(ld4(S.vpos + e.x)) * ew.x + xyz(ld4(S.vpos + e.y)) * ew.y;
        ln = normalize_w(xyz(ld4(S.vnorm + e.x)) * ew.x + xyz(ld4(S.vnorm + e.y)) * ew.y);
        f2 t0 = S.vuv[e.x], t1 = S.vuv[e.y];
        luv = vec2f{t0.x, t0.y} * ew.x + vec2f{t1.x, t1.y} * ew.y;
    } else {
        lp = xyz(ld4(S.vpos + e.x)) * ew.x + xyz(ld4(S.vpos + e.y)) * ew.y + xyz(ld4(S.vpos + e.z)) * ew.z;
        ln = normalize_w(xyz(ld4(S.vnorm + e.x)) * ew.x + xyz(ld4(S.vnorm + e.y)) * ew.y +
                         xyz(ld4(S.vnorm + e.z)) * ew.z);
        f2 t0 = S.vuv[e.x], t1 = S.vuv[e.y], t2 = S.vuv[e.z];
        luv = vec2f{t0.x, t0.y} * ew.x + vec2f{t1.x, t1.y} * ew.y + vec2f{t2.x, t2.y} * ew.z;
    }
    sf.p = transform_point(f, lp);
    sf.n = normalize_w(transform_vector(f, ln));  // transform_direction
    sf.uv = luv;
    return sf;
}

// uv (raytrace.cpp:236-239) and eval_camera (raytrace.cpp:6-37)
__device__ __forceinline__ ray3 camera_ray(const dev_camera& cam, int W, int H, int ns, int i, int j, int ii,
                                           int jj) {
    float u = (i + (ii + 0.5f) / ns) / W;
    float v = (j + (jj + 0.5f) / ns) / H;
    vec3f q;
    q.x = cam.ox + (u - 0.5f) * cam.w * cam.xx + (v - 0.5f) * cam.h * cam.yx - cam.focus * cam.zx;
    q.y = cam.oy + (u - 0.5f) * cam.w * cam.xy + (v - 0.5f) * cam.h * cam.yy - cam.focus * cam.zy;
    q.z = cam.oz + (u - 0.5f) * cam.w * cam.xz + (v - 0.5f) * cam.h * cam.yz - cam.focus * cam.zz;
    vec3f o = {cam.ox, cam.oy, cam.oz};
    return {o, normalize(q - o), ray_eps, flt_max};
}

// this wave's counter line (yrt_device.h: cnt_slots lines of cnt_count counters)
__device__ __forceinline__ unsigned long long* counter_line(unsigned long long* counters) {
    const unsigned wave = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) +
                          (threadIdx.x >> 6);
    return counters + (size_t)(wave % cnt_slots) * cnt_count;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace yrt
