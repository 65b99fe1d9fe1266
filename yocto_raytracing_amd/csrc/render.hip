// render.hip -- the gfx950 hot path: raytrace() (src/raytrace.cpp:213-254) as one
// thread per pixel, with eval_camera (:6-37), shade (:88-211), eval_texture
// (:39-86) and the two-level BVH queries intersect_first/intersect_any
// (src/scene.cpp:371-494) restated over the HBM layout of yrt_device.h.
//
// Parity contract: every floating-point operation is the
// reference's, in the reference's order, compiled with -ffp-contract=off and HIP's
// correctly rounded fp32 division/sqrt. Traversal replays the reference's stack
// discipline exactly (pop; slab test; inner node pushes start, start+1; leaves in
// slot order), so closest-hit tie-breaking matches. Per pixel the s*s samples are
// summed in the reference's jj-major / ii-minor order. The only libm call left on
// the device is pow() in the specular term, evaluated in f64 and rounded once
// (correctly rounded in all but ~2^-29 of cases, vs glibc powf's <=0.82 ulp).
//
// Mapping to CDNA4: 128-lane workgroups cover 16x8 pixels (each wave64 an 16x4
// tile: neighbouring rays traverse the same nodes); traversal stacks live in LDS,
// one column per lane (stride = workgroup size, conflict-free); nodes, instances
// and primitives are 16-byte records fetched with global_load_dwordx4.
#include <hip/hip_runtime.h>

#include "yrt_render.h"

namespace yrt {
namespace {

constexpr int BLOCK_X = 16, BLOCK_Y = 8, BLOCK = BLOCK_X * BLOCK_Y;
constexpr int MAX_BOUNCES = 16;  // compile-time cap of the per-level shading records

struct ray3 {
    vec3f o, d;
    float tmin, tmax;
};

struct work_counts {
    unsigned long long box = 0, inst = 0, prim = 0, hits = 0, tex = 0;
};

__device__ __forceinline__ float4 ld4(const f4* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ int4 ld4(const i4* p) { return *reinterpret_cast<const int4*>(p); }
__device__ __forceinline__ vec3f xyz(float4 v) { return {v.x, v.y, v.z}; }
__device__ __forceinline__ int ibits(float f) { return __float_as_int(f); }
__device__ __forceinline__ uint32_t ubits(float f) { return __float_as_uint(f); }

// intersect_check_bbox (scene.cpp:371-382); invd is 1/ray.d, hoisted per traversal
__device__ __forceinline__ bool box_hit(const ray3& r, vec3f invd, float4 lo, float4 hi) {
    float t0x = (lo.x - r.o.x) * invd.x, t0y = (lo.y - r.o.y) * invd.y, t0z = (lo.z - r.o.z) * invd.z;
    float t1x = (hi.x - r.o.x) * invd.x, t1y = (hi.y - r.o.y) * invd.y, t1z = (hi.z - r.o.z) * invd.z;
    if (invd.x < 0) { float t = t0x; t0x = t1x; t1x = t; }
    if (invd.y < 0) { float t = t0y; t0y = t1y; t1y = t; }
    if (invd.z < 0) { float t = t0z; t0z = t1z; t1z = t; }
    float tmin = smax(t0z, smax(t0y, smax(t0x, r.tmin)));
    float tmax = smin(t1z, smin(t1y, smin(t1x, r.tmax)));
    tmax *= 1.00000024f;
    return tmin <= tmax;
}

// intersect_triangle (scene.cpp:229-263) with e1 = v1-v0, e2 = v2-v0 precomputed
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
__device__ __forceinline__ bool line_hit(const ray3& ray, vec3f v0, vec3f v1, float r0, float r1,
                                         float& dist, vec4f& ew) {
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

// bottom level: intersect_bvh(shape) (scene.cpp:386-442)
template <bool ANY, bool COUNT>
__device__ bool trace_shape(const dev_scene_view& S, int root, int kind, ray3 tray, float& dist,
                            int& ei, vec4f& ew, int* stk, work_counts& wc) {
    vec3f invd = {1.0f / tray.d.x, 1.0f / tray.d.y, 1.0f / tray.d.z};
    int sp = 0;
    stk[0] = root;
    sp = 1;
    bool hit = false;
    while (sp) {
        int ni = stk[--sp * BLOCK];
        float4 lo = ld4(S.snodes + 2 * ni), hi = ld4(S.snodes + 2 * ni + 1);
        if (COUNT) wc.box++;
        if (!box_hit(tray, invd, lo, hi)) continue;
        int start = ibits(lo.w);
        uint32_t cl = ubits(hi.w);
        int count = (int)(cl & 0xffffu);
        if (!(cl & leaf_bit)) {
            for (int i = start; i < start + count; i++) {
                if (sp < shape_stack_cap) stk[sp * BLOCK] = i;
                sp++;
            }
            if (sp > shape_stack_cap) return hit;  // cannot happen: host checked depth
        } else {
            for (int i = start; i < start + count; i++) {
                float4 a = ld4(S.sprims + 3 * i), b = ld4(S.sprims + 3 * i + 1);
                if (COUNT) wc.prim++;
                bool h;
                if (kind == kind_triangles) {
                    float4 c = ld4(S.sprims + 3 * i + 2);
                    h = tri_hit(tray, xyz(a), xyz(b), xyz(c), dist, ew);
                } else if (kind == kind_lines) {
                    float4 c = ld4(S.sprims + 3 * i + 2);
                    h = line_hit(tray, xyz(a), xyz(b), b.w, c.x, dist, ew);
                } else {
                    h = point_hit(tray, xyz(a), b.x, dist, ew);
                }
                if (!h) continue;
                hit = true;
                tray.tmax = dist;
                ei = ibits(a.w);
                if (ANY) return true;
            }
        }
    }
    return hit;
}

// top level: intersect_bvh(scene) (scene.cpp:446-479). Returns the instance leaf slot.
template <bool ANY, bool COUNT>
__device__ bool trace_scene(const dev_scene_view& S, ray3 tray, int& slot, int& ei, vec4f& ew,
                            float& dist, int* tstk, int* sstk, work_counts& wc) {
    vec3f invd = {1.0f / tray.d.x, 1.0f / tray.d.y, 1.0f / tray.d.z};
    int sp = 0;
    tstk[0] = 0;
    sp = 1;
    bool hit = false;
    while (sp) {
        int ni = tstk[--sp * BLOCK];
        float4 lo = ld4(S.tnodes + 2 * ni), hi = ld4(S.tnodes + 2 * ni + 1);
        if (COUNT) wc.box++;
        if (!box_hit(tray, invd, lo, hi)) continue;
        int start = ibits(lo.w);
        uint32_t cl = ubits(hi.w);
        int count = (int)(cl & 0xffffu);
        if (!(cl & leaf_bit)) {
            for (int i = start; i < start + count; i++) {
                if (sp < top_stack_cap) tstk[sp * BLOCK] = i;
                sp++;
            }
            if (sp > top_stack_cap) return hit;
        } else {
            for (int k = start; k < start + count; k++) {
                float4 fx = ld4(S.tinst + 4 * k), fy = ld4(S.tinst + 4 * k + 1);
                float4 fz = ld4(S.tinst + 4 * k + 2), fo = ld4(S.tinst + 4 * k + 3);
                if (COUNT) wc.inst++;
                frame3f f = {xyz(fx), xyz(fy), xyz(fz), xyz(fo)};
                ray3 lray = {transform_point_inverse(f, tray.o), transform_direction_inverse(f, tray.d),
                             tray.tmin, tray.tmax};  // transform_ray_inverse, vmath.h:275-278
                int4 sh = ld4(S.shapes + ibits(fx.w));
                if (!trace_shape<ANY, COUNT>(S, sh.x, sh.y, lray, dist, ei, ew, sstk, wc)) continue;
                tray.tmax = dist;
                slot = k;
                hit = true;
                if (ANY) return true;
            }
        }
    }
    return hit;
}

// specular exponent: the reference calls powf; evaluate in f64, round once
__device__ __forceinline__ float powf_cr(float x, float y) { return (float)pow((double)x, (double)y); }

// lookup_texture + eval_texture (raytrace.cpp:39-86), srgb always on. fmod(u,1)*w in
// double equals the f32 product here: the fmod is exact and the product of two
// floats is exact in double, so both round once to the same float.
template <bool COUNT>
__device__ vec3f eval_texture(const dev_scene_view& S, int tex, vec2f uv, work_counts& wc) {
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
        return {S.srgb[p & 0xff], S.srgb[(p >> 8) & 0xff], S.srgb[(p >> 16) & 0xff]};
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
};

// eval_pos / eval_norm / eval_texcoord (scene.h:159-218) for the hit (slot, ei, ew)
__device__ surface eval_surface(const dev_scene_view& S, int slot, int ei, vec4f ew) {
    float4 fx = ld4(S.tinst + 4 * slot), fy = ld4(S.tinst + 4 * slot + 1);
    float4 fz = ld4(S.tinst + 4 * slot + 2), fo = ld4(S.tinst + 4 * slot + 3);
    frame3f f = {xyz(fx), xyz(fy), xyz(fz), xyz(fo)};
    int4 sh = ld4(S.shapes + ibits(fx.w));
    int4 e = ld4(S.elems + sh.z + ei);
    surface sf;
    sf.mat = ibits(fz.w);
    sf.kind = sh.y;
    vec3f lp, ln;
    vec2f luv;
    if (sh.y == kind_points) {
        lp = xyz(ld4(S.vpos + e.x));
        ln = xyz(ld4(S.vnorm + e.x));
        luv = {0, 0};  // points carry no texcoord: the reference reads an empty vector here
    } else if (sh.y == kind_lines) {
        lp = xyz(ld4(S.vpos + e.x)) * ew.x + xyz(ld4(S.vpos + e.y)) * ew.y;
        ln = normalize(xyz(ld4(S.vnorm + e.x)) * ew.x + xyz(ld4(S.vnorm + e.y)) * ew.y);
        f2 t0 = S.vuv[e.x], t1 = S.vuv[e.y];
        luv = vec2f{t0.x, t0.y} * ew.x + vec2f{t1.x, t1.y} * ew.y;
    } else {
        lp = xyz(ld4(S.vpos + e.x)) * ew.x + xyz(ld4(S.vpos + e.y)) * ew.y + xyz(ld4(S.vpos + e.z)) * ew.z;
        ln = normalize(xyz(ld4(S.vnorm + e.x)) * ew.x + xyz(ld4(S.vnorm + e.y)) * ew.y +
                       xyz(ld4(S.vnorm + e.z)) * ew.z);
        f2 t0 = S.vuv[e.x], t1 = S.vuv[e.y], t2 = S.vuv[e.z];
        luv = vec2f{t0.x, t0.y} * ew.x + vec2f{t1.x, t1.y} * ew.y + vec2f{t2.x, t2.y} * ew.z;
    }
    sf.p = transform_point(f, lp);
    sf.n = transform_direction(f, ln);
    sf.uv = luv;
    return sf;
}

struct lane_state {
    int* tstk;
    int* sstk;
    work_counts wc;
    unsigned long long rays = 0;
    unsigned long long truncated = 0;
};

// shade() (raytrace.cpp:88-211) with the recursion unrolled: level k records its
// light sum D_k, ambient la_k and kr_k; the result folds back to front as
// R_k = (D_k + R_{k+1}*kr_k) + la_k, the reference's accumulation order (:182,203,206).
template <bool COUNT>
__device__ vec3f shade_path(const dev_scene_view& S, const dev_render_args& A, ray3 ray,
                            lane_state& L) {
    vec3f rec_d[MAX_BOUNCES], rec_la[MAX_BOUNCES], rec_kr[MAX_BOUNCES];
    int depth = 0;
    vec3f R = {0, 0, 0};
    int max_depth = A.max_depth < MAX_BOUNCES ? A.max_depth : MAX_BOUNCES;
    for (;;) {
        int slot = -1, ei = -1;
        vec4f ew = {0, 0, 0, 0};
        float dist = 0;
        L.rays++;
        bool hit = trace_scene<false, COUNT>(S, ray, slot, ei, ew, dist, L.tstk, L.sstk, L.wc);
        if (!hit) {
            R = {0, 0, 0};
            break;
        }
        if (COUNT) L.wc.hits++;
        surface sf = eval_surface(S, slot, ei, ew);
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
            tkd = eval_texture<COUNT>(S, kd_txt, sf.uv, L.wc);
            la = la * tkd;
        }
        if (ks_txt >= 0) tks = eval_texture<COUNT>(S, ks_txt, sf.uv, L.wc);
        vec3f c = {0.0f, 0.0f, 0.0f};
        for (int li = 0; li < S.nlights; li++) {
            const f4* lr = S.lights + 6 * li;
            frame3f lf = {xyz(ld4(lr)), xyz(ld4(lr + 1)), xyz(ld4(lr + 2)), xyz(ld4(lr + 3))};
            vec3f lp0 = xyz(ld4(lr + 4)), ke = xyz(ld4(lr + 5));
            vec3f tp = transform_point(lf, lp0 - sf.p);
            vec3f l = normalize(tp);
            float r = length(tp);
            ray3 sr = {sf.p, l, 0.01f, r - 0.01f};
            int s2 = -1, e2 = -1;
            vec4f w2;
            float d2;
            L.rays++;
            if (trace_scene<true, COUNT>(S, sr, s2, e2, w2, d2, L.tstk, L.sstk, L.wc)) continue;
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
                ls = ls * powf_cr(sinnh, ns);
            } else {
                ld = ld * smax(0.0f, dot(sf.n, l));
                ls = ls * powf_cr(smax(0.0f, dot(sf.n, h)), ns);
            }
            c = c + (ld + ls);
        }
        if (!reflective) {
            R = c + la;
            break;
        }
        if (depth + 1 >= max_depth) {
            // the reference recurses without bound; here the cap counts as a miss
            L.truncated++;
            rec_d[depth] = c;
            rec_la[depth] = la;
            rec_kr[depth] = kr;
            depth++;
            R = {0, 0, 0};
            break;
        }
        rec_d[depth] = c;
        rec_la[depth] = la;
        rec_kr[depth] = kr;
        depth++;
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

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <bool COUNT>
__device__ void flush_counters(unsigned long long* counters, const lane_state& L,
                               unsigned long long samples) {
    unsigned long long vals[9] = {L.rays, samples, L.truncated, 0, L.wc.box, L.wc.inst,
                                  L.wc.prim, L.wc.hits, L.wc.tex};
    int n = COUNT ? 9 : 3;
    for (int k = 0; k < n; k++) {
        unsigned long long s = wave_sum(vals[k]);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(counters + k, s);
    }
}

// raytrace() (raytrace.cpp:213-254) for the window/bands in A; one lane = one pixel
template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void render_kernel(dev_scene_view S, dev_render_args A,
                                                       float4* __restrict__ out,
                                                       unsigned long long* counters) {
    extern __shared__ int lds[];
    lane_state L;
    L.tstk = lds + threadIdx.x;
    L.sstk = lds + top_stack_cap * BLOCK + threadIdx.x;
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
            const dev_camera& cam = A.cam;
            int ns = A.samples;
            vec4f acc = {0, 0, 0, 0};
            for (int jj = 0; jj < ns; jj++) {
                for (int ii = 0; ii < ns; ii++) {
                    // uv (raytrace.cpp:236-239) and eval_camera (:6-37)
                    float u = (i + (ii + 0.5f) / ns) / A.width;
                    float v = (j + (jj + 0.5f) / ns) / A.height;
                    vec3f q;
                    q.x = cam.ox + (u - 0.5f) * cam.w * cam.xx + (v - 0.5f) * cam.h * cam.yx - cam.focus * cam.zx;
                    q.y = cam.oy + (u - 0.5f) * cam.w * cam.xy + (v - 0.5f) * cam.h * cam.yy - cam.focus * cam.zy;
                    q.z = cam.oz + (u - 0.5f) * cam.w * cam.xz + (v - 0.5f) * cam.h * cam.yz - cam.focus * cam.zz;
                    vec3f o = {cam.ox, cam.oy, cam.oz};
                    ray3 ray = {o, normalize(q - o), ray_eps, flt_max};
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
template <bool ANY>
__global__ __launch_bounds__(BLOCK) void trace_kernel(dev_scene_view S, const float* __restrict__ rays,
                                                      int n, unsigned char* hit, int* inst, int* eis,
                                                      float* ews, float* dists,
                                                      unsigned long long* counters) {
    extern __shared__ int lds[];
    int* tstk = lds + threadIdx.x;
    int* sstk = lds + top_stack_cap * BLOCK + threadIdx.x;
    int k = blockIdx.x * BLOCK + threadIdx.x;
    work_counts wc;
    if (k < n) {
        const float* r = rays + (size_t)k * 8;
        ray3 ray = {{r[0], r[1], r[2]}, {r[3], r[4], r[5]}, r[6], r[7]};
        int slot = -1, ei = -1;
        vec4f ew = {0, 0, 0, 0};
        float dist = 0;
        bool h = trace_scene<ANY, false>(S, ray, slot, ei, ew, dist, tstk, sstk, wc);
        hit[k] = h ? 1 : 0;
        if (!ANY) {
            // intersect_first returns a default record on a miss (scene.cpp:485-486)
            inst[k] = h ? ibits(S.tinst[4 * slot + 1].w) : -1;
            eis[k] = h ? ei : -1;
            ews[4 * k + 0] = h ? ew.x : 0;
            ews[4 * k + 1] = h ? ew.y : 0;
            ews[4 * k + 2] = h ? ew.z : 0;
            ews[4 * k + 3] = h ? ew.w : 0;
            dists[k] = h ? dist : 0;
        }
    }
    unsigned long long s = wave_sum(k < n ? 1ull : 0ull);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(counters + cnt_rays, s);
}

// tonemap (image.cpp:55-77): exposure 0, no filmic, gamma 1/2.2, truncating *255
__global__ void tonemap_kernel(const float4* __restrict__ in, int n, uchar4* __restrict__ out) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    float4 h = in[k];
    const float g = 1 / 2.2f;
    float r = powf_cr(h.x, g), gg = powf_cr(h.y, g), b = powf_cr(h.z, g);
    out[k] = make_uchar4((unsigned char)(sclamp(r, 0.0f, 1.0f) * 255),
                         (unsigned char)(sclamp(gg, 0.0f, 1.0f) * 255),
                         (unsigned char)(sclamp(b, 0.0f, 1.0f) * 255),
                         (unsigned char)(sclamp(h.w, 0.0f, 1.0f) * 255));
}

constexpr size_t stack_lds_bytes() { return (size_t)(top_stack_cap + shape_stack_cap) * BLOCK * sizeof(int); }

}  // namespace

hipError_t launch_render(const device_scene& ds, const dev_render_args& args, void* out_rgba,
                         unsigned long long* counters, bool count_work, hipStream_t stream) {
    if (args.tile_w <= 0 || args.tile_h <= 0) return hipSuccess;
    dim3 grid((args.tile_w + BLOCK_X - 1) / BLOCK_X, (args.tile_h + BLOCK_Y - 1) / BLOCK_Y);
    if (count_work)
        hipLaunchKernelGGL(render_kernel<true>, grid, dim3(BLOCK), stack_lds_bytes(), stream, ds.view,
                           args, (float4*)out_rgba, counters);
    else
        hipLaunchKernelGGL(render_kernel<false>, grid, dim3(BLOCK), stack_lds_bytes(), stream, ds.view,
                           args, (float4*)out_rgba, counters);
    return hipGetLastError();
}

hipError_t launch_trace(const device_scene& ds, const float* rays, int n, int any, unsigned char* hit,
                        int* inst, int* ei, float* ew, float* dist, unsigned long long* counters,
                        hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    dim3 grid((n + BLOCK - 1) / BLOCK);
    if (any)
        hipLaunchKernelGGL(trace_kernel<true>, grid, dim3(BLOCK), stack_lds_bytes(), stream, ds.view, rays,
                           n, hit, inst, ei, ew, dist, counters);
    else
        hipLaunchKernelGGL(trace_kernel<false>, grid, dim3(BLOCK), stack_lds_bytes(), stream, ds.view, rays,
                           n, hit, inst, ei, ew, dist, counters);
    return hipGetLastError();
}

hipError_t launch_tonemap(const float* rgba, int n, unsigned char* out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(tonemap_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, (const float4*)rgba, n,
                       (uchar4*)out);
    return hipGetLastError();
}

}  // namespace yrt
