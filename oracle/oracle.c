/* oracle/oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU parity oracle.
 *
 * A plain-C restatement of the reference's hot path, used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg purely as a checker.
 * It is never linked into, called by, or measured as the product (libyrt.so).
 *
 * What it restates (reference = sebcossu/yocto_raytracing, /root/reference/src):
 *   build_bvh / make_node / split_prims       scene.cpp:509-658
 *   intersect_check_bbox                      scene.cpp:371-382
 *   intersect_triangle / _point / _line       scene.cpp:229-307
 *   intersect_bvh (shape, scene)              scene.cpp:386-479
 *   intersect_first / intersect_any           scene.cpp:483-494
 *   eval_pos / eval_norm / eval_texcoord      scene.h:159-218
 *   eval_camera                               raytrace.cpp:6-37
 *   lookup_texture / eval_texture             raytrace.cpp:39-86
 *   shade (recursive, as the reference)       raytrace.cpp:88-211
 *   raytrace (row subset)                     raytrace.cpp:213-254
 * Math follows vmath.h exactly: select-based min/max (vmath.h:215-217),
 * normalize returning its input at length 0 (vmath.h:118-122), the operation
 * order of dot/cross/transform_*, and glibc powf/tanf/sqrtf as the reference
 * calls them. Compiled by gcc with -ffp-contract=off (x86-64 baseline: no FMA).
 *
 * Pinning: tests/test_oracle.py checks this file against the reference itself
 * (oracle/_ref, built from the unmodified sources) -- BVH bytes, per-ray
 * intersection records and rendered float images -- and against the committed
 * golden fixtures in tests/golden/ generated from that build.
 *
 * Input: the .yrtscene interchange file. Rows are rendered in
 * parallel with OpenMP when available; pixels are independent and each is summed
 * in the reference's order, so the result does not depend on the thread count.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;
typedef struct { int x, y; } i2;
typedef struct { int x, y, z; } i3;
typedef struct { v3 x, y, z, o; } frame;
typedef struct { v3 min, max; } bbox;
typedef struct { v3 o, d; float tmin, tmax; } ray;

/* bvh_node, scene.h:9-15 (same 32-byte layout) */
typedef struct {
    bbox box;
    uint32_t start;
    uint16_t count;
    uint8_t isleaf;
    uint8_t axis;
} node;

typedef struct {
    node* nodes;
    int nnodes, cap;
    int* leaf;
    int nleaf;
} bvh;

typedef struct {
    int npos, nnorm, ntc, nrad, npts, nlines, ntris;
    v3 *pos, *norm;
    v2* tc;
    float* rad;
    int* pts;
    i2* lines;
    i3* tris;
    bvh tree;
} shape;

typedef struct { v3 ke, kd, ks, kr; float rs; int kd_txt, ks_txt; } material;
typedef struct { frame f; int shp, mat; } instance;
typedef struct { frame f; float fovy, aspect, aperture, focus; } camera;
typedef struct { int w, h; unsigned char* rgba; } texture;

typedef struct {
    int ncam, ntex, nmat, nshp, nist;
    camera* cams;
    texture* texs;
    material* mats;
    shape* shps;
    instance* ists;
    bvh tree;
    /* the instances shade()'s light loop acts on (material ke > 0 in every component), in
     * instance order: the loop over all instances skips the others without effect, so
     * visiting only these is the same computation (raytrace.cpp:121-125) */
    int nlight;
    int* light;
} scene;

/* ---------------- vmath.h ---------------- */
static v3 add(v3 a, v3 b) { v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static v3 sub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static v3 mul(v3 a, v3 b) { v3 r = {a.x * b.x, a.y * b.y, a.z * b.z}; return r; }
static v3 muls(v3 a, float b) { v3 r = {a.x * b, a.y * b, a.z * b}; return r; }
static v3 divs(v3 a, float b) { v3 r = {a.x / b, a.y / b, a.z / b}; return r; }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 cross(v3 a, v3 b) {
    v3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}
static float length(v3 a) { return sqrtf(dot(a, a)); }
static v3 normalize(v3 a) {
    float l = length(a);
    if (l == 0) return a;
    return muls(a, 1 / l);
}
static float fminsel(float x, float y) { return (x < y) ? x : y; }
static float fmaxsel(float x, float y) { return (x > y) ? x : y; }
static float clampsel(float x, float a, float b) { return fminsel(fmaxsel(x, a), b); }
static v3 xform_point(const frame* a, v3 b) {
    return add(add(add(muls(a->x, b.x), muls(a->y, b.y)), muls(a->z, b.z)), a->o);
}
static v3 xform_vector(const frame* a, v3 b) { return add(add(muls(a->x, b.x), muls(a->y, b.y)), muls(a->z, b.z)); }
static v3 xform_point_inv(const frame* a, v3 b) {
    v3 bo = sub(b, a->o);
    v3 r = {dot(a->x, bo), dot(a->y, bo), dot(a->z, bo)};
    return r;
}
static v3 xform_dir_inv(const frame* a, v3 b) {
    v3 r = {dot(a->x, b), dot(a->y, b), dot(a->z, b)};
    return normalize(r);
}
static const bbox invalid_box = {{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}};
static bbox expand_pt(bbox a, v3 b) {
    bbox r = {{fminsel(a.min.x, b.x), fminsel(a.min.y, b.y), fminsel(a.min.z, b.z)},
              {fmaxsel(a.max.x, b.x), fmaxsel(a.max.y, b.y), fmaxsel(a.max.z, b.z)}};
    return r;
}
static bbox expand_box(bbox a, bbox b) {
    bbox r = {{fminsel(a.min.x, b.min.x), fminsel(a.min.y, b.min.y), fminsel(a.min.z, b.min.z)},
              {fmaxsel(a.max.x, b.max.x), fmaxsel(a.max.y, b.max.y), fmaxsel(a.max.z, b.max.z)}};
    return r;
}
static float axis_val(v3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

/* ---------------- build_bvh (scene.cpp:509-658) ---------------- */
typedef struct { bbox box; v3 center; int pid; } bprim;

static int split_prims(bprim* p, int start, int end, int* axis, int* mid) {
    bbox cb = invalid_box;
    for (int i = start; i < end; i++) cb = expand_pt(cb, p[i].center);
    v3 size = sub(cb.max, cb.min);
    if (size.x == 0 && size.y == 0 && size.z == 0) return 0;
    if (size.x >= size.y && size.x >= size.z) *axis = 0;
    else if (size.y >= size.x && size.y >= size.z) *axis = 1;
    else *axis = 2;
    v3 halfv = divs(add(cb.min, cb.max), 2);
    float half = axis_val(halfv, *axis);
    /* std::partition on a bidirectional range: two-sided swap partition */
    int first = start, last = end;
    for (;;) {
        for (;;) {
            if (first == last) { *mid = first; return 1; }
            if (axis_val(p[first].center, *axis) < half) first++;
            else break;
        }
        last--;
        for (;;) {
            if (first == last) { *mid = first; return 1; }
            if (!(axis_val(p[last].center, *axis) < half)) last--;
            else break;
        }
        bprim t = p[first]; p[first] = p[last]; p[last] = t;
        first++;
    }
}

static int make_node(bvh* t, int nid, bprim* p, int start, int end) {
    bbox b = invalid_box;
    for (int i = start; i < end; i++) b = expand_box(b, p[i].box);
    int split = 0, axis = -1, mid = -1;
    if (end - start > 4) split = split_prims(p, start, end, &axis, &mid);
    if (split && (mid <= start || mid >= end)) return -1; /* reference would recurse forever */
    t->nodes[nid].box = b;
    if (!split) {
        t->nodes[nid].isleaf = 1;
        t->nodes[nid].start = (uint32_t)start;
        t->nodes[nid].count = (uint16_t)(end - start);
        return 0;
    }
    int first = t->nnodes;
    t->nodes[nid].isleaf = 0;
    t->nodes[nid].axis = (uint8_t)axis;
    t->nodes[nid].start = (uint32_t)first;
    t->nodes[nid].count = 2;
    memset(&t->nodes[t->nnodes], 0, 2 * sizeof(node));
    t->nnodes += 2;
    if (make_node(t, first, p, start, mid) < 0) return -1;
    return make_node(t, first + 1, p, mid, end);
}

static int build_tree(bvh* t, bprim* p, int n) {
    t->cap = 2 * n + 2;
    t->nodes = (node*)calloc((size_t)t->cap, sizeof(node));
    t->nnodes = 1;
    if (make_node(t, 0, p, 0, n) < 0) return -1;
    t->leaf = (int*)malloc(sizeof(int) * (size_t)(n ? n : 1));
    t->nleaf = n;
    for (int i = 0; i < n; i++) t->leaf[i] = p[i].pid;
    return 0;
}

static bbox pad_box(bbox b, v3 p, float r) {
    v3 rr = {r, r, r};
    bbox e = {sub(p, rr), add(p, rr)};
    return expand_box(b, e);
}

static bbox box_to_world(const frame* f, bbox b) {
    v3 c[8] = {{b.min.x, b.min.y, b.min.z}, {b.min.x, b.min.y, b.max.z}, {b.min.x, b.max.y, b.min.z},
               {b.min.x, b.max.y, b.max.z}, {b.max.x, b.min.y, b.min.z}, {b.max.x, b.min.y, b.max.z},
               {b.max.x, b.max.y, b.min.z}, {b.max.x, b.max.y, b.max.z}};
    bbox r = invalid_box;
    for (int i = 0; i < 8; i++) r = expand_pt(r, xform_point(f, c[i]));
    return r;
}

static int build_scene_bvh(scene* s) {
    for (int si = 0; si < s->nshp; si++) {
        shape* sh = &s->shps[si];
        int n = sh->npts + sh->nlines + sh->ntris, k = 0;
        bprim* p = (bprim*)malloc(sizeof(bprim) * (size_t)(n ? n : 1));
        for (int ei = 0; ei < sh->npts; ei++, k++) {
            int e = sh->pts[ei];
            bbox b = pad_box(invalid_box, sh->pos[e], sh->rad[e]);
            p[k].box = b; p[k].center = divs(add(b.min, b.max), 2.0f); p[k].pid = ei;
        }
        for (int ei = 0; ei < sh->nlines; ei++, k++) {
            i2 e = sh->lines[ei];
            bbox b = pad_box(invalid_box, sh->pos[e.x], sh->rad[e.x]);
            b = pad_box(b, sh->pos[e.y], sh->rad[e.y]);
            p[k].box = b; p[k].center = divs(add(b.min, b.max), 2.0f); p[k].pid = ei;
        }
        for (int ei = 0; ei < sh->ntris; ei++, k++) {
            i3 e = sh->tris[ei];
            bbox b = pad_box(invalid_box, sh->pos[e.x], 0);
            b = pad_box(b, sh->pos[e.y], 0);
            b = pad_box(b, sh->pos[e.z], 0);
            p[k].box = b; p[k].center = divs(add(b.min, b.max), 2.0f); p[k].pid = ei;
        }
        int rc = build_tree(&sh->tree, p, n);
        free(p);
        if (rc < 0) return -1;
    }
    bprim* p = (bprim*)malloc(sizeof(bprim) * (size_t)(s->nist ? s->nist : 1));
    for (int ii = 0; ii < s->nist; ii++) {
        bbox b = box_to_world(&s->ists[ii].f, s->shps[s->ists[ii].shp].tree.nodes[0].box);
        p[ii].box = b; p[ii].center = divs(add(b.min, b.max), 2.0f); p[ii].pid = ii;
    }
    int rc = build_tree(&s->tree, p, s->nist);
    free(p);
    return rc;
}

/* ---------------- intersections (scene.cpp:229-307, 371-382) ---------------- */
static int hit_tri(const ray* r, v3 v0, v3 v1, v3 v2, float* dist, v4* ew) {
    v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    v3 rr = cross(r->d, e2);
    float den = dot(rr, e1);
    if (den == 0) return 0;
    float inv_den = 1.0f / den;
    v3 c = sub(r->o, v0);
    float w1 = dot(rr, c) * inv_den;
    if (w1 < 0 || w1 > 1) return 0;
    v3 s = cross(c, e1);
    float w2 = dot(s, r->d) * inv_den;
    if (w2 < 0.0 || w1 + w2 > 1.0) return 0;
    float t = dot(s, e2) * inv_den;
    if (t < r->tmin || t > r->tmax) return 0;
    *dist = t;
    ew->x = 1 - w1 - w2; ew->y = w1; ew->z = w2; ew->w = 0;
    return 1;
}

static int hit_point(const ray* r, v3 p, float rad, float* dist, v4* ew) {
    v3 w = sub(p, r->o);
    float t = dot(w, r->d) / dot(r->d, r->d);
    if (t < r->tmin || t > r->tmax) return 0;
    v3 rp = add(r->o, muls(r->d, t));
    v3 prp = sub(p, rp);
    if (dot(prp, prp) > rad * rad) return 0;
    *dist = t;
    ew->x = 1; ew->y = 0; ew->z = 0; ew->w = 0;
    return 1;
}

static int hit_line(const ray* r, v3 v0, v3 v1, float r0, float r1, float* dist, v4* ew) {
    v3 u = r->d, v = sub(v1, v0), w = sub(r->o, v0);
    float a = dot(u, u), b = dot(u, v), c = dot(v, v), d = dot(u, w), e = dot(v, w);
    float det = a * c - b * b;
    if (det == 0) return 0;
    float t = (b * e - c * d) / det, s = (a * e - b * d) / det;
    if (t < r->tmin || t > r->tmax) return 0;
    s = clampsel(s, (float)0, (float)1);
    v3 p0 = add(r->o, muls(r->d, t)), p1 = add(v0, muls(sub(v1, v0), s));
    v3 p01 = sub(p0, p1);
    float rr = r0 * (1 - s) + r1 * s;
    if (dot(p01, p01) > rr * rr) return 0;
    *dist = t;
    ew->x = 1 - s; ew->y = s; ew->z = 0; ew->w = 0;
    return 1;
}

static int hit_box(const ray* r, bbox b) {
    v3 invd = {1.0f / r->d.x, 1.0f / r->d.y, 1.0f / r->d.z};
    v3 t0 = mul(sub(b.min, r->o), invd), t1 = mul(sub(b.max, r->o), invd);
    float t;
    if (invd.x < 0) { t = t0.x; t0.x = t1.x; t1.x = t; }
    if (invd.y < 0) { t = t0.y; t0.y = t1.y; t1.y = t; }
    if (invd.z < 0) { t = t0.z; t0.z = t1.z; t1.z = t; }
    float tmin = fmaxsel(t0.z, fmaxsel(t0.y, fmaxsel(t0.x, r->tmin)));
    float tmax = fminsel(t1.z, fminsel(t1.y, fminsel(t1.x, r->tmax)));
    tmax *= 1.00000024f;
    return tmin <= tmax;
}

/* intersect_bvh(shape) scene.cpp:386-442 */
static int trace_shape(const shape* shp, const ray* rin, int any, float* dist, int* ei, v4* ew) {
    int stack[64], cur = 0;
    stack[cur++] = 0;
    ray tr = *rin;
    int hit = 0;
    while (cur) {
        node n = shp->tree.nodes[stack[--cur]];
        if (!hit_box(&tr, n.box)) continue;
        if (!n.isleaf) {
            for (uint32_t i = n.start; i < n.start + n.count; i++) stack[cur++] = (int)i;
        } else if (shp->ntris) {
            for (uint32_t i = n.start; i < n.start + n.count; i++) {
                i3 e = shp->tris[shp->tree.leaf[i]];
                if (!hit_tri(&tr, shp->pos[e.x], shp->pos[e.y], shp->pos[e.z], dist, ew)) continue;
                hit = 1; tr.tmax = *dist; *ei = shp->tree.leaf[i];
                if (any) return 1;
            }
        } else if (shp->nlines) {
            for (uint32_t i = n.start; i < n.start + n.count; i++) {
                i2 e = shp->lines[shp->tree.leaf[i]];
                if (!hit_line(&tr, shp->pos[e.x], shp->pos[e.y], shp->rad[e.x], shp->rad[e.y], dist, ew)) continue;
                hit = 1; tr.tmax = *dist; *ei = shp->tree.leaf[i];
                if (any) return 1;
            }
        } else if (shp->npts) {
            for (uint32_t i = n.start; i < n.start + n.count; i++) {
                int e = shp->pts[shp->tree.leaf[i]];
                if (!hit_point(&tr, shp->pos[e], shp->rad[e], dist, ew)) continue;
                hit = 1; tr.tmax = *dist; *ei = shp->tree.leaf[i];
                if (any) return 1;
            }
        }
    }
    return hit;
}

/* intersect_bvh(scene) scene.cpp:446-479 */
static int trace_scene(const scene* s, const ray* rin, int any, float* dist, int* ist, int* ei, v4* ew) {
    int stack[64], cur = 0;
    stack[cur++] = 0;
    ray tr = *rin;
    int hit = 0;
    while (cur) {
        node n = s->tree.nodes[stack[--cur]];
        if (!hit_box(&tr, n.box)) continue;
        if (!n.isleaf) {
            for (uint32_t i = n.start; i < n.start + n.count; i++) stack[cur++] = (int)i;
        } else {
            for (uint32_t i = n.start; i < n.start + n.count; i++) {
                int ii = s->tree.leaf[i];
                const instance* is = &s->ists[ii];
                ray lr;
                lr.o = xform_point_inv(&is->f, tr.o);
                lr.d = xform_dir_inv(&is->f, tr.d);
                lr.tmin = tr.tmin;
                lr.tmax = tr.tmax;
                if (!trace_shape(&s->shps[is->shp], &lr, any, dist, ei, ew)) continue;
                tr.tmax = *dist; *ist = ii; hit = 1;
                if (any) return 1;
            }
        }
    }
    return hit;
}

/* ---------------- shading (raytrace.cpp) ---------------- */
static v3 lookup_tex(const texture* t, int i, int j) {
    const unsigned char* p = t->rgba + ((size_t)j * t->w + i) * 4;
    float gamma = 2.2f;
    v3 v;
    v.x = fminf(1.0f, powf((float)p[0] / 255.0f, gamma));
    v.y = fminf(1.0f, powf((float)p[1] / 255.0f, gamma));
    v.z = fminf(1.0f, powf((float)p[2] / 255.0f, gamma));
    return v;
}

static v3 eval_tex(const texture* t, v2 uv) {
    float w = (float)t->w, h = (float)t->h;
    float s = (float)(fmod((double)uv.x, 1.0) * (double)w);
    float tt = (float)(fmod((double)uv.y, 1.0) * (double)h);
    int i = (int)floorf(s), j = (int)floorf(tt);
    int i1 = (int)fmod((double)(i + 1), (double)w), j1 = (int)fmod((double)(j + 1), (double)h);
    float wi = s - i, wj = tt - j;
    v3 cij = muls(muls(lookup_tex(t, i, j), 1 - wi), 1 - wj);
    v3 ci1j = muls(muls(lookup_tex(t, i1, j), wi), 1 - wj);
    v3 cij1 = muls(muls(lookup_tex(t, i, j1), 1 - wi), wj);
    v3 ci1j1 = muls(muls(lookup_tex(t, i1, j1), wi), wj);
    return add(add(add(cij, ci1j), cij1), ci1j1);
}

typedef struct { long long rays; int max_depth; long long truncated; } ctx;

static v3 shade(const scene* s, v3 amb, const ray* r, int depth, ctx* cx) {
    float dist = 0;
    int ii = -1, ei = -1;
    v4 ew = {0, 0, 0, 0};
    v3 zero = {0, 0, 0};
    cx->rays++;
    if (!trace_scene(s, r, 0, &dist, &ii, &ei, &ew)) return zero;
    const instance* is = &s->ists[ii];
    const shape* sh = &s->shps[is->shp];
    const material* m = &s->mats[is->mat];
    /* eval_norm / eval_pos / eval_texcoord (scene.h:159-218), points first */
    v3 ln, lp;
    v2 uv = {0, 0};
    if (sh->npts) {
        int p = sh->pts[ei];
        lp = sh->pos[p];
        ln = sh->norm[p];
        if (sh->ntc) uv = sh->tc[p];
    } else if (sh->nlines) {
        i2 l = sh->lines[ei];
        lp = add(muls(sh->pos[l.x], ew.x), muls(sh->pos[l.y], ew.y));
        ln = normalize(add(muls(sh->norm[l.x], ew.x), muls(sh->norm[l.y], ew.y)));
        if (sh->ntc) {
            uv.x = sh->tc[l.x].x * ew.x + sh->tc[l.y].x * ew.y;
            uv.y = sh->tc[l.x].y * ew.x + sh->tc[l.y].y * ew.y;
        }
    } else {
        i3 t = sh->tris[ei];
        lp = add(add(muls(sh->pos[t.x], ew.x), muls(sh->pos[t.y], ew.y)), muls(sh->pos[t.z], ew.z));
        ln = normalize(add(add(muls(sh->norm[t.x], ew.x), muls(sh->norm[t.y], ew.y)), muls(sh->norm[t.z], ew.z)));
        if (sh->ntc) {
            uv.x = sh->tc[t.x].x * ew.x + sh->tc[t.y].x * ew.y + sh->tc[t.z].x * ew.z;
            uv.y = sh->tc[t.x].y * ew.x + sh->tc[t.y].y * ew.y + sh->tc[t.z].y * ew.z;
        }
    }
    v3 n = normalize(xform_vector(&is->f, ln));
    v3 p = xform_point(&is->f, lp);
    v3 c = {0.0f, 0.0f, 0.0f};
    const texture* tkd = m->kd_txt >= 0 ? &s->texs[m->kd_txt] : 0;
    const texture* tks = m->ks_txt >= 0 ? &s->texs[m->ks_txt] : 0;
    v3 la = mul(amb, m->kd);
    if (tkd) la = mul(la, eval_tex(tkd, uv));
    for (int lk = 0; lk < s->nlight; lk++) {
        const instance* L = &s->ists[s->light[lk]];
        v3 ke = s->mats[L->mat].ke;
        v3 lpos = s->shps[L->shp].pos[0];
        v3 l = normalize(xform_point(&L->f, sub(lpos, p)));
        float rr = length(xform_point(&L->f, sub(lpos, p)));
        ray sr = {p, l, 0.01f, rr - 0.01f};
        float d2;
        int i2_, e2;
        v4 w2;
        cx->rays++;
        if (trace_scene(s, &sr, 1, &d2, &i2_, &e2, &w2)) continue;
        float rs = m->rs;
        float ns = (rs != 0) ? 2 / powf(rs, 4.0f) - 2 : 1e6f;
        v3 v = normalize(sub(r->o, p));
        v3 h = normalize(add(v, l));
        v3 kd = m->kd, ks = m->ks;
        if (tkd) kd = mul(kd, eval_tex(tkd, uv));
        if (tks) ks = mul(ks, eval_tex(tks, uv));
        v3 ld = mul(kd, divs(ke, rr * rr));
        v3 ls = mul(ks, divs(ke, rr * rr));
        if (sh->nlines) {
            float pnl = dot(n, l), pnh = dot(n, h);
            if (pnl < 0.0f) pnl *= -1;
            if (pnh < 0.0f) pnh *= -1;
            float sinnl = sqrtf(1.0f - pnl), sinnh = sqrtf(1.0f - pnh);
            ld = muls(ld, sinnl);
            ls = muls(ls, powf(sinnh, ns));
        } else {
            ld = muls(ld, fmaxsel(0.0f, dot(n, l)));
            ls = muls(ls, powf(fmaxsel(0.0f, dot(n, h)), ns));
        }
        c = add(c, add(ld, ls));
    }
    v3 kr = m->kr;
    if (kr.x > 0.0f || kr.y > 0.0f || kr.z > 0.0f) {
        v3 col = zero;
        if (cx->max_depth > 0 && depth + 1 >= cx->max_depth) {
            cx->truncated++;
        } else {
            v3 v = normalize(sub(r->o, p));
            v3 dr = sub(muls(muls(n, 2.0f), dot(n, v)), v);
            ray nr = {p, dr, 1e-4f, FLT_MAX};
            col = shade(s, amb, &nr, depth + 1, cx);
        }
        v3 t = {col.x * kr.x, col.y * kr.y, col.z * kr.z};
        c = add(c, t);
    }
    return add(c, la);
}

static ray eval_camera(const camera* cam, float u, float v) {
    v3 o = cam->f.o, x = cam->f.x, y = muls(cam->f.y, -1), z = cam->f.z;
    float h = 2.0f * cam->focus * tanf(cam->fovy / 2.0f);
    float w = h * cam->aspect;
    float focus = cam->focus;
    v3 q;
    q.x = o.x + (u - 0.5f) * w * x.x + (v - 0.5f) * h * y.x - focus * z.x;
    q.y = o.y + (u - 0.5f) * w * x.y + (v - 0.5f) * h * y.y - focus * z.y;
    q.z = o.z + (u - 0.5f) * w * x.z + (v - 0.5f) * h * y.z - focus * z.z;
    ray r = {o, normalize(sub(q, o)), 1e-4f, FLT_MAX};
    return r;
}

/* ---------------- .yrtscene reader ---------------- */
static int rd(gzFile f, void* p, size_t n) { return n == 0 || gzread(f, p, (unsigned)n) == (int)n; }
static int rdu(gzFile f, uint32_t* v) { return rd(f, v, 4); }
static void* rdvec(gzFile f, int* n, size_t elem, int* ok) {
    uint32_t c = 0;
    if (!rdu(f, &c) || c > (1u << 28)) { *ok = 0; *n = 0; return 0; }
    *n = (int)c;
    void* p = malloc(elem * (c ? c : 1));
    if (!rd(f, p, elem * c)) *ok = 0;
    return p;
}

void oracle_free(void* vs);

void* oracle_load(const char* path) {
    gzFile f = gzopen(path, "rb");
    if (!f) return 0;
    scene* s = (scene*)calloc(1, sizeof(scene));
    char magic[8];
    int ok = rd(f, magic, 8) && memcmp(magic, "YRTSCN1", 8) == 0;
    uint32_t n = 0;
    ok = ok && rdu(f, &n);
    s->ncam = (int)n;
    s->cams = (camera*)calloc(n ? n : 1, sizeof(camera));
    for (uint32_t i = 0; ok && i < n; i++) ok = rd(f, &s->cams[i], sizeof(camera));
    ok = ok && rdu(f, &n);
    s->ntex = (int)n;
    s->texs = (texture*)calloc(n ? n : 1, sizeof(texture));
    for (uint32_t i = 0; ok && i < n; i++) {
        ok = rd(f, &s->texs[i].w, 4) && rd(f, &s->texs[i].h, 4);
        size_t bytes = (size_t)s->texs[i].w * s->texs[i].h * 4;
        s->texs[i].rgba = (unsigned char*)malloc(bytes ? bytes : 1);
        ok = ok && rd(f, s->texs[i].rgba, bytes);
    }
    ok = ok && rdu(f, &n);
    s->nmat = (int)n;
    s->mats = (material*)calloc(n ? n : 1, sizeof(material));
    for (uint32_t i = 0; ok && i < n; i++) ok = rd(f, &s->mats[i], sizeof(material));
    ok = ok && rdu(f, &n);
    s->nshp = (int)n;
    s->shps = (shape*)calloc(n ? n : 1, sizeof(shape));
    for (uint32_t i = 0; ok && i < n; i++) {
        shape* sh = &s->shps[i];
        sh->pos = (v3*)rdvec(f, &sh->npos, sizeof(v3), &ok);
        sh->norm = (v3*)rdvec(f, &sh->nnorm, sizeof(v3), &ok);
        sh->tc = (v2*)rdvec(f, &sh->ntc, sizeof(v2), &ok);
        sh->rad = (float*)rdvec(f, &sh->nrad, sizeof(float), &ok);
        sh->pts = (int*)rdvec(f, &sh->npts, sizeof(int), &ok);
        sh->lines = (i2*)rdvec(f, &sh->nlines, sizeof(i2), &ok);
        sh->tris = (i3*)rdvec(f, &sh->ntris, sizeof(i3), &ok);
    }
    ok = ok && rdu(f, &n);
    s->nist = (int)n;
    s->ists = (instance*)calloc(n ? n : 1, sizeof(instance));
    for (uint32_t i = 0; ok && i < n; i++) ok = rd(f, &s->ists[i], sizeof(instance));
    gzclose(f);
    s->light = (int*)calloc(n ? n : 1, sizeof(int));
    for (uint32_t i = 0; ok && i < n; i++) {
        const instance* L = &s->ists[i];
        if (L->mat < 0 || L->mat >= s->nmat) continue;
        const v3 ke = s->mats[L->mat].ke;
        if (ke.x > 0.0f && ke.y > 0.0f && ke.z > 0.0f) s->light[s->nlight++] = (int)i;
    }
    if (!ok || build_scene_bvh(s) < 0) {
        oracle_free(s);
        return 0;
    }
    return s;
}

void oracle_free(void* vs) {
    scene* s = (scene*)vs;
    if (!s) return;
    for (int i = 0; i < s->ntex; i++) free(s->texs[i].rgba);
    for (int i = 0; i < s->nshp; i++) {
        shape* sh = &s->shps[i];
        free(sh->pos); free(sh->norm); free(sh->tc); free(sh->rad); free(sh->pts); free(sh->lines);
        free(sh->tris); free(sh->tree.nodes); free(sh->tree.leaf);
    }
    free(s->cams); free(s->texs); free(s->mats); free(s->shps); free(s->ists); free(s->light);
    free(s->tree.nodes); free(s->tree.leaf);
    free(s);
}

static void put_tree(gzFile f, const bvh* t) {
    uint32_t n = (uint32_t)t->nnodes;
    gzwrite(f, &n, 4);
    if (n) gzwrite(f, t->nodes, n * (unsigned)sizeof(node));
    n = (uint32_t)t->nleaf;
    gzwrite(f, &n, 4);
    if (n) gzwrite(f, t->leaf, n * 4u);
}

/* .yrtbvh, same bytes as the reference harness writes */
int oracle_write_bvh(void* vs, const char* path) {
    scene* s = (scene*)vs;
    gzFile f = gzopen(path, "wb6");
    if (!f) return -1;
    gzwrite(f, "YRTBVH1", 8);
    uint32_t n = (uint32_t)s->nshp;
    gzwrite(f, &n, 4);
    for (int i = 0; i < s->nshp; i++) put_tree(f, &s->shps[i].tree);
    put_tree(f, &s->tree);
    gzclose(f);
    return 0;
}

int oracle_image_size(void* vs, int cami, int resolution, int* w, int* h) {
    scene* s = (scene*)vs;
    if (cami < 0 || cami >= s->ncam) return -1;
    *w = (int)roundf(s->cams[cami].aspect * resolution);
    *h = resolution;
    return 0;
}

/* threads of the OpenMP loops below (row-parallel render, ray-parallel trace); returns
 * the count in effect. The reference is single-threaded: 1 is its equivalent. */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* raytrace() (raytrace.cpp:213-254) for image rows rows[0..nrows) and columns
 * [x0, x0+ncols); width 0 -> round(aspect*res). out: nrows*ncols*4 floats.
 * max_depth 0 = unbounded recursion (the reference). Returns rays traced
 * (negative on error); *truncated gets the number of depth-capped paths. */
long long oracle_render_rows(void* vs, float amb, int cami, int resolution, int width, int samples,
                             int max_depth, const int* rows, int nrows, int x0, int ncols, float* out,
                             long long* truncated) {
    scene* s = (scene*)vs;
    if (cami < 0 || cami >= s->ncam || samples <= 0) return -1;
    const camera* cam = &s->cams[cami];
    int W = width > 0 ? width : (int)roundf(cam->aspect * resolution), H = resolution;
    v3 a = {amb, amb, amb};
    long long rays = 0, trunc = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : rays, trunc)
    for (int r = 0; r < nrows; r++) {
        int j = rows[r];
        ctx cx = {0, max_depth, 0};
        for (int c = 0; c < ncols; c++) {
            int i = x0 + c;
            v4 acc = {0, 0, 0, 0};
            for (int jj = 0; jj < samples; jj++) {
                for (int ii = 0; ii < samples; ii++) {
                    float u = (i + (ii + 0.5f) / samples) / W;
                    float v = (j + (jj + 0.5f) / samples) / H;
                    ray ry = eval_camera(cam, u, v);
                    v3 col = shade(s, a, &ry, 0, &cx);
                    acc.x = acc.x + col.x;
                    acc.y = acc.y + col.y;
                    acc.z = acc.z + col.z;
                    acc.w = acc.w + 1.0f;
                }
            }
            float* px = out + ((size_t)r * ncols + c) * 4;
            px[0] = acc.x / (float)(samples * samples);
            px[1] = acc.y / (float)(samples * samples);
            px[2] = acc.z / (float)(samples * samples);
            px[3] = 1.0f;
        }
        rays += cx.rays;
        trunc += cx.truncated;
    }
    if (truncated) *truncated = trunc;
    return rays;
}

/* camera ray of pixel (i,j) sub-sample (ii,jj): o.xyz d.xyz tmin tmax */
int oracle_camera_ray(void* vs, int cami, int resolution, int width, int samples, int i, int j, int ii,
                      int jj, float* ray8) {
    scene* s = (scene*)vs;
    if (cami < 0 || cami >= s->ncam) return -1;
    const camera* cam = &s->cams[cami];
    int W = width > 0 ? width : (int)roundf(cam->aspect * resolution), H = resolution;
    float u = (i + (ii + 0.5f) / samples) / W;
    float v = (j + (jj + 0.5f) / samples) / H;
    ray r = eval_camera(cam, u, v);
    float o[8] = {r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, r.tmin, r.tmax};
    memcpy(ray8, o, sizeof o);
    return 0;
}

/* batch intersect_first / intersect_any */
int oracle_trace(void* vs, const float* rays, int n, int any, unsigned char* hit, int* inst, int* eis,
                 float* ews, float* dists) {
    scene* s = (scene*)vs;
#pragma omp parallel for schedule(static)
    for (int k = 0; k < n; k++) {
        const float* r8 = rays + (size_t)k * 8;
        ray r = {{r8[0], r8[1], r8[2]}, {r8[3], r8[4], r8[5]}, r8[6], r8[7]};
        float dist = 0;
        int ii = -1, ei = -1;
        v4 ew = {0, 0, 0, 0};
        int h = trace_scene(s, &r, any, &dist, &ii, &ei, &ew);
        hit[k] = (unsigned char)(h ? 1 : 0);
        if (!any) {
            inst[k] = h ? ii : -1;
            eis[k] = h ? ei : -1;
            ews[4 * k + 0] = h ? ew.x : 0;
            ews[4 * k + 1] = h ? ew.y : 0;
            ews[4 * k + 2] = h ? ew.z : 0;
            ews[4 * k + 3] = h ? ew.w : 0;
            dists[k] = h ? dist : 0;
        }
    }
    return 0;
}
