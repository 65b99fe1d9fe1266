// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as product).
//
// A thin extern "C" harness around the *unmodified* reference sources under
// /root/reference/src, compiled by oracle/Makefile into oracle/_ref/libyrtref.so.
// It lets tests/, bench.py's cpu_baseline leg and tests/golden/make_golden.py call
// the reference's own functions:
//   load_scene        src/scene.cpp:113   (Yocto OBJ loader, untouched)
//   build_bvh         src/scene.cpp:554   (binary midpoint BVH)
//   raytrace          src/raytrace.cpp:213
//   eval_camera/shade src/raytrace.cpp:6,88 (row-subset render, same loop body as :228-250)
//   intersect_first/any src/scene.cpp:483,489
//   save_hdr_or_ldr   src/image.cpp:81   (stbi_write_hdr / tonemap + stbi_write_png)
// and to serialise the reference's in-memory scene / BVH into the repo's own
// interchange formats (.yrtscene, .yrtbvh; spec in DESIGN.md §3) so the product
// loader and BVH builder can be compared byte-for-byte with the reference.
//
// Ray counting: shade() (raytrace.o) calls intersect_first/any (scene.o) across
// object files, so the link step wraps those two symbols (-Wl,--wrap) and the
// wrappers below count every traced ray of the reference itself, per thread (the
// all-cores baseline, ref_render_rows_mt, runs shade() on many threads at once).
#include "scene.h"

#include <zlib.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

// reference functions defined in src/raytrace.cpp (compiled with -Dmain=reference_main)
ray3f eval_camera(const camera* cam, const vec2f& uv);
vec4f shade(const scene* scn, const std::vector<instance*>& lights, const vec3f& amb,
            const ray3f& ray);
image4f raytrace(const scene* scn, const vec3f& amb, int resolution, int samples);

static thread_local long long g_rays = 0;

extern "C" {
intersection3f __real__Z15intersect_firstPK5sceneRK5ray3f(const scene*, const ray3f&);
bool __real__Z13intersect_anyPK5sceneRK5ray3f(const scene*, const ray3f&);
intersection3f __wrap__Z15intersect_firstPK5sceneRK5ray3f(const scene* s, const ray3f& r) {
    g_rays++;
    return __real__Z15intersect_firstPK5sceneRK5ray3f(s, r);
}
bool __wrap__Z13intersect_anyPK5sceneRK5ray3f(const scene* s, const ray3f& r) {
    g_rays++;
    return __real__Z13intersect_anyPK5sceneRK5ray3f(s, r);
}
}

namespace {

struct gzout {
    gzFile f;
    explicit gzout(const char* path) { f = gzopen(path, "wb6"); }
    ~gzout() {
        if (f) gzclose(f);
    }
    void raw(const void* p, size_t n) {
        if (n) gzwrite(f, p, (unsigned)n);
    }
    void u32(uint32_t v) { raw(&v, 4); }
    void i32(int32_t v) { raw(&v, 4); }
    template <class T>
    void vec(const std::vector<T>& v) {
        u32((uint32_t)v.size());
        raw(v.data(), v.size() * sizeof(T));
    }
};

struct gzin {
    gzFile f;
    bool ok = true;
    explicit gzin(const char* path) { f = gzopen(path, "rb"); ok = f != nullptr; }
    ~gzin() {
        if (f) gzclose(f);
    }
    void raw(void* p, size_t n) {
        if (!n) return;
        if (gzread(f, p, (unsigned)n) != (int)n) ok = false;
    }
    uint32_t u32() { uint32_t v = 0; raw(&v, 4); return v; }
    int32_t i32() { int32_t v = 0; raw(&v, 4); return v; }
    template <class T>
    void vec(std::vector<T>& v) {
        v.resize(u32());
        raw(v.data(), v.size() * sizeof(T));
    }
};

template <class T>
int index_of(const std::vector<T*>& v, const T* p) {
    for (size_t i = 0; i < v.size(); i++)
        if (v[i] == p) return (int)i;
    return -1;
}

void write_nodes(gzout& o, const bvh_tree* bvh) {
    static_assert(sizeof(bvh_node) == 32, "bvh_node layout");
    o.vec(bvh->nodes);
    o.vec(bvh->leaf_prims);
}

}  // namespace

extern "C" {

// load_scene (scene.cpp:113) followed by build_bvh(scn, false) exactly as main() does
// (raytrace.cpp:274,278).
void* ref_load_scene(const char* path) {
    auto scn = load_scene(path);
    build_bvh(scn, false);
    return scn;
}

void ref_free_scene(void* scn) { delete (scene*)scn; }

// Serialise the reference's loaded scene into the .yrtscene interchange format.
int ref_write_scene(void* vscn, const char* path) {
    auto scn = (const scene*)vscn;
    gzout o(path);
    if (!o.f) return -1;
    o.raw("YRTSCN1", 8);
    o.u32((uint32_t)scn->cameras.size());
    for (auto cam : scn->cameras) {
        o.raw(&cam->frame, 48);
        o.raw(&cam->fovy, 4);
        o.raw(&cam->aspect, 4);
        o.raw(&cam->aperture, 4);
        o.raw(&cam->focus, 4);
    }
    o.u32((uint32_t)scn->textures.size());
    for (auto txt : scn->textures) {
        o.i32(txt->ldr.width);
        o.i32(txt->ldr.height);
        o.raw(txt->ldr.pixels.data(), txt->ldr.pixels.size() * 4);
    }
    o.u32((uint32_t)scn->materials.size());
    for (auto m : scn->materials) {
        o.raw(&m->ke, 12);
        o.raw(&m->kd, 12);
        o.raw(&m->ks, 12);
        o.raw(&m->kr, 12);
        o.raw(&m->rs, 4);
        o.i32(index_of(scn->textures, m->kd_txt));
        o.i32(index_of(scn->textures, m->ks_txt));
    }
    o.u32((uint32_t)scn->shapes.size());
    for (auto s : scn->shapes) {
        o.vec(s->pos);
        o.vec(s->norm);
        o.vec(s->texcoord);
        o.vec(s->radius);
        o.vec(s->points);
        o.vec(s->lines);
        o.vec(s->triangles);
    }
    o.u32((uint32_t)scn->instances.size());
    for (auto ist : scn->instances) {
        o.raw(&ist->frame, 48);
        o.i32(index_of(scn->shapes, ist->shp));
        o.i32(index_of(scn->materials, ist->mat));
    }
    return 0;
}

// Build a reference `scene` (reference structs, reference allocation) from a
// .yrtscene file, then run the reference's build_bvh. Used where the OBJ inputs
// are absent (GPU box): the reference code still does all BVH/trace/shade work.
void* ref_read_scene(const char* path) {
    gzin in(path);
    if (!in.ok) return nullptr;
    char magic[8];
    in.raw(magic, 8);
    if (memcmp(magic, "YRTSCN1", 8) != 0) return nullptr;
    auto scn = new scene();
    auto ncam = in.u32();
    for (uint32_t i = 0; i < ncam; i++) {
        auto cam = new camera();
        in.raw(&cam->frame, 48);
        in.raw(&cam->fovy, 4);
        in.raw(&cam->aspect, 4);
        in.raw(&cam->aperture, 4);
        in.raw(&cam->focus, 4);
        scn->cameras.push_back(cam);
    }
    auto ntex = in.u32();
    for (uint32_t i = 0; i < ntex; i++) {
        auto txt = new texture();
        int w = in.i32(), h = in.i32();
        txt->ldr = image4b(w, h);
        in.raw(txt->ldr.pixels.data(), (size_t)w * h * 4);
        scn->textures.push_back(txt);
    }
    auto nmat = in.u32();
    for (uint32_t i = 0; i < nmat; i++) {
        auto m = new material();
        in.raw(&m->ke, 12);
        in.raw(&m->kd, 12);
        in.raw(&m->ks, 12);
        in.raw(&m->kr, 12);
        in.raw(&m->rs, 4);
        int kt = in.i32(), st = in.i32();
        m->kd_txt = kt >= 0 ? scn->textures[kt] : nullptr;
        m->ks_txt = st >= 0 ? scn->textures[st] : nullptr;
        scn->materials.push_back(m);
    }
    auto nshp = in.u32();
    for (uint32_t i = 0; i < nshp; i++) {
        auto s = new shape();
        in.vec(s->pos);
        in.vec(s->norm);
        in.vec(s->texcoord);
        in.vec(s->radius);
        in.vec(s->points);
        in.vec(s->lines);
        in.vec(s->triangles);
        scn->shapes.push_back(s);
    }
    auto nist = in.u32();
    for (uint32_t i = 0; i < nist; i++) {
        auto ist = new instance();
        in.raw(&ist->frame, 48);
        int si = in.i32(), mi = in.i32();
        ist->shp = scn->shapes[si];
        ist->mat = mi >= 0 ? scn->materials[mi] : nullptr;
        scn->instances.push_back(ist);
    }
    if (!in.ok) {
        delete scn;
        return nullptr;
    }
    build_bvh(scn, false);
    return scn;
}

// Serialise the reference BVHs (per shape, then the instance level) to .yrtbvh.
int ref_write_bvh(void* vscn, const char* path) {
    auto scn = (const scene*)vscn;
    gzout o(path);
    if (!o.f) return -1;
    o.raw("YRTBVH1", 8);
    o.u32((uint32_t)scn->shapes.size());
    for (auto s : scn->shapes) write_nodes(o, s->bvh);
    write_nodes(o, scn->bvh);
    return 0;
}

// raytrace() (raytrace.cpp:213) into a caller buffer of W*H*4 floats.
int ref_image_size(void* vscn, int resolution, int* w, int* h) {
    auto scn = (const scene*)vscn;
    auto cam = scn->cameras.front();
    *w = (int)std::round(cam->aspect * resolution);
    *h = resolution;
    return 0;
}

long long ref_render(void* vscn, float amb, int resolution, int samples, float* out) {
    g_rays = 0;
    auto img = raytrace((const scene*)vscn, vec3f{amb, amb, amb}, resolution, samples);
    memcpy(out, img.pixels.data(), img.pixels.size() * sizeof(vec4f));
    return g_rays;
}

// Rows subset of the same image: identical loop body to raytrace.cpp:232-249 for
// pixel rows rows[0..nrows), each row W pixels, into out[nrows*W*4]. Returns the
// number of rays the reference traced.
long long ref_render_rows(void* vscn, float amb, int resolution, int samples, const int* rows,
                          int nrows, float* out) {
    auto scn = (const scene*)vscn;
    auto cam = scn->cameras.front();
    int W = (int)std::round(cam->aspect * resolution), H = resolution;
    vec3f a = {amb, amb, amb};
    g_rays = 0;
    for (int r = 0; r < nrows; r++) {
        int j = rows[r];
        for (int i = 0; i < W; i++) {
            vec4f acc = {0, 0, 0, 0};
            for (auto jj = 0; jj < samples; jj++) {
                for (auto ii = 0; ii < samples; ii++) {
                    vec2f uv = {(i + (ii + 0.5f) / samples) / W, (j + (jj + 0.5f) / samples) / H};
                    auto ray = eval_camera(cam, uv);
                    acc += shade(scn, scn->instances, a, ray);
                }
            }
            float* px = out + ((size_t)r * W + i) * 4;
            px[0] = acc.x / float(samples * samples);
            px[1] = acc.y / float(samples * samples);
            px[2] = acc.z / float(samples * samples);
            px[3] = 1.0f;
        }
    }
    return g_rays;
}

// The same rows rendered by nthreads host threads (the reference's CPU path on all cores,
// for bench.py's cpu_baseline_all_cores): each thread takes the next row from a shared
// counter and runs the loop body above on it -- eval_camera and shade() are the
// reference's, and shade() only reads the scene (its per-call `new`s leak, as in the
// reference; malloc is thread-safe). Returns the rays traced by all threads.
long long ref_render_rows_mt(void* vscn, float amb, int resolution, int samples, const int* rows, int nrows,
                             float* out, int nthreads) {
    auto scn = (const scene*)vscn;
    auto cam = scn->cameras.front();
    const int W = (int)std::round(cam->aspect * resolution);
    std::atomic<int> next{0};
    std::atomic<long long> rays{0};
    auto work = [&]() {
        long long mine = 0;
        for (int r; (r = next.fetch_add(1)) < nrows;) {
            mine += ref_render_rows(vscn, amb, resolution, samples, rows + r, 1, out + (size_t)r * W * 4);
        }
        rays += mine;
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; t++) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    (void)cam;
    return rays.load();
}

// Per-ray queries. rays: n x 8 floats (o.xyz, d.xyz, tmin, tmax).
// Outputs: hit[n] (u8), inst[n], ei[n], ew[n*4], dist[n]. any != 0 -> intersect_any.
int ref_trace(void* vscn, const float* rays, int n, int any, unsigned char* hit, int* inst,
              int* ei, float* ew, float* dist) {
    auto scn = (const scene*)vscn;
    for (int k = 0; k < n; k++) {
        const float* r = rays + (size_t)k * 8;
        ray3f ray;
        ray.o = {r[0], r[1], r[2]};
        ray.d = {r[3], r[4], r[5]};
        ray.tmin = r[6];
        ray.tmax = r[7];
        if (any) {
            hit[k] = intersect_any(scn, ray) ? 1 : 0;
        } else {
            auto isec = intersect_first(scn, ray);
            hit[k] = isec.hit() ? 1 : 0;
            inst[k] = isec.hit() ? index_of(scn->instances, isec.ist) : -1;
            ei[k] = isec.ei;
            memcpy(ew + (size_t)k * 4, &isec.ew, 16);
            dist[k] = isec.dist;
        }
    }
    return 0;
}

// Camera rays exactly as eval_camera (raytrace.cpp:6-37) makes them, for the
// uv of raytrace.cpp:236-239 at pixel (i, j), sub-sample (ii, jj).
int ref_camera_ray(void* vscn, int resolution, int samples, int i, int j, int ii, int jj,
                   float* ray8) {
    auto scn = (const scene*)vscn;
    auto cam = scn->cameras.front();
    int W = (int)std::round(cam->aspect * resolution), H = resolution;
    vec2f uv = {(i + (ii + 0.5f) / samples) / W, (j + (jj + 0.5f) / samples) / H};
    auto ray = eval_camera(cam, uv);
    float v[8] = {ray.o.x, ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z, ray.tmin, ray.tmax};
    memcpy(ray8, v, sizeof v);
    return 0;
}

// The reference's own PNG loader (image.cpp:25-35, stb_image) for its shipped images.
// Call with out == nullptr to get the size, then again with a w*h*4 buffer.
int ref_load_image4b(const char* path, int* w, int* h, unsigned char* out) {
    auto img = load_image4b(path);
    *w = img.width;
    *h = img.height;
    if (out) memcpy(out, img.pixels.data(), img.pixels.size() * 4);
    return img.pixels.empty() ? -1 : 0;
}

// The reference's own image writer (image.cpp:81-88 save_hdr_or_ldr: stbi_write_hdr for
// .hdr, tonemap + stbi_write_png otherwise) on a caller-supplied RGBA float frame.
int ref_save_image(const char* path, const float* rgba, int w, int h) {
    image4f img(w, h);
    memcpy(img.pixels.data(), rgba, (size_t)w * h * 16);
    save_hdr_or_ldr(path, img);
    return 0;
}

}  // extern "C"
