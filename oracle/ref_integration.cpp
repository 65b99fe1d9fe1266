// oracle/ref_integration.cpp -- the reference-side binding of the drop-in, compiled
// against the reference's OWN headers (src/scene.h, src/image.h) and include/yrt.h.
// It is what a maintainer of sebcossu/yocto_raytracing adds to use the MI355X path
// from the reference's in-memory scene. oracle/Makefile builds
// it into oracle/_ref/libyrtref_int.so; tests/test_integration.py checks it against
// the reference (same scene bytes; on the GPU, the same image as raytrace()).
//
//   yrt_host_scene* yrt_from_reference_scene(const scene*)     scene.h:26-155 -> yrt.h builder
//   image4f raytrace_gpu(const scene*, const vec3f&, int, int) same signature as raytrace(),
//                                                               src/raytrace.cpp:213
//   image4f raytrace_gpu(const scene*, const vec3f&, int, int, int gpus)
//                                                               the same on GPUs 0..gpus-1 of the node
//                                                               (yrt_multi: bands + RCCL gather)
//   void raytrace_gpu_release(const scene*)                     drop the scene's device copies
#include "scene.h"
#include "yrt.h"

#include <cmath>
#include <cstdio>
#include <vector>
#include <cstring>
#include <unordered_map>

namespace {

template <class T>
int index_in(const std::vector<T*>& v, const T* p) {
    if (!p) return -1;
    for (size_t i = 0; i < v.size(); i++)
        if (v[i] == p) return (int)i;
    return -1;
}

void frame12(const frame3f& f, float out[12]) {
    const float v[12] = {f.x.x, f.x.y, f.x.z, f.y.x, f.y.y, f.y.z, f.z.x, f.z.y, f.z.z, f.o.x, f.o.y, f.o.z};
    memcpy(out, v, sizeof v);
}

}  // namespace

// Hand the reference's scene (scene.h:136-155) to libyrt field by field. The arrays
// are copied; the reference keeps ownership of its scene. Returns nullptr (with
// yrt_last_error() set) on failure.
yrt_host_scene* yrt_from_reference_scene(const scene* scn) {
    yrt_host_scene* hs = nullptr;
    if (yrt_host_scene_create(&hs) != YRT_OK) return nullptr;
    auto fail = [&] {
        yrt_host_scene_free(hs);
        return (yrt_host_scene*)nullptr;
    };
    float f[12];
    for (auto cam : scn->cameras) {
        frame12(cam->frame, f);
        if (yrt_host_scene_add_camera(hs, f, cam->fovy, cam->aspect, cam->aperture, cam->focus, nullptr)) return fail();
    }
    for (auto txt : scn->textures) {  // raytrace() reads the 8-bit `ldr` image (raytrace.cpp:45-53)
        if (yrt_host_scene_add_texture(hs, txt->ldr.width, txt->ldr.height, &txt->ldr.pixels[0].x, nullptr))
            return fail();
    }
    for (auto m : scn->materials) {
        yrt_material_desc d = {{m->ke.x, m->ke.y, m->ke.z}, {m->kd.x, m->kd.y, m->kd.z},
                               {m->ks.x, m->ks.y, m->ks.z}, {m->kr.x, m->kr.y, m->kr.z},
                               m->rs, index_in(scn->textures, m->kd_txt), index_in(scn->textures, m->ks_txt)};
        if (yrt_host_scene_add_material(hs, &d, nullptr)) return fail();
    }
    for (auto s : scn->shapes) {
        yrt_shape_desc d = {};
        d.npos = (int)s->pos.size();
        d.pos = s->pos.empty() ? nullptr : &s->pos[0].x;
        d.norm = s->norm.size() == s->pos.size() && !s->norm.empty() ? &s->norm[0].x : nullptr;
        d.texcoord = s->texcoord.size() == s->pos.size() && !s->texcoord.empty() ? &s->texcoord[0].x : nullptr;
        d.radius = s->radius.size() == s->pos.size() && !s->radius.empty() ? s->radius.data() : nullptr;
        d.npoints = (int)s->points.size();
        d.points = s->points.data();
        d.nlines = (int)s->lines.size();
        d.lines = s->lines.empty() ? nullptr : &s->lines[0].x;
        d.ntriangles = (int)s->triangles.size();
        d.triangles = s->triangles.empty() ? nullptr : &s->triangles[0].x;
        if (yrt_host_scene_add_shape(hs, &d, nullptr)) return fail();
    }
    for (auto ist : scn->instances) {
        frame12(ist->frame, f);
        if (yrt_host_scene_add_instance(hs, f, index_in(scn->shapes, ist->shp), index_in(scn->materials, ist->mat),
                                        nullptr))
            return fail();
    }
    // the same BVH the reference builds (build_bvh(scn, false), raytrace.cpp:278)
    if (yrt_host_scene_build_bvh(hs, 0)) return fail();
    return hs;
}

// device copies, one per scene, made on first use and kept until released
static std::unordered_map<const scene*, yrt_scene*> resident;
// multi-GPU replicas, one per scene (and GPU count)
static std::unordered_map<const scene*, std::pair<int, yrt_multi*>> resident_multi;

// drop the device copies of `scn` (call before deleting or editing the scene)
void raytrace_gpu_release(const scene* scn) {
    auto it = resident.find(scn);
    if (it != resident.end()) {
        yrt_scene_free(it->second);
        resident.erase(it);
    }
    auto im = resident_multi.find(scn);
    if (im != resident_multi.end()) {
        yrt_multi_free(im->second.second);
        resident_multi.erase(im);
    }
}

// raytrace() (src/raytrace.cpp:213) on the GPU: same arguments, same image4f. The
// device copy of each scene is made once and reused by later calls.
image4f raytrace_gpu(const scene* scn, const vec3f& amb, int resolution, int samples) {
    auto& ds = resident[scn];
    if (!ds) {
        yrt_host_scene* hs = yrt_from_reference_scene(scn);
        if (!hs || yrt_scene_upload(hs, 0, &ds) != YRT_OK) {
            fprintf(stderr, "raytrace_gpu: %s\n", yrt_last_error());
            exit(1);  // the reference's own failure style (scene.cpp:119-122)
        }
        yrt_host_scene_free(hs);
    }
    yrt_render_params p;
    yrt_render_params_default(&p);
    p.ambient[0] = amb.x, p.ambient[1] = amb.y, p.ambient[2] = amb.z;
    p.resolution = resolution;
    p.samples = samples;
    int w = 0, h = 0;
    yrt_image_size(ds, &p, &w, &h);
    image4f img(w, h);
    if (yrt_render(ds, &p, &img.pixels[0].x, YRT_MEM_HOST, nullptr) != YRT_OK) {
        fprintf(stderr, "raytrace_gpu: %s\n", yrt_last_error());
        exit(1);
    }
    return img;
}

// raytrace() on GPUs 0..gpus-1 of the node: the scene replicated on each, interleaved
// 8-row bands per GPU, the framebuffer gathered over RCCL (yrt.h yrt_multi_*)
image4f raytrace_gpu(const scene* scn, const vec3f& amb, int resolution, int samples, int gpus) {
    if (gpus <= 1) return raytrace_gpu(scn, amb, resolution, samples);
    auto& slot = resident_multi[scn];
    if (!slot.second || slot.first != gpus) {
        if (slot.second) yrt_multi_free(slot.second);
        slot.second = nullptr;
        yrt_host_scene* hs = yrt_from_reference_scene(scn);
        std::vector<int> devices(gpus);
        for (int k = 0; k < gpus; k++) devices[k] = k;
        if (!hs || yrt_multi_create(hs, devices.data(), gpus, &slot.second) != YRT_OK) {
            fprintf(stderr, "raytrace_gpu: %s\n", yrt_last_error());
            exit(1);
        }
        slot.first = gpus;
        yrt_host_scene_free(hs);
    }
    yrt_render_params p;
    yrt_render_params_default(&p);
    p.ambient[0] = amb.x, p.ambient[1] = amb.y, p.ambient[2] = amb.z;
    p.resolution = resolution;
    p.samples = samples;
    const int w = (int)round(scn->cameras.front()->aspect * resolution), h = resolution;  // raytrace.cpp:215-216
    image4f img(w, h);
    if (yrt_multi_render(slot.second, &p, &img.pixels[0].x, YRT_MEM_HOST) != YRT_OK) {
        fprintf(stderr, "raytrace_gpu: %s\n", yrt_last_error());
        exit(1);
    }
    return img;
}

// ---- ctypes entry points for tests/test_integration.py ----
extern "C" {

int ref_int_save_scene(void* refscn, const char* path) {
    yrt_host_scene* hs = yrt_from_reference_scene((const scene*)refscn);
    if (!hs) return -1;
    int rc = yrt_scene_save(hs, path);
    yrt_host_scene_free(hs);
    return rc;
}

int ref_int_save_bvh(void* refscn, const char* path) {
    yrt_host_scene* hs = yrt_from_reference_scene((const scene*)refscn);
    if (!hs) return -1;
    int rc = yrt_host_scene_save_bvh(hs, path);
    yrt_host_scene_free(hs);
    return rc;
}

void ref_int_release(void* refscn) { raytrace_gpu_release((const scene*)refscn); }

int ref_int_render(void* refscn, float amb, int resolution, int samples, float* out) {
    image4f img = raytrace_gpu((const scene*)refscn, {amb, amb, amb}, resolution, samples);
    memcpy(out, img.pixels.data(), img.pixels.size() * sizeof(vec4f));
    return 0;
}

int ref_int_render_gpus(void* refscn, float amb, int resolution, int samples, int gpus, float* out) {
    image4f img = raytrace_gpu((const scene*)refscn, {amb, amb, amb}, resolution, samples, gpus);
    memcpy(out, img.pixels.data(), img.pixels.size() * sizeof(vec4f));
    return 0;
}

}  // extern "C"
