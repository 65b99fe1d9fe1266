// capi.cpp -- the C-ABI of include/yrt.h over the host scene code and the gfx950
// kernels. No exceptions cross this boundary: every entry point catches and maps
// to a status code, with the message kept per thread (yrt_last_error).
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/yrt.h"
#include "yrt_render.h"

struct yrt_host_scene {
    yrt::scene scn;
};

struct yrt_scene {
    yrt::device_scene* ds = nullptr;
    unsigned long long* counters = nullptr;  // device, yrt::cnt_count entries
    void* scratch = nullptr;                 // device staging for host-memory calls
    size_t scratch_bytes = 0;
    hipStream_t last_stream = nullptr;
    int trace_algorithm = YRT_ALGO_WAVEFRONT;  // walks used by yrt_trace_first/any
};

namespace {

thread_local std::string g_last_error;

void hip_check(hipError_t e, const char* what) {
    if (e == hipErrorOutOfMemory) throw yrt::device_oom(std::string(what) + ": " + hipGetErrorString(e));
    if (e != hipSuccess) throw yrt::device_error(std::string(what) + ": " + hipGetErrorString(e));
}

// exception type -> status code (yrt_scene.h lists the mapping); the message is kept
template <class F>
int guarded(F&& f) {
    try {
        g_last_error.clear();
        return f();
    } catch (const yrt::device_oom& e) {
        g_last_error = e.what();
        return YRT_ERR_OOM;
    } catch (const yrt::device_error& e) {
        g_last_error = e.what();
        return YRT_ERR_HIP;
    } catch (const yrt::unsupported_error& e) {
        g_last_error = e.what();
        return YRT_ERR_UNSUPPORTED;
    } catch (const std::bad_alloc&) {
        g_last_error = "out of memory";
        return YRT_ERR_OOM;
    } catch (const std::invalid_argument& e) {
        g_last_error = e.what();
        return YRT_ERR_INVALID_ARG;
    } catch (const std::runtime_error& e) {
        g_last_error = e.what();
        return YRT_ERR_IO;
    } catch (...) {
        g_last_error = "internal error";
        return YRT_ERR_INTERNAL;
    }
}

// the device tonemap's level thresholds, computed once with this host's powf
const yrt::tonemap_table& tonemap_table() {
    static yrt::tonemap_table t;
    static std::once_flag once;
    std::call_once(once, [] {
        yrt::tonemap_thresholds(t.thr);
        t.neg_inf_level = yrt::tonemap_neg_inf_level();
    });
    return t;
}

void* scratch(yrt_scene* s, size_t bytes) {
    if (bytes > s->scratch_bytes) {
        if (s->scratch) hip_check(hipFree(s->scratch), "hipFree");
        s->scratch = nullptr;
        s->scratch_bytes = 0;
        hip_check(hipMalloc(&s->scratch, bytes), "hipMalloc(scratch)");
        s->scratch_bytes = bytes;
    }
    return s->scratch;
}

struct resolved_window {
    int W, H, x0, y0, tw, th;
};

resolved_window resolve(const yrt::device_scene& ds, const yrt_render_params& p) {
    if (p.resolution <= 0 || p.samples <= 0) throw std::invalid_argument("resolution and samples must be > 0");
    if (p.camera < 0 || p.camera >= (int)ds.cameras.size()) throw std::invalid_argument("camera index out of range");
    if (p.band <= 0 || p.band_stride <= 0 || p.band_offset < 0 || p.band_offset >= p.band_stride)
        throw std::invalid_argument("bad band interleave");
    const auto& cam = ds.cameras[p.camera];
    resolved_window r;
    r.W = p.width > 0 ? p.width : (int)std::round(cam.aspect * p.resolution);  // raytrace.cpp:216
    r.H = p.resolution;
    r.x0 = p.x0;
    r.y0 = p.y0;
    if (r.x0 < 0 || r.y0 < 0 || r.x0 >= r.W || r.y0 >= r.H) throw std::invalid_argument("window origin outside image");
    int rows_avail = r.H - r.y0;
    // local rows available under the band interleave
    int bands_total = (rows_avail + p.band - 1) / p.band;
    int my_bands = bands_total > p.band_offset ? (bands_total - p.band_offset + p.band_stride - 1) / p.band_stride : 0;
    r.tw = p.tile_w > 0 ? p.tile_w : r.W - r.x0;
    r.th = p.tile_h > 0 ? p.tile_h : my_bands * p.band;
    if (r.x0 + r.tw > r.W) throw std::invalid_argument("window wider than image");
    return r;
}

}  // namespace

void yrt::set_last_error(const std::string& msg) { g_last_error = msg; }

namespace {
yrt::frame3f frame_of(const float* f) {
    return {{f[0], f[1], f[2]}, {f[3], f[4], f[5]}, {f[6], f[7], f[8]}, {f[9], f[10], f[11]}};
}
// a scene edited after build_bvh needs a new build before upload
template <typename T>
int append(yrt_host_scene* hs, std::vector<T>& v, T&& item, int* index) {
    v.push_back(std::move(item));
    hs->scn.has_bvh = false;
    if (index) *index = (int)v.size() - 1;
    return YRT_OK;
}
}  // namespace

extern "C" {

int yrt_abi_version(void) { return YRT_ABI_VERSION; }

const char* yrt_status_string(int s) {
    switch (s) {
        case YRT_OK: return "ok";
        case YRT_ERR_INVALID_ARG: return "invalid argument";
        case YRT_ERR_IO: return "i/o or format error";
        case YRT_ERR_UNSUPPORTED: return "unsupported input";
        case YRT_ERR_HIP: return "HIP runtime error";
        case YRT_ERR_NO_DEVICE: return "no GPU device";
        case YRT_ERR_OOM: return "out of memory";
        case YRT_ERR_INTERNAL: return "internal error";
        default: return "unknown status";
    }
}

const char* yrt_last_error(void) { return g_last_error.c_str(); }

int yrt_device_count(int* count) {
    if (!count) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        *count = n;
        return n > 0 ? YRT_OK : YRT_ERR_NO_DEVICE;
    });
}

int yrt_scene_load(const char* path, yrt_host_scene** out) {
    if (!path || !out) return YRT_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded([&] {
        auto hs = new yrt_host_scene();
        try {
            yrt::load_scene_any(path, hs->scn);
        } catch (...) {
            delete hs;
            throw;
        }
        *out = hs;
        return YRT_OK;
    });
}

int yrt_scene_save(const yrt_host_scene* hs, const char* path) {
    if (!hs || !path) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::save_yrtscene(path, hs->scn);
        return YRT_OK;
    });
}

int yrt_host_scene_build_bvh(yrt_host_scene* hs, int equal_num) {
    if (!hs) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::build_bvh(hs->scn, equal_num != 0);
        return YRT_OK;
    });
}

int yrt_host_scene_build_bvh_gpu(yrt_host_scene* hs, int equal_num, int device, float* kernel_ms) {
    if (!hs) return YRT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        g_last_error = "no HIP device visible";
        return YRT_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= ndev) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::build_bvh_gpu(hs->scn, equal_num != 0, device, kernel_ms);
        return YRT_OK;
    });
}

int yrt_host_scene_save_bvh(const yrt_host_scene* hs, const char* path) {
    if (!hs || !path) return YRT_ERR_INVALID_ARG;
    if (!hs->scn.has_bvh) {
        g_last_error = "scene has no BVH";
        return YRT_ERR_INVALID_ARG;
    }
    return guarded([&] {
        yrt::save_yrtbvh(path, hs->scn);
        return YRT_OK;
    });
}

int yrt_host_scene_info(const yrt_host_scene* hs, long long* info) {
    if (!hs || !info) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        const auto& s = hs->scn;
        long long lights = 0, tris = 0, lines = 0, points = 0, sdepth = 0;
        for (auto& i : s.instances) {
            if (i.mat < 0) continue;
            auto ke = s.materials[i.mat].ke;
            if (ke.x > 0 && ke.y > 0 && ke.z > 0) lights++;
        }
        for (auto& sh : s.shapes) {
            tris += sh.triangles.size();
            lines += sh.lines.size();
            points += sh.points.size();
            if (s.has_bvh) sdepth = std::max<long long>(sdepth, yrt::bvh_max_depth(sh.bvh));
        }
        long long v[12] = {(long long)s.cameras.size(), (long long)s.textures.size(),
                           (long long)s.materials.size(), (long long)s.shapes.size(),
                           (long long)s.instances.size(), lights,
                           s.has_bvh ? (long long)s.bvh.nodes.size() : 0,
                           s.has_bvh ? (long long)yrt::bvh_max_depth(s.bvh) : 0, sdepth, tris, lines, points};
        memcpy(info, v, sizeof v);
        return YRT_OK;
    });
}

int yrt_host_image_size(const yrt_host_scene* hs, int camera, int resolution, int* w, int* h) {
    if (!hs || !w || !h || camera < 0 || camera >= (int)hs->scn.cameras.size() || resolution <= 0)
        return YRT_ERR_INVALID_ARG;
    *w = (int)std::round(hs->scn.cameras[camera].aspect * resolution);
    *h = resolution;
    return YRT_OK;
}

void yrt_host_scene_free(yrt_host_scene* hs) { delete hs; }

int yrt_host_scene_create(yrt_host_scene** out) {
    if (!out) return YRT_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded([&] {
        *out = new yrt_host_scene();
        return YRT_OK;
    });
}


int yrt_host_scene_add_camera(yrt_host_scene* hs, const float frame[12], float fovy, float aspect, float aperture,
                              float focus, int* index) {
    if (!hs || !frame) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::camera c;
        c.frame = frame_of(frame);
        c.fovy = fovy, c.aspect = aspect, c.aperture = aperture, c.focus = focus;
        return append(hs, hs->scn.cameras, std::move(c), index);
    });
}

int yrt_host_scene_add_texture(yrt_host_scene* hs, int w, int h, const unsigned char* rgba8, int* index) {
    if (!hs || !rgba8 || w <= 0 || h <= 0) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::texture t;
        t.width = w, t.height = h;
        t.pixels.resize((size_t)w * h);
        memcpy(t.pixels.data(), rgba8, (size_t)w * h * 4);
        return append(hs, hs->scn.textures, std::move(t), index);
    });
}

int yrt_host_scene_add_material(yrt_host_scene* hs, const yrt_material_desc* d, int* index) {
    if (!hs || !d) return YRT_ERR_INVALID_ARG;
    const int nt = (int)hs->scn.textures.size();
    if (d->kd_txt < -1 || d->kd_txt >= nt || d->ks_txt < -1 || d->ks_txt >= nt) {
        g_last_error = "material texture index out of range";
        return YRT_ERR_INVALID_ARG;
    }
    return guarded([&] {
        yrt::material m;
        m.ke = {d->ke[0], d->ke[1], d->ke[2]};
        m.kd = {d->kd[0], d->kd[1], d->kd[2]};
        m.ks = {d->ks[0], d->ks[1], d->ks[2]};
        m.kr = {d->kr[0], d->kr[1], d->kr[2]};
        m.rs = d->rs;
        m.kd_txt = d->kd_txt, m.ks_txt = d->ks_txt;
        return append(hs, hs->scn.materials, std::move(m), index);
    });
}

int yrt_host_scene_add_shape(yrt_host_scene* hs, const yrt_shape_desc* d, int* index) {
    if (!hs || !d || d->npos < 0 || d->npoints < 0 || d->nlines < 0 || d->ntriangles < 0 ||
        (d->npos && !d->pos) || (d->npoints && !d->points) || (d->nlines && !d->lines) ||
        (d->ntriangles && !d->triangles))
        return YRT_ERR_INVALID_ARG;
    const int kinds = (d->npoints > 0) + (d->nlines > 0) + (d->ntriangles > 0);
    if (kinds > 1) {
        g_last_error = "shape mixes primitive types (unsupported)";
        return YRT_ERR_UNSUPPORTED;
    }
    if ((d->npoints || d->nlines) && !d->radius) {
        g_last_error = "points/lines need a radius per vertex";
        return YRT_ERR_INVALID_ARG;
    }
    auto bad = [&](const int* e, long long n) {
        for (long long k = 0; k < n; k++)
            if (e[k] < 0 || e[k] >= d->npos) return true;
        return false;
    };
    if (bad(d->points, d->npoints) || bad(d->lines, 2ll * d->nlines) || bad(d->triangles, 3ll * d->ntriangles)) {
        g_last_error = "element index outside the vertex array";
        return YRT_ERR_INVALID_ARG;
    }
    return guarded([&] {
        yrt::shape s;
        const size_t n = (size_t)d->npos;
        s.pos.resize(n);
        memcpy(s.pos.data(), d->pos, n * 12);
        if (d->norm) {
            s.norm.resize(n);
            memcpy(s.norm.data(), d->norm, n * 12);
        }
        if (d->texcoord) {
            s.texcoord.resize(n);
            memcpy(s.texcoord.data(), d->texcoord, n * 8);
        }
        if (d->radius) s.radius.assign(d->radius, d->radius + n);
        s.points.assign(d->points, d->points + d->npoints);
        s.lines.resize(d->nlines);
        if (d->nlines) memcpy(s.lines.data(), d->lines, (size_t)d->nlines * 8);
        s.triangles.resize(d->ntriangles);
        if (d->ntriangles) memcpy(s.triangles.data(), d->triangles, (size_t)d->ntriangles * 12);
        return append(hs, hs->scn.shapes, std::move(s), index);
    });
}

int yrt_host_scene_add_instance(yrt_host_scene* hs, const float frame[12], int shape, int material, int* index) {
    if (!hs || !frame || shape < 0 || shape >= (int)hs->scn.shapes.size() || material < 0 ||
        material >= (int)hs->scn.materials.size())
        return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::instance i;
        i.frame = frame_of(frame);
        i.shp = shape;
        i.mat = material;
        return append(hs, hs->scn.instances, std::move(i), index);
    });
}

int yrt_scene_upload(const yrt_host_scene* hs, int device, yrt_scene** out) {
    if (!hs || !out) return YRT_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        g_last_error = "no HIP device visible";
        return YRT_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= ndev) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        auto s = new yrt_scene();
        try {
            s->ds = yrt::device_scene_create(hs->scn, device);
            hip_check(hipMalloc(&s->counters, yrt::cnt_slots * yrt::cnt_count * sizeof(unsigned long long)), "hipMalloc(counters)");
            hip_check(hipMemset(s->counters, 0, yrt::cnt_slots * yrt::cnt_count * sizeof(unsigned long long)), "hipMemset");
            // hipMemset of device memory may still be running when it returns, on the null
            // stream, which a caller's non-blocking stream does not wait for: a first render
            // on such a stream would race it (seen: a fresh handle's first frame lost part of
            // k_primary's counts)
            hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        } catch (...) {
            yrt_scene_free(s);
            throw;
        }
        *out = s;
        return YRT_OK;
    });
}

int yrt_scene_set_trace_algorithm(yrt_scene* s, int algorithm) {
    if (!s || algorithm < YRT_ALGO_WAVEFRONT || algorithm > YRT_ALGO_WAVEFRONT_LANE) return YRT_ERR_INVALID_ARG;
    s->trace_algorithm = algorithm;
    return YRT_OK;
}

int yrt_scene_set_tile_lists(yrt_scene* s, int mode) {
    if (!s || mode < YRT_LISTS_AUTO || mode > YRT_LISTS_OFF) return YRT_ERR_INVALID_ARG;
    s->ds->lists_mode = mode;
    return YRT_OK;
}

int yrt_scene_tile_lists(yrt_scene* s, int* camera_on, int* bundles_on, unsigned long long* sums) {
    if (!s) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::device_scene& ds = *s->ds;
        hip_check(hipSetDevice(ds.device), "hipSetDevice");
        if (ds.list_stats_ev && ds.list_stats_recorded) hip_check(hipEventSynchronize(ds.list_stats_ev), "list sums");
        if (camera_on) *camera_on = ds.last_camera_lists;
        if (bundles_on) *bundles_on = ds.last_bundles;
        if (sums)
            for (int i = 0; i < 4; i++) sums[i] = ds.list_stats_host ? ds.list_stats_host[i] : 0;
        return YRT_OK;
    });
}

int yrt_scene_tile_list_masks(yrt_scene* s, unsigned long long* excluded) {
    if (!s || !excluded) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::device_scene& ds = *s->ds;
        hip_check(hipSetDevice(ds.device), "hipSetDevice");
        if (ds.list_stats_ev && ds.list_stats_recorded) hip_check(hipEventSynchronize(ds.list_stats_ev), "list sums");
        for (int i = 0; i < 2; i++) excluded[i] = ds.list_stats_host ? ds.list_stats_host[4 + i] : 0;
        return YRT_OK;
    });
}

int yrt_scene_set_lds_staging(yrt_scene* s, int on) {
    if (!s || (on != 0 && on != 1)) return YRT_ERR_INVALID_ARG;
    s->ds->lds_staging = on;
    return YRT_OK;
}

int yrt_scene_lds_staging(yrt_scene* s, int* staged) {
    if (!s || !staged) return YRT_ERR_INVALID_ARG;
    *staged = s->ds->last_lds_staging;
    return YRT_OK;
}

size_t yrt_scene_device_bytes(const yrt_scene* s) { return s && s->ds ? s->ds->arena_bytes : 0; }

void yrt_scene_free(yrt_scene* s) {
    if (!s) return;
    if (s->ds) (void)hipSetDevice(s->ds->device);
    if (s->counters) (void)hipFree(s->counters);
    if (s->scratch) (void)hipFree(s->scratch);
    yrt::device_scene_destroy(s->ds);
    delete s;
}

void yrt_render_params_default(yrt_render_params* p) {
    if (!p) return;
    memset(p, 0, sizeof *p);
    p->ambient[0] = p->ambient[1] = p->ambient[2] = 0.1f;  // main(): -a default 0.1
    p->resolution = 720;                                    // -r default 720
    p->samples = 1;                                         // -s default 1
    p->max_depth = 16;
    p->band = 1;
    p->band_stride = 1;
}

int yrt_image_size(const yrt_scene* s, const yrt_render_params* p, int* w, int* h) {
    if (!s || !p || !w || !h) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        auto r = resolve(*s->ds, *p);
        *w = r.W;
        *h = r.H;
        return YRT_OK;
    });
}

int yrt_render(yrt_scene* s, const yrt_render_params* p, float* out, int mem, void* stream) {
    if (!s || !p || !out) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        auto r = resolve(*s->ds, *p);
        hipStream_t st = (hipStream_t)stream;
        hip_check(hipSetDevice(s->ds->device), "hipSetDevice");
        yrt::dev_render_args a = {};
        a.cam = yrt::make_dev_camera(s->ds->cameras[p->camera]);
        for (int k = 0; k < 3; k++) a.amb[k] = p->ambient[k];
        a.width = r.W;
        a.height = r.H;
        a.samples = p->samples;
        a.max_depth = p->max_depth > 0 ? p->max_depth : 16;
        a.x0 = r.x0;
        a.tile_w = r.tw;
        a.y0 = r.y0;
        a.tile_h = r.th;
        a.band = p->band;
        a.band_stride = p->band_stride;
        a.band_offset = p->band_offset;
        a.out_stride = p->out_stride > 0 ? p->out_stride : r.tw;
        if (a.out_stride < r.tw) throw std::invalid_argument("out_stride smaller than the window width");
        size_t bytes = (size_t)a.out_stride * r.th * 4 * sizeof(float);
        void* dst = mem == YRT_MEM_DEVICE ? (void*)out : scratch(s, bytes);
        // (the wavefront algorithms zero the counter lines in their first kernel, k_chunk_setup)
        if (p->algorithm == YRT_ALGO_MEGAKERNEL)
            hip_check(hipMemsetAsync(s->counters, 0, yrt::cnt_slots * yrt::cnt_count * sizeof(unsigned long long), st),
                      "hipMemsetAsync");
        // timing 1: start a new record; 2: keep accumulating across calls (bench loops)
        if (!(p->timing == 2 && s->ds->timer.on)) s->ds->timer.reset(p->timing != 0);
        if (p->algorithm == YRT_ALGO_MEGAKERNEL && s->ds->reflective && a.max_depth > yrt::megakernel_max_depth)
            throw yrt::unsupported_error("the megakernel keeps " + std::to_string(yrt::megakernel_max_depth) +
                                         " mirror levels per lane; deeper recursions need the wavefront algorithm");
        if (p->algorithm == YRT_ALGO_MEGAKERNEL)
            hip_check(yrt::launch_render(*s->ds, a, dst, s->counters, p->count_work != 0, st), "render kernel launch");
        else if (p->algorithm == YRT_ALGO_WAVEFRONT || p->algorithm == YRT_ALGO_WAVEFRONT_LANE)
            hip_check(yrt::launch_render_wavefront(*s->ds, a, dst, s->counters, p->count_work != 0,
                                                   p->algorithm == YRT_ALGO_WAVEFRONT, st),
                      "wavefront render launch");
        else
            throw std::invalid_argument("unknown algorithm");
        s->last_stream = st;
        if (mem != YRT_MEM_DEVICE) {
            hip_check(hipMemcpyAsync(out, dst, bytes, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
            hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
        }
        return YRT_OK;
    });
}

static int trace_impl(yrt_scene* s, const float* rays, int n, int any, unsigned char* hit, int* inst, int* ei,
                      float* ew, float* dist, int mem, void* stream) {
    if (!s || n < 0 || (n && (!rays || !hit))) return YRT_ERR_INVALID_ARG;
    if (!any && n && (!inst || !ei || !ew || !dist)) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        hipStream_t st = (hipStream_t)stream;
        hip_check(hipSetDevice(s->ds->device), "hipSetDevice");
        hip_check(hipMemsetAsync(s->counters, 0, yrt::cnt_slots * yrt::cnt_count * sizeof(unsigned long long), st), "hipMemsetAsync");
        s->last_stream = st;
        if (n == 0) return YRT_OK;
        if (mem == YRT_MEM_DEVICE) {
            hip_check(yrt::launch_trace(*s->ds, rays, n, any, hit, inst, ei, ew, dist, s->counters,
                                              s->trace_algorithm == YRT_ALGO_WAVEFRONT, st), "trace launch");
            return YRT_OK;
        }
        size_t rb = (size_t)n * 8 * 4, hb = ((size_t)n + 255) & ~(size_t)255, ib = (size_t)n * 4, eb = (size_t)n * 16;
        char* base = (char*)scratch(s, rb + hb + 3 * ib + eb + 1024);
        float* d_rays = (float*)base;
        unsigned char* d_hit = (unsigned char*)(base + rb);
        int* d_inst = (int*)(base + rb + hb);
        int* d_ei = (int*)(base + rb + hb + ib);
        float* d_dist = (float*)(base + rb + hb + 2 * ib);
        float* d_ew = (float*)(base + rb + hb + 3 * ib);
        hip_check(hipMemcpyAsync(d_rays, rays, rb, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
        hip_check(yrt::launch_trace(*s->ds, d_rays, n, any, d_hit, d_inst, d_ei, d_ew, d_dist, s->counters,
                                    s->trace_algorithm == YRT_ALGO_WAVEFRONT, st),
                  "trace launch");
        hip_check(hipMemcpyAsync(hit, d_hit, n, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
        if (!any) {
            hip_check(hipMemcpyAsync(inst, d_inst, ib, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
            hip_check(hipMemcpyAsync(ei, d_ei, ib, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
            hip_check(hipMemcpyAsync(dist, d_dist, ib, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
            hip_check(hipMemcpyAsync(ew, d_ew, eb, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
        }
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
        return YRT_OK;
    });
}

int yrt_trace_first(yrt_scene* s, const float* rays, int n, unsigned char* hit, int* inst, int* ei, float* ew,
                    float* dist, int mem, void* stream) {
    return trace_impl(s, rays, n, 0, hit, inst, ei, ew, dist, mem, stream);
}

int yrt_trace_any(yrt_scene* s, const float* rays, int n, unsigned char* hit, int mem, void* stream) {
    return trace_impl(s, rays, n, 1, hit, nullptr, nullptr, nullptr, nullptr, mem, stream);
}

int yrt_last_stats(yrt_scene* s, yrt_stats* out) {
    if (!s || !out) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        std::vector<unsigned long long> lines((size_t)yrt::cnt_slots * yrt::cnt_count);
        hip_check(hipSetDevice(s->ds->device), "hipSetDevice");
        hip_check(hipStreamSynchronize(s->last_stream), "hipStreamSynchronize");
        hip_check(hipMemcpy(lines.data(), s->counters, lines.size() * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost),
                  "hipMemcpy(counters)");
        unsigned long long c[yrt::cnt_count] = {};
        for (int l = 0; l < yrt::cnt_slots; l++)
            for (int k = 0; k < yrt::cnt_count; k++) c[k] += lines[(size_t)l * yrt::cnt_count + k];
        // the wavefront path counts its shadow rays only under cnt_shadow_rays
        out->rays = c[yrt::cnt_rays] + c[yrt::cnt_shadow_rays];
        out->camera_samples = c[yrt::cnt_samples];
        out->depth_truncated = c[yrt::cnt_depth_truncated];
        out->stack_overflow = c[yrt::cnt_stack_overflow];
        out->box_tests = c[yrt::cnt_box_tests];
        out->instance_entries = c[yrt::cnt_inst_entries];
        out->prim_tests = c[yrt::cnt_prim_tests];
        out->shaded_hits = c[yrt::cnt_shaded_hits];
        out->texture_lookups = c[yrt::cnt_tex_lookups];
        out->shadow_rays = c[yrt::cnt_shadow_rays];
        out->shadow_box_tests = c[yrt::cnt_shadow_box_tests];
        out->shadow_instance_entries = c[yrt::cnt_shadow_inst_entries];
        out->shadow_prim_tests = c[yrt::cnt_shadow_prim_tests];
        out->wave_node_visits = c[yrt::cnt_wave_node_visits];
        out->wave_prim_visits = c[yrt::cnt_wave_prim_visits];
        out->shadow_wave_node_visits = c[yrt::cnt_shadow_wave_node_visits];
        out->shadow_rays_culled = c[yrt::cnt_shadow_culled];
        return YRT_OK;
    });
}

int yrt_last_timings(yrt_scene* s, yrt_timings* out) {
    if (!s || !out) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        hip_check(hipSetDevice(s->ds->device), "hipSetDevice");
        s->ds->timer.collect(out->ms, out->launches);
        return YRT_OK;
    });
}

int yrt_tonemap(const float* rgba, int n, unsigned char* out, int mem, void* stream) {
    if (n < 0 || (n && (!rgba || !out))) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        if (mem == YRT_MEM_DEVICE) {
            hip_check(yrt::launch_tonemap(rgba, n, out, tonemap_table(), (hipStream_t)stream), "tonemap launch");
        } else {
            int h = 1;
            yrt::tonemap_rgba8(rgba, n, h, out);
        }
        return YRT_OK;
    });
}

int yrt_save_image(const char* path, const float* rgba, int w, int h) {
    if (!path || !rgba || w <= 0 || h <= 0) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        yrt::save_hdr_or_ldr(path, rgba, w, h);
        return YRT_OK;
    });
}

int yrt_save_image_mem(const char* path, const float* rgba, int w, int h, int mem, void* stream) {
    if (mem != YRT_MEM_DEVICE) return yrt_save_image(path, rgba, w, h);
    if (!path || !rgba || w <= 0 || h <= 0) return YRT_ERR_INVALID_ARG;
    return guarded([&] {
        const std::string p = path;
        const size_t n = (size_t)w * h;
        hipStream_t st = (hipStream_t)stream;
        if (p.size() >= 4 && p.substr(p.size() - 4) == ".hdr") {
            // RGBE on the GPU (4 B/pixel over PCIe), the run-length scanlines on the host
            unsigned char* d8 = nullptr;
            hip_check(hipMalloc(&d8, n * 4), "hipMalloc(rgbe)");
            std::vector<unsigned char> rgbe(n * 4);
            hipError_t e = yrt::launch_rgbe(rgba, w, h, d8, st);
            if (e == hipSuccess) e = hipMemcpyAsync(rgbe.data(), d8, n * 4, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            (void)hipFree(d8);
            hip_check(e, "device rgbe");
            yrt::save_hdr_rgbe(p, rgbe.data(), w, h);
            return YRT_OK;
        }
        // tonemap on the GPU, then only the 8-bit image crosses PCIe
        unsigned char* d8 = nullptr;
        hip_check(hipMalloc(&d8, n * 4), "hipMalloc(tonemap)");
        std::vector<unsigned char> ldr(n * 4);
        hipError_t e = yrt::launch_tonemap(rgba, (int)n, d8, tonemap_table(), st);
        if (e == hipSuccess) e = hipMemcpyAsync(ldr.data(), d8, n * 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        (void)hipFree(d8);
        hip_check(e, "device tonemap");
        yrt::save_ldr_png(p, ldr.data(), w, h);
        return YRT_OK;
    });
}

}  // extern "C"
