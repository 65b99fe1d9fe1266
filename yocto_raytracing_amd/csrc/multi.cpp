// multi.cpp -- raytrace() across the GPUs of one node from ONE host process
// (SURVEY.md §8e): the scene replicated on every device, the frame cut into
// interleaved 8-row bands, and the float framebuffer gathered to the root device
// over RCCL (grouped ncclSend/ncclRecv, point-to-point over xGMI) and reassembled in
// image order. Replaces the single-device raytrace() call of main()
// (src/raytrace.cpp:282); every pixel depends only on the read-only scene
// (raytrace.cpp:228-250), so no other exchange exists.
//
// Band geometry: image band b (rows 8b..8b+7) belongs to rank b % n, as local band
// b / n. Every rank renders the same padded number of bands, ceil(nbands / n), so
// every send has the same size; rows past the image read zero and are never copied
// out. Reassembly: one strided 2-D copy per rank for its complete bands (destination
// pitch n bands) plus one copy for the image's last band if it is partial.
//
// Transport (yrt_multi_info): RCCL when the devices are distinct (ncclCommInitAll, one
// communicator per device in this process); plain device copies when they are not
// (the same device listed twice: a rehearsal of the band geometry on one GPU; RCCL
// refuses two ranks on one device). YRT_MULTI_TRANSPORT=rccl forces RCCL (also for
// n = 1, where the root's shard goes through an RCCL self send/receive). There is no
// silent fallback: distinct devices without a loadable RCCL are an error.
//
// RCCL is loaded with dlopen on first use (librccl.so.1: the process's copy if the
// host already loaded one, e.g. PyTorch's, else ROCm's), so libyrt.so does not link it
// and single-GPU use never touches it.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/yrt.h"
#include "yrt_scene.h"

namespace {

// ---- the few RCCL entry points used (rccl.h, NCCL 2.27 ABI) ----
typedef struct ncclComm* ncclComm_t;
typedef int ncclResult_t;  // ncclSuccess == 0
constexpr int nccl_float32 = 7;  // ncclFloat32
struct rccl_api {
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    std::string load_error;
};

const rccl_api& rccl() {
    static rccl_api api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            api.load_error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        auto sym = [&](const char* n) {
            void* p = dlsym(h, n);
            if (!p) api.load_error = std::string("librccl.so.1 lacks ") + n;
            return p;
        };
        api.comm_init_all = (decltype(api.comm_init_all))sym("ncclCommInitAll");
        api.comm_destroy = (decltype(api.comm_destroy))sym("ncclCommDestroy");
        api.group_start = (decltype(api.group_start))sym("ncclGroupStart");
        api.group_end = (decltype(api.group_end))sym("ncclGroupEnd");
        api.send = (decltype(api.send))sym("ncclSend");
        api.recv = (decltype(api.recv))sym("ncclRecv");
        api.error_string = (decltype(api.error_string))sym("ncclGetErrorString");
    });
    return api;
}

void nccl_check(ncclResult_t r, const char* what) {
    if (r != 0)
        throw yrt::device_error(std::string(what) + ": " +
                                (rccl().error_string ? rccl().error_string(r) : std::to_string(r)));
}

void hip_check(hipError_t e, const char* what) {
    if (e == hipErrorOutOfMemory) throw yrt::device_oom(std::string(what) + ": " + hipGetErrorString(e));
    if (e != hipSuccess) throw yrt::device_error(std::string(what) + ": " + hipGetErrorString(e));
}

// a yrt_* status from another entry point, rethrown with its message
void yrt_check(int status, const char* what) {
    if (status == YRT_OK) return;
    std::string m = std::string(what) + ": " + yrt_last_error();
    switch (status) {
        case YRT_ERR_INVALID_ARG: throw std::invalid_argument(m);
        case YRT_ERR_UNSUPPORTED: throw yrt::unsupported_error(m);
        case YRT_ERR_OOM: throw yrt::device_oom(m);
        case YRT_ERR_HIP:
        case YRT_ERR_NO_DEVICE: throw yrt::device_error(m);
        default: throw std::runtime_error(m);
    }
}

thread_local std::string g_multi_error;

}  // namespace

constexpr int band_rows = 8;

struct yrt_multi {
    int n = 0;
    std::vector<int> devices;
    std::vector<yrt_scene*> scenes;
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> done;   // per device: its shard is rendered
    hipEvent_t ev_start = nullptr, ev_rendered = nullptr, ev_end = nullptr;  // on the root
    std::vector<ncclComm_t> comms;  // RCCL transport only
    bool use_rccl = false;
    // buffers: shards[r] on device r (rows_pad x W RGBA f32); on the root, the gathered
    // slots (n x shard) and, for host output, the reassembled frame
    std::vector<void*> shards;
    size_t shard_bytes = 0;
    void* gathered = nullptr;
    size_t gathered_bytes = 0;
    void* frame = nullptr;
    size_t frame_bytes = 0;
    float render_ms = 0, gather_ms = 0;

    ~yrt_multi() {
        for (int r = 0; r < (int)scenes.size(); r++) {
            (void)hipSetDevice(devices[r]);
            if (r < (int)shards.size() && shards[r]) (void)hipFree(shards[r]);
            if (r < (int)done.size() && done[r]) (void)hipEventDestroy(done[r]);
            if (r < (int)streams.size() && streams[r]) (void)hipStreamDestroy(streams[r]);
        }
        if (!devices.empty()) {
            (void)hipSetDevice(devices[0]);
            if (gathered) (void)hipFree(gathered);
            if (frame) (void)hipFree(frame);
            for (auto e : {ev_start, ev_rendered, ev_end})
                if (e) (void)hipEventDestroy(e);
        }
        for (auto c : comms)
            if (c) (void)rccl().comm_destroy(c);
        for (auto s : scenes) yrt_scene_free(s);
    }

    // device buffer `p` of at least `bytes` on `dev`
    static void grow(void*& p, size_t& have, size_t bytes, int dev, const char* what) {
        if (bytes <= have) return;
        hip_check(hipSetDevice(dev), "hipSetDevice");
        if (p) hip_check(hipFree(p), "hipFree");
        p = nullptr;
        have = 0;
        hip_check(hipMalloc(&p, bytes), what);
        have = bytes;
    }
};

namespace {

template <class F>
int guarded_multi(F&& f) {
    try {
        g_multi_error.clear();
        return f();
    } catch (const yrt::device_oom& e) {
        g_multi_error = e.what();
        return YRT_ERR_OOM;
    } catch (const yrt::device_error& e) {
        g_multi_error = e.what();
        return YRT_ERR_HIP;
    } catch (const yrt::unsupported_error& e) {
        g_multi_error = e.what();
        return YRT_ERR_UNSUPPORTED;
    } catch (const std::bad_alloc&) {
        g_multi_error = "out of memory";
        return YRT_ERR_OOM;
    } catch (const std::invalid_argument& e) {
        g_multi_error = e.what();
        return YRT_ERR_INVALID_ARG;
    } catch (const std::exception& e) {
        g_multi_error = e.what();
        return YRT_ERR_INTERNAL;
    }
}

// the multi entry points keep their own message; yrt_last_error reports it
int finish(int status) {
    if (status != YRT_OK) yrt::set_last_error(g_multi_error.c_str());
    return status;
}

}  // namespace

extern "C" {

int yrt_multi_create(const yrt_host_scene* hs, const int* devices, int n, yrt_multi** out) {
    if (!hs || !devices || n <= 0 || !out) return YRT_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        yrt::set_last_error("no HIP device visible");
        return YRT_ERR_NO_DEVICE;
    }
    for (int r = 0; r < n; r++)
        if (devices[r] < 0 || devices[r] >= ndev) {
            yrt::set_last_error("device index out of range");
            return YRT_ERR_INVALID_ARG;
        }
    return finish(guarded_multi([&] {
        auto m = new yrt_multi();
        try {
            m->n = n;
            m->devices.assign(devices, devices + n);
            std::vector<int> sorted = m->devices;
            std::sort(sorted.begin(), sorted.end());
            const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
            const char* tr = getenv("YRT_MULTI_TRANSPORT");
            const std::string want = tr ? tr : "";
            if (want == "rccl") {
                if (!distinct) throw std::invalid_argument("RCCL transport needs distinct devices");
                m->use_rccl = true;
            } else if (want == "copy" || want.empty()) {
                if (want == "copy" && n > 1 && distinct)
                    throw std::invalid_argument("copy transport is for a device listed more than once");
                m->use_rccl = n > 1 && distinct;
            } else {
                throw std::invalid_argument("YRT_MULTI_TRANSPORT must be rccl or copy");
            }
            for (int r = 0; r < n; r++) {
                yrt_scene* s = nullptr;
                yrt_check(yrt_scene_upload(hs, devices[r], &s), "yrt_scene_upload");
                m->scenes.push_back(s);
                hip_check(hipSetDevice(devices[r]), "hipSetDevice");
                hipStream_t st = nullptr;
                hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
                m->streams.push_back(st);
                hipEvent_t ev = nullptr;
                hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
                m->done.push_back(ev);
            }
            m->shards.assign(n, nullptr);
            hip_check(hipSetDevice(devices[0]), "hipSetDevice");
            hip_check(hipEventCreate(&m->ev_start), "hipEventCreate");
            hip_check(hipEventCreate(&m->ev_rendered), "hipEventCreate");
            hip_check(hipEventCreate(&m->ev_end), "hipEventCreate");
            if (m->use_rccl) {
                const rccl_api& api = rccl();
                if (!api.load_error.empty()) throw yrt::device_error(api.load_error);
                m->comms.assign(n, nullptr);
                nccl_check(api.comm_init_all(m->comms.data(), n, m->devices.data()), "ncclCommInitAll");
            }
        } catch (...) {
            delete m;
            throw;
        }
        *out = m;
        return YRT_OK;
    }));
}

void yrt_multi_free(yrt_multi* m) { delete m; }

int yrt_multi_info(const yrt_multi* m, int* n, int* transport) {
    if (!m || !n || !transport) return YRT_ERR_INVALID_ARG;
    *n = m->n;
    *transport = m->use_rccl ? YRT_TRANSPORT_RCCL : YRT_TRANSPORT_COPY;
    return YRT_OK;
}

int yrt_multi_render(yrt_multi* m, const yrt_render_params* p, float* out, int mem) {
    if (!m || !p || !out) return YRT_ERR_INVALID_ARG;
    if (p->x0 || p->y0 || p->tile_w || p->tile_h || p->band != 1 || p->band_stride != 1 || p->band_offset ||
        p->out_stride) {
        yrt::set_last_error("yrt_multi_render renders whole frames: window and band fields must be defaults");
        return YRT_ERR_INVALID_ARG;
    }
    return finish(guarded_multi([&] {
        const int n = m->n;
        int W = 0, H = 0;
        yrt_check(yrt_image_size(m->scenes[0], p, &W, &H), "yrt_image_size");
        const int nbands = (H + band_rows - 1) / band_rows;
        const int kmax = (nbands + n - 1) / n;  // bands per rank, padded
        const int rows_pad = kmax * band_rows;
        const size_t row_bytes = (size_t)W * 16;
        const size_t band_bytes = row_bytes * band_rows;
        const size_t shard = (size_t)rows_pad * row_bytes;
        const int root = m->devices[0];
        // buffers: with RCCL every rank renders into its own shard and sends it (the
        // root to itself); with copies the root renders straight into gathered slot 0
        for (int r = 0; r < n; r++)
            if (m->use_rccl || r > 0) {
                size_t have = m->shards[r] ? m->shard_bytes : 0;
                yrt_multi::grow(m->shards[r], have, shard, m->devices[r], "hipMalloc(shard)");
            }
        m->shard_bytes = std::max(m->shard_bytes, shard);
        yrt_multi::grow(m->gathered, m->gathered_bytes, shard * n, root, "hipMalloc(gathered frame)");
        float* dst = out;
        if (mem != YRT_MEM_DEVICE) {
            yrt_multi::grow(m->frame, m->frame_bytes, (size_t)H * row_bytes, root, "hipMalloc(frame)");
            dst = (float*)m->frame;
        }
        hip_check(hipSetDevice(root), "hipSetDevice");
        hip_check(hipEventRecord(m->ev_start, m->streams[0]), "hipEventRecord");

        // ---- render: one host thread per device (a reflective scene's render reads a
        // ray count back per level, so one thread would serialise the devices) ----
        std::vector<int> status(n, YRT_OK);
        std::vector<std::string> msg(n);
        auto render_rank = [&](int r) {
            yrt_render_params q = *p;
            q.band = band_rows;
            q.band_stride = n;
            q.band_offset = r;
            q.tile_h = rows_pad;  // rows past the image read zero
            q.out_stride = W;
            void* target = (m->use_rccl || r > 0) ? m->shards[r] : m->gathered;
            status[r] = yrt_render(m->scenes[r], &q, (float*)target, YRT_MEM_DEVICE, m->streams[r]);
            if (status[r] == YRT_OK) {
                if (hipSetDevice(m->devices[r]) != hipSuccess || hipEventRecord(m->done[r], m->streams[r]) != hipSuccess)
                    status[r] = YRT_ERR_HIP, msg[r] = "hipEventRecord";
            } else {
                msg[r] = yrt_last_error();
            }
        };
        if (n == 1) {
            render_rank(0);
        } else {
            std::vector<std::thread> th;
            for (int r = 0; r < n; r++) th.emplace_back(render_rank, r);
            for (auto& t : th) t.join();
        }
        if (std::any_of(status.begin(), status.end(), [](int st) { return st != YRT_OK; })) {
            // the other ranks' streams may still run kernels that write their shards: let
            // them drain before the error leaves (a later grow() or yrt_multi_free would
            // otherwise free buffers in use); their own errors are ignored here
            for (int r = 0; r < n; r++)
                if (hipSetDevice(m->devices[r]) == hipSuccess) (void)hipStreamSynchronize(m->streams[r]);
            (void)hipGetLastError();
        }
        for (int r = 0; r < n; r++)
            if (status[r] != YRT_OK) {
                yrt::set_last_error(msg[r].c_str());
                yrt_check(status[r], ("render on device " + std::to_string(m->devices[r])).c_str());
            }
        hip_check(hipSetDevice(root), "hipSetDevice");
        for (int r = 0; r < n; r++) hip_check(hipStreamWaitEvent(m->streams[0], m->done[r], 0), "hipStreamWaitEvent");
        hip_check(hipEventRecord(m->ev_rendered, m->streams[0]), "hipEventRecord");

        // ---- gather to the root ----
        char* g = (char*)m->gathered;
        if (m->use_rccl) {
            const rccl_api& api = rccl();
            const size_t count = shard / 4;  // floats
            nccl_check(api.group_start(), "ncclGroupStart");
            for (int r = 0; r < n; r++) {
                // each send is ordered after its rank's render on the rank's stream
                nccl_check(api.send(m->shards[r], count, nccl_float32, 0, m->comms[r], m->streams[r]), "ncclSend");
                nccl_check(api.recv(g + (size_t)r * shard, count, nccl_float32, r, m->comms[0], m->streams[0]),
                           "ncclRecv");
            }
            nccl_check(api.group_end(), "ncclGroupEnd");
        } else {
            for (int r = 1; r < n; r++)
                hip_check(hipMemcpyPeerAsync(g + (size_t)r * shard, root, m->shards[r], m->devices[r], shard,
                                             m->streams[0]),
                          "hipMemcpyPeerAsync");
        }
        // ---- reassemble in image order: image band b = local band k of rank b % n ----
        const int full = H / band_rows;  // complete image bands
        for (int r = 0; r < n && r < nbands; r++) {
            const int cnt = full > r ? (full - r + n - 1) / n : 0;
            if (cnt)
                hip_check(hipMemcpy2DAsync((char*)dst + (size_t)r * band_bytes, (size_t)n * band_bytes,
                                           g + (size_t)r * shard, band_bytes, band_bytes, cnt,
                                           hipMemcpyDeviceToDevice, m->streams[0]),
                          "hipMemcpy2DAsync");
        }
        if (H % band_rows) {
            const int b = full, r = b % n, k = b / n;
            hip_check(hipMemcpyAsync((char*)dst + (size_t)b * band_bytes, g + (size_t)r * shard + (size_t)k * band_bytes,
                                     (size_t)(H % band_rows) * row_bytes, hipMemcpyDeviceToDevice, m->streams[0]),
                      "hipMemcpyAsync");
        }
        hip_check(hipEventRecord(m->ev_end, m->streams[0]), "hipEventRecord");
        if (mem != YRT_MEM_DEVICE)
            hip_check(hipMemcpyAsync(out, m->frame, (size_t)H * row_bytes, hipMemcpyDeviceToHost, m->streams[0]),
                      "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(m->streams[0]), "hipStreamSynchronize");
        hip_check(hipEventElapsedTime(&m->render_ms, m->ev_start, m->ev_rendered), "hipEventElapsedTime");
        hip_check(hipEventElapsedTime(&m->gather_ms, m->ev_rendered, m->ev_end), "hipEventElapsedTime");
        return YRT_OK;
    }));
}

int yrt_multi_last_stats(yrt_multi* m, yrt_stats* out) {
    if (!m || !out) return YRT_ERR_INVALID_ARG;
    memset(out, 0, sizeof *out);
    for (auto s : m->scenes) {
        yrt_stats st;
        const int status = yrt_last_stats(s, &st);
        if (status != YRT_OK) return status;
        const unsigned long long* a = (const unsigned long long*)&st;
        unsigned long long* o = (unsigned long long*)out;
        for (size_t k = 0; k < sizeof st / sizeof *a; k++) o[k] += a[k];
    }
    return YRT_OK;
}

int yrt_multi_last_timings(const yrt_multi* m, float* render_ms, float* gather_ms) {
    if (!m || !render_ms || !gather_ms) return YRT_ERR_INVALID_ARG;
    *render_ms = m->render_ms;
    *gather_ms = m->gather_ms;
    return YRT_OK;
}

int yrt_render_multi(const yrt_host_scene* hs, const int* devices, int n, const yrt_render_params* p, float* out,
                     int mem) {
    yrt_multi* m = nullptr;
    int s = yrt_multi_create(hs, devices, n, &m);
    if (s != YRT_OK) return s;
    s = yrt_multi_render(m, p, out, mem);
    std::string keep = s != YRT_OK ? yrt_last_error() : "";
    yrt_multi_free(m);
    if (s != YRT_OK) yrt::set_last_error(keep.c_str());
    return s;
}

}  // extern "C"
