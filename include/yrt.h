/* yrt.h -- C-ABI of the MI355X-native renderer for the yocto_raytracing hot path.
 *
 * Plain C: opaque handles, plain pointers and sizes, int status codes, no
 * exceptions and no torch types across the boundary. Every entry point names the
 * reference interface it replaces (reference = sebcossu/yocto_raytracing, src/).
 *
 * Typical use, mirroring main() in src/raytrace.cpp:256-287:
 *     yrt_host_scene* hs;  yrt_scene_load("scene.obj", &hs);       // load_scene
 *     yrt_host_scene_build_bvh(hs, 0);                             // build_bvh(scn, false)
 *     yrt_scene* ds;  yrt_scene_upload(hs, 0, &ds);                // (new) copy to HBM
 *     yrt_render_params p;  yrt_render_params_default(&p);  p.resolution = 720; p.samples = 3;
 *     int w, h;  yrt_image_size(ds, &p, &w, &h);
 *     yrt_render(ds, &p, host_rgba_w_h_4, YRT_MEM_HOST, NULL);     // raytrace()
 *     yrt_save_image("out.png", host_rgba_w_h_4, w, h);            // save_hdr_or_ldr
 */
#ifndef YRT_H
#define YRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YRT_ABI_VERSION 1

/* status codes (the reference has none: it exit(1)s in the loader, scene.cpp:119-122) */
enum {
    YRT_OK = 0,
    YRT_ERR_INVALID_ARG = 1,
    YRT_ERR_IO = 2,          /* file missing / unreadable / malformed */
    YRT_ERR_UNSUPPORTED = 3, /* input the kernels do not handle (mixed shapes, hdr textures, deep BVH) */
    YRT_ERR_HIP = 4,         /* HIP runtime error (message via yrt_last_error) */
    YRT_ERR_NO_DEVICE = 5,
    YRT_ERR_OOM = 6,
    YRT_ERR_INTERNAL = 7
};

typedef struct yrt_host_scene yrt_host_scene; /* host scene + BVH (scene*, scene.h:136-155) */
typedef struct yrt_scene yrt_scene;           /* scene resident in one GPU's HBM */

/* memory location of a caller buffer */
enum { YRT_MEM_HOST = 0, YRT_MEM_DEVICE = 1 };

typedef struct yrt_render_params {
    float ambient[3];  /* raytrace(..., amb, ...): main() passes {a,a,a}, a = -a (0.1) */
    int resolution;    /* vertical resolution -r (raytrace.cpp:216) */
    int width;         /* 0: round(camera.aspect * resolution) as the reference; >0: explicit */
    int samples;       /* -s: samples PER AXIS, s*s per pixel (raytrace.cpp:232-234) */
    int max_depth;     /* trace_first calls per camera sample; reference: unbounded. 0 -> 16.
                          Any depth with the wavefront algorithms (per-level records in HBM);
                          the megakernel keeps 16 per lane (deeper: YRT_ERR_UNSUPPORTED) */
    int camera;        /* camera index; reference: cameras.front() == 0 */
    int x0, y0;        /* window origin in image pixels */
    int tile_w, tile_h;/* window size; 0 -> to the image edge */
    int band;          /* row interleave for multi-GPU sharding: rows are taken in bands of */
    int band_stride;   /*   `band` rows; local band b is image band b*band_stride+band_offset */
    int band_offset;   /*   (band=1,stride=1,offset=0: contiguous rows) */
    int out_stride;    /* output row stride in pixels; 0 -> tile_w */
    int count_work;    /* 1: also count box/instance/primitive tests (slower; for roofline bytes) */
    int algorithm;     /* YRT_ALGO_*: identical results, different schedules */
    int timing;        /* 1: record HIP events per kernel phase (read with yrt_last_timings);
                          2: keep adding to the previous record (time a loop of renders) */
} yrt_render_params;

/* render algorithms: identical outputs, different schedules
 *   WAVEFRONT       kernel per stage, one lane per camera sample, wave-coherent (packet) BVH walk
 *   MEGAKERNEL      one kernel, one lane per pixel walking the reference's loops
 *   WAVEFRONT_LANE  kernel per stage, one independent BVH walk per lane */
enum { YRT_ALGO_WAVEFRONT = 0, YRT_ALGO_MEGAKERNEL = 1, YRT_ALGO_WAVEFRONT_LANE = 2 };
enum { YRT_LISTS_AUTO = 0, YRT_LISTS_ON = 1, YRT_LISTS_OFF = 2 };

/* counters accumulated by the last yrt_render / yrt_trace_* on a scene handle */
typedef struct yrt_stats {
    unsigned long long rays;            /* intersect_first + intersect_any calls */
    unsigned long long camera_samples;  /* eval_camera calls */
    unsigned long long depth_truncated; /* paths cut by max_depth (0 = parity-neutral) */
    unsigned long long stack_overflow;
    unsigned long long box_tests;       /* count_work only */
    unsigned long long instance_entries;
    unsigned long long prim_tests;
    unsigned long long shaded_hits;
    unsigned long long texture_lookups;
    unsigned long long shadow_rays;     /* the shadow-ray phase alone (intersect_any calls; the
                                         * reference's count: a shadow ray whose light term is
                                         * exactly zero is counted but not traced, DESIGN.md §5,
                                         * see shadow_rays_culled) */
    unsigned long long shadow_box_tests;        /* count_work only */
    unsigned long long shadow_instance_entries; /* count_work only */
    unsigned long long shadow_prim_tests;       /* count_work only */
    unsigned long long wave_node_visits;        /* count_work, packet walk: node steps per wave */
    unsigned long long wave_prim_visits;        /* count_work, packet walk: primitive steps per wave */
    unsigned long long shadow_wave_node_visits; /* the same, shadow-ray phase alone */
    unsigned long long shadow_rays_culled;      /* of shadow_rays: answered without a walk because
                                                 * the light term is exactly zero (recorded as
                                                 * occluded; 0 with count_work, which walks every
                                                 * ray). Rays walked = rays - shadow_rays_culled */
} yrt_stats;

/* GPU time per kernel phase of the last render (HIP events on the launch stream) */
enum {
    YRT_PHASE_PRIMARY = 0,    /* camera rays + closest hit + surface */
    YRT_PHASE_SHADOW = 1,     /* shadow rays (any hit) */
    YRT_PHASE_SHADE = 2,      /* lighting + mirror-ray compaction */
    YRT_PHASE_BOUNCE = 3,     /* closest hit of mirror rays */
    YRT_PHASE_FOLD = 4,       /* reflection fold */
    YRT_PHASE_ACCUMULATE = 5, /* ordered per-pixel sum */
    YRT_PHASE_MEGAKERNEL = 6, /* the one-kernel path */
    YRT_PHASE_LISTS = 7,      /* per-render camera-relative records and candidate-leaf lists */
    YRT_PHASE_COUNT = 8
};
typedef struct yrt_timings {
    float ms[YRT_PHASE_COUNT];
    int launches[YRT_PHASE_COUNT];
} yrt_timings;

/* ---- library ---- */
int yrt_abi_version(void);
const char* yrt_status_string(int status);
/* message of the last error on this thread (empty string if none) */
const char* yrt_last_error(void);
int yrt_device_count(int* count);

/* ---- host scene: loader, serialisation, BVH ---- */
/* load_scene (src/scene.cpp:113-225): Yocto OBJ (.obj) or the .yrtscene interchange file */
int yrt_scene_load(const char* path, yrt_host_scene** out);
/* serialise the shading-relevant arrays (.yrtscene, gzip) */
int yrt_scene_save(const yrt_host_scene* hs, const char* path);
/* build_bvh(scene*, bool equal_num) (src/scene.cpp:554-565, decl scene.h:238) */
int yrt_host_scene_build_bvh(yrt_host_scene* hs, int equal_num);
/* build_bvh with the tree construction (node boxes, splits, partitions) on GPU `device`:
 * the same nodes and leaf order as yrt_host_scene_build_bvh, byte for byte. equal_num != 0
 * is YRT_ERR_UNSUPPORTED. kernel_ms (may be NULL): GPU time of the build's level passes */
int yrt_host_scene_build_bvh_gpu(yrt_host_scene* hs, int equal_num, int device, float* kernel_ms);
/* dump the BVHs (.yrtbvh) byte-compatible with the reference's bvh_node (scene.h:9-15) */
int yrt_host_scene_save_bvh(const yrt_host_scene* hs, const char* path);
/* counts: [cameras, textures, materials, shapes, instances, lights, bvh nodes(instance
 * level), bvh depth(instance level), max shape bvh depth, triangles, lines, points] */
int yrt_host_scene_info(const yrt_host_scene* hs, long long* info12);
/* image size raytrace() would produce: W = round(aspect*res), H = res (raytrace.cpp:215-216) */
int yrt_host_image_size(const yrt_host_scene* hs, int camera, int resolution, int* w, int* h);
void yrt_host_scene_free(yrt_host_scene* hs);

/* ---- host scene from memory: the reference's scene* built field by field ----
 * For a host program that already holds a scene (scene.h:26-155) -- e.g. the
 * reference's own main() after load_scene -- instead of a file. Arrays are copied.
 * Frames are 12 floats {x.xyz, y.xyz, z.xyz, o.xyz} (frame3f, vmath.h). Indices
 * returned through `index` are what materials/instances refer to (-1 = none). */
typedef struct yrt_material_desc { /* material, scene.h:62-86 */
    float ke[3], kd[3], ks[3], kr[3];
    float rs;
    int kd_txt, ks_txt; /* texture index or -1 */
} yrt_material_desc;
typedef struct yrt_shape_desc { /* shape, scene.h:26-50; one primitive kind per shape */
    int npos;
    const float* pos;      /* npos x 3 */
    const float* norm;     /* npos x 3 or NULL */
    const float* texcoord; /* npos x 2 or NULL */
    const float* radius;   /* npos or NULL (required for points/lines) */
    int npoints;
    const int* points;     /* npoints */
    int nlines;
    const int* lines;      /* nlines x 2 */
    int ntriangles;
    const int* triangles;  /* ntriangles x 3 */
} yrt_shape_desc;
int yrt_host_scene_create(yrt_host_scene** out);
/* camera, scene.h:115-123 */
int yrt_host_scene_add_camera(yrt_host_scene* hs, const float frame[12], float fovy, float aspect, float aperture,
                              float focus, int* index);
/* texture, scene.h:54-58: 8-bit RGBA rows, pixels[j*w+i] */
int yrt_host_scene_add_texture(yrt_host_scene* hs, int w, int h, const unsigned char* rgba8, int* index);
int yrt_host_scene_add_material(yrt_host_scene* hs, const yrt_material_desc* m, int* index);
int yrt_host_scene_add_shape(yrt_host_scene* hs, const yrt_shape_desc* s, int* index);
/* instance, scene.h:99-111 */
int yrt_host_scene_add_instance(yrt_host_scene* hs, const float frame[12], int shape, int material, int* index);

/* ---- device scene ---- */
/* flatten to the HBM layout and upload to `device` (needs a built BVH) */
int yrt_scene_upload(const yrt_host_scene* hs, int device, yrt_scene** out);
size_t yrt_scene_device_bytes(const yrt_scene* ds);
void yrt_scene_free(yrt_scene* ds);

/* ---- the hot path ---- */
void yrt_render_params_default(yrt_render_params* p);
int yrt_image_size(const yrt_scene* ds, const yrt_render_params* p, int* w, int* h);
/* raytrace() (src/raytrace.cpp:213-254). out: RGBA f32, row-major pixels[j*W+i]
 * (image4f, image.h:8-17) restricted to the params window/bands; `mem` says whether
 * `out` is a host or device pointer; `stream` is a hipStream_t (NULL = default).
 * A host `out` makes the call synchronous; a device `out` is stream-ordered. */
int yrt_render(yrt_scene* ds, const yrt_render_params* p, float* out, int mem, void* stream);
/* batch intersect_first (src/scene.cpp:483-488). rays: n x {o.xyz, d.xyz, tmin, tmax}.
 * Outputs per ray: hit (0/1), instance index (-1 on miss), element index ei (-1 on miss),
 * ew[4] barycentrics, dist. All pointers in `mem` space. */
int yrt_trace_first(yrt_scene* ds, const float* rays, int n, unsigned char* hit, int* inst, int* ei,
                    float* ew, float* dist, int mem, void* stream);
/* batch intersect_any (src/scene.cpp:489-493) */
int yrt_trace_any(yrt_scene* ds, const float* rays, int n, unsigned char* hit, int mem, void* stream);
/* walks used by yrt_trace_first/any on this handle (identical results): YRT_ALGO_WAVEFRONT
 * (default) = the render path's wave-coherent closest-hit walk and 4-wide any-hit walk;
 * YRT_ALGO_MEGAKERNEL / YRT_ALGO_WAVEFRONT_LANE = one independent walk per lane */
int yrt_scene_set_trace_algorithm(yrt_scene* ds, int algorithm);
/* per-tile candidate lists of yrt_render (camera frontier lists and shadow
 * bundles; identical images either way): YRT_LISTS_ON builds them whenever the scene allows
 * (an instance tree of >= 8 wide records; shadow bundles for at most 8 lights, a rotated
 * light's rays walking the tree; ON also runs level 0's shadow rays on the persistent grid at
 * any frame size), YRT_LISTS_AUTO (default) does the same from 9 samples per pixel (their
 * cost is per pixel tile, their gain per sample), YRT_LISTS_OFF never builds them. No mode
 * reads anything back during a render. Set it between renders of the handle, not while one
 * is in flight. */
int yrt_scene_set_tile_lists(yrt_scene* ds, int mode);
/* the lists' state after the last yrt_render on this handle (synchronises with it):
 * whether each kind is in use, and sums[4] = {camera-list entries, camera lists, bundle-list
 * entries, bundle lists} of the last render that built lists (a list that fell back to the
 * tree counts as its capacity + 1) */
int yrt_scene_tile_lists(yrt_scene* ds, int* camera_on, int* bundles_on, unsigned long long* sums);
/* the instances the lists' masks excluded in the last render that built lists (synchronises
 * with it): excluded[0] = over every camera list's leaves, the instances whose world box the
 * tile's cone excludes; excluded[1] = the same over every shadow bundle's list and its hull
 * (instance masks; the walks pass over them, identical images) */
int yrt_scene_tile_list_masks(yrt_scene* ds, unsigned long long* excluded);
/* LDS staging of the instance tree's hot top (the north_star's "hot node tiles staged in LDS";
 * DESIGN.md §5). on = 1: yrt_render's persistent closest-hit grid copies the first 511
 * camera-relative spine records, and its persistent any-hit grid the first 85 4-wide records
 * (scenes with at least that many), into LDS once per block, and the walks read those records
 * from LDS instead of through the scalar cache. The tile lists are not built while it is on:
 * their walks start below the tree's top. Identical images either way. Off (0) by default:
 * measured slower, the top records being scalar-cache hits already. Set it between renders. */
int yrt_scene_set_lds_staging(yrt_scene* ds, int on);
/* what the last yrt_render on this handle staged: bit 0 the closest hit, bit 1 the any hit */
int yrt_scene_lds_staging(yrt_scene* ds, int* staged);
/* counters of the last render/trace call on this handle (synchronises the stream) */
int yrt_last_stats(yrt_scene* ds, yrt_stats* stats);
/* per-phase GPU times of the last yrt_render with p->timing = 1 (synchronises) */
int yrt_last_timings(yrt_scene* ds, yrt_timings* timings);

/* ---- image output ---- */
/* tonemap (src/image.cpp:55-77, exposure 0, srgb) of n RGBA f32 pixels into RGBA8 */
int yrt_tonemap(const float* rgba, int n, unsigned char* out, int mem, void* stream);
/* save_hdr_or_ldr (src/image.cpp:81-88): .hdr -> RGBE, else PNG of the tonemap */
int yrt_save_image(const char* path, const float* rgba, int w, int h);
/* the same for a frame in `mem` space: with YRT_MEM_DEVICE the PNG's tonemap runs on the
 * GPU (the stream's device) and only the RGBA8 image crosses PCIe; .hdr copies the floats */
int yrt_save_image_mem(const char* path, const float* rgba, int w, int h, int mem, void* stream);

/* ---- the GPUs of one node, one host process ----
 * Replaces main()'s single raytrace() call (src/raytrace.cpp:282) for N devices: the
 * scene is replicated on every device, device r renders the interleaved 8-row image
 * bands r, r+n, r+2n, ..., and the float framebuffer is gathered to devices[0] over
 * RCCL (grouped ncclSend/ncclRecv over xGMI) and reassembled in image order. A device
 * listed twice uses plain device copies instead (a rehearsal on fewer GPUs). */
typedef struct yrt_multi yrt_multi;
enum { YRT_TRANSPORT_COPY = 0, YRT_TRANSPORT_RCCL = 1 };
int yrt_multi_create(const yrt_host_scene* hs, const int* devices, int n, yrt_multi** out);
void yrt_multi_free(yrt_multi* m);
/* n devices and the gather transport (YRT_TRANSPORT_*) */
int yrt_multi_info(const yrt_multi* m, int* n, int* transport);
/* raytrace() of the whole frame (window/band fields of p must be defaults). out: W*H*4
 * floats, host memory or device memory on devices[0]. Synchronous. */
int yrt_multi_render(yrt_multi* m, const yrt_render_params* p, float* out, int mem);
/* counters of the last yrt_multi_render summed over the devices */
int yrt_multi_last_stats(yrt_multi* m, yrt_stats* stats);
/* ms of the last yrt_multi_render on the root's stream: until every shard is rendered,
 * then gather + reassembly */
int yrt_multi_last_timings(const yrt_multi* m, float* render_ms, float* gather_ms);
/* one-shot: create, render, free */
int yrt_render_multi(const yrt_host_scene* hs, const int* devices, int n, const yrt_render_params* p, float* out,
                     int mem);

#ifdef __cplusplus
}
#endif
#endif /* YRT_H */
