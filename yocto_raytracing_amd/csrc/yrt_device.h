// yrt_device.h -- HBM layout of a scene on one MI355X, shared by
// the host flattener (device_scene.cpp) and the gfx950 kernels (render.hip).
//
// Everything is 16-byte records so each fetch is one global_load_dwordx4:
//   tnodes  2 x f4 per instance-BVH node  {min.xyz, start} {max.xyz, count|leaf<<31}
//   tinst   4 x f4 per instance-BVH leaf slot (instances permuted to leaf order)
//           {frame.x, shape | identity << 30} {frame.y, shape wide root | kind << 30} {frame.z, material}
//           {frame.o, shape root node | kind << 30}
//   tinst_id int per instance-BVH leaf slot: the instance's index in the scene
//   snodes  2 x f4 per shape-BVH node, all shapes concatenated, child/leaf indices absolute
//   sprims  3 x f4 per shape-BVH leaf slot (primitives permuted to leaf order)
//           triangle {v0, ei} {v1-v0, -} {v2-v0, -}   (the reference's e1/e2, scene.cpp:232-233)
//           line     {v0, ei} {v1, r0}  {r1, -, -, -}
//           point    {p, ei}  {r, -, -, -} {-}
//   shapes  i4 per shape {root node, kind, elem base, vertex base}
//   elems   i4 per element (original index order) with absolute vertex indices
//   vpos/vnorm f4, vuv f2 per vertex
//   mats    4 x f4 {kd, ns} {ks, kd_txt} {kr, ks_txt} {ke, flags}
//   lights  6 x f4 {frame.x} {frame.y} {frame.z} {frame.o} {pos0 of the light shape} {ke}
//   texels  RGBA8 of every texture; texinfo i4 {offset, width, height, -}
//   srgb    256 floats: fmin(1, pow(c/255, 2.2)) (raytrace.cpp:51-53) precomputed on the host
//   wnodes  8 x f4 per 4-wide node of the any-hit walk (device_scene.cpp wide_builder):
//           {lo.x[4]} {lo.y[4]} {lo.z[4]} {hi.x[4]} {hi.y[4]} {hi.z[4]} {ref[4]} {info[4]},
//           instance level and all shapes in one array, absolute indices
//   winst   5 x f4 per instance-BVH leaf slot for the any-hit walk: the frame and the
//           object-space root box of the instance's shape (the box the reference tests
//           first on entering it, scene.cpp:386-442), packed as winst_rows describes
//   aprims  9 floats per sprims slot: a triangle's v0, e1, e2 packed (the any-hit leaf loads)
#pragma once

#include <stdint.h>

namespace yrt {

struct alignas(16) f4 {
    float x, y, z, w;
};
struct alignas(16) i4 {
    int x, y, z, w;
};
struct alignas(8) f2 {
    float x, y;
};

enum shape_kind : int { kind_triangles = 0, kind_lines = 1, kind_points = 2, kind_empty = 3 };
enum mat_flags : int { mat_reflective = 1 };

constexpr uint32_t leaf_bit = 0x80000000u;
// tinst row 0 .w: set when the instance frame's rotation rows are bitwise the identity's
constexpr uint32_t inst_identity_bit = 0x40000000u;
constexpr uint32_t inst_shape_mask = 0x3fffffffu;
// tinst row 2 .w: the material index | its shadow class << mat_class_shift. The class says
// when a light's term for a hit on the material is +-0 from the geometry alone, so that its
// shadow ray need not be traced (wavefront.hip light_term_zero): 0 never; 1 no specular
// (Ks == 0, ns in [0, FLT_MAX], |Kd| <= 2^20); c >= 2 specular with ns >= mat_class_ns(c)
// (|Kd|, |Ks| <= 2^20). Materials are limited to 2^24.
constexpr int mat_class_shift = 24;
constexpr uint32_t mat_index_mask = 0x00ffffffu;
constexpr int mat_class_max = 15;
constexpr float mat_class_ns(int c) { return (float)(16 << (c - 2)); }  // c in [2, 15]: 16 .. 131072

// winst (the any-hit walk's instance records) packs what that walk reads into five rows --
// {frame.x, tinst row 0 .w} {frame.y, wide root | kind} {frame.z, box lo.x}
// {frame.o, box lo.y} {box lo.z, hi.x, hi.y, hi.z} -- one s_load_dwordx16 + x4 (20 SGPRs)
// instead of tinst's four rows plus two box rows (x16 + x8, 24 SGPRs)
constexpr int winst_rows = 5;

// 4-wide any-hit records (device_scene.cpp wide_builder): 128 bytes per wide node --
// six f4 rows of child bounds {lo.x[4]}, {lo.y[4]}, {lo.z[4]}, {hi.x[4]}, {hi.y[4]},
// {hi.z[4]}, one f4 of child words, one f4 {slot count, -, -, -}. A child word is the
// child record's byte offset (inner: usable as the load's SGPR offset as is), or
// wide_leaf | count << wide_count_shift | first slot (a leaf of the reference BVH).
constexpr uint32_t wide_leaf = 0x80000000u;
constexpr int wide_count_shift = 28;
constexpr uint32_t wide_index_mask = 0x0fffffffu;
constexpr int wide_record_bytes = 128;
// a shadow bundle's leaf word (wavefront.hip k_bundle_lists, when the view's inst_masks is
// set): wide_leaf | count << 28 | skip << 21 | first slot, skip bit i = the leaf's instance i
// is excluded by the bundle's hull (first < 2^21)
constexpr uint32_t bundle_first_mask = 0x1fffffu;
constexpr int bundle_skip_shift = 21;
constexpr uint32_t bundle_leaf_word(int first, int count, uint32_t skip) {
    return wide_leaf | (uint32_t)count << wide_count_shift | (skip & 0x7fu) << bundle_skip_shift | (uint32_t)first;
}
// the depth of the instance tree's cut the camera lists start from (k_camera_lists): 0 = the
// root alone; at most 2^depth entries, which must fit one list (camera_list_max)
#ifndef YRT_CAMERA_CUT_DEPTH
#define YRT_CAMERA_CUT_DEPTH 5
#endif
constexpr int camera_cut_depth = YRT_CAMERA_CUT_DEPTH;
constexpr int spine_len = 2;  // nodes per closest-hit walk record (a node and its child start+1)
// spine records (tpair/spair): spine_len x {lo, hi} f4 pairs; an inner node's lo.w is
// the byte offset of its child start's record (child start+1's is the next record)
constexpr int spine_record_bytes = 32 * spine_len;
constexpr int spine_record_f4 = spine_record_bytes / 16;

struct dev_scene_view {
    const f4* tnodes;
    const f4* tinst;
    const f4* snodes;
    const f4* sprims;
    const i4* shapes;
    const i4* elems;
    const f4* vpos;
    const f4* vnorm;
    const f2* vuv;
    const f4* mats;
    const f4* lights;
    const uint32_t* texels;
    const i4* texinfo;
    const float* srgb;
    const f4* wnodes;
    const f4* winst;
    const float* aprims;  // 9 floats per sprims slot: a triangle's v0, e1, e2 (any-hit walk)
    const f4* tpair;  // 2*spine_len x f4 per instance-BVH node: its record, then its
                      // child start+1's, that child's start+1's, ... (right spine)
    const f4* spair;  // the same for the shape BVHs (same indexing as snodes)
    const int* tinst_id;
    // per instance slot: a world-space box holding every point whose instance-space image
    // lies in the shape's root box, grown by a margin far above the rounding of the walks'
    // instance transforms (device_scene.cpp), NaN for frames it cannot bound; the list
    // builders drop the instances of a listed leaf that their cone or hull excludes
    const f4* ibox;
    // the camera lists' starting frontier: the instance tree's cut at depth camera_cut_depth
    // in the reference's DFS order, as byte offsets of the nodes' records (device_scene.cpp)
    const int* tcut;
    int ntcut;
    int inst_masks;  // 1: instance slots fit the bundle records' 21-bit first-slot field
    int wtop_root;
    int nwtop;  // records of the instance-level wide tree (breadth first: the top levels lead)
    int wide;  // 1: any-hit queries use the 4-wide walk
    int nlights;
    int ntnodes;
    int ntextures;
#ifdef YRT_DEBUG_BOUNDS  // diagnostic build: array sizes for the walks' bounds checks
    int nsnodes, nsprims, ninst, nwnodes;
#endif
};

// per-frame camera constants, hoisted from eval_camera (raytrace.cpp:16-24); tanf is
// evaluated on the host with the same libm call the reference makes
struct dev_camera {
    float ox, oy, oz;
    float xx, xy, xz;
    float yx, yy, yz;  // frame.y * -1
    float zx, zy, zz;
    float h, w, focus;
};

struct dev_render_args {
    dev_camera cam;
    float amb[3];
    int width, height;  // full image size (uv denominators, raytrace.cpp:237-238)
    int samples;        // per axis
    int max_depth;      // trace_first calls per camera sample (reference: unbounded)
    int x0, tile_w;     // columns [x0, x0+tile_w)
    int y0, tile_h;     // local rows [0, tile_h): image row = y0 + band interleave
    int band, band_stride, band_offset;  // local band b -> image band b*band_stride+band_offset
    int out_stride;     // floats4 per output row
};

// device counters (u64): rays, camera samples, depth-truncated paths, stack overflows,
// then the optional work counters (box tests, instance entries, primitive tests, hits)
enum counter_index {
    cnt_rays = 0,
    cnt_samples = 1,
    cnt_depth_truncated = 2,
    cnt_stack_overflow = 3,
    cnt_box_tests = 4,
    cnt_inst_entries = 5,
    cnt_prim_tests = 6,
    cnt_shaded_hits = 7,
    cnt_tex_lookups = 8,
    // the shadow-ray phase alone (k_shadow), for its own roofline
    cnt_shadow_rays = 9,
    cnt_shadow_box_tests = 10,
    cnt_shadow_inst_entries = 11,
    cnt_shadow_prim_tests = 12,
    // the packet walk: node records / primitive records fetched per WAVE (one per
    // step whatever the number of active lanes): lanes-per-step = box_tests / this
    cnt_wave_node_visits = 13,
    cnt_wave_prim_visits = 14,
    cnt_shadow_wave_node_visits = 15,
    // shadow rays counted (the reference's intersect_any calls) but answered without a walk:
    // their light term is exactly zero (wavefront.hip light_term_zero), recorded as occluded
    cnt_shadow_culled = 16,
    cnt_count = 32  // (17 used; a line is two 128-byte cache lines)
};

// The counters live in cnt_slots lines of cnt_count u64 (256 bytes each); a wave adds
// its sums into the line picked by its global wave index and the host adds the lines.
// One shared address for every wave serialises the device-scope atomics: with a
// single line the per-wave counter flush alone cost ~30 ms of a 78 ms c4 shadow pass.
constexpr int cnt_slots = 1024;
static_assert(cnt_count * 8 % 128 == 0, "a counter line is whole 128-byte cache lines");

}  // namespace yrt
