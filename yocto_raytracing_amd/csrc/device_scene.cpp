// device_scene.cpp -- flatten a host scene into the HBM layout of yrt_device.h and
// upload it as one arena (one hipMalloc, one copy per section).
//
// Semantics carried over from the reference's pointer graph (src/scene.h) into
// indices, so the kernels can reproduce raytrace()/shade() exactly:
//   * the light list is the instances whose material has ke.x>0 && ke.y>0 && ke.z>0,
//     in instance order -- the same iteration shade() performs over ALL instances
//     (raytrace.cpp:121-126), minus the ones that fail the test
//   * light position = transform_point(frame, pos.front() - p) needs pos.front() of
//     the light's shape (raytrace.cpp:129-130)
//   * ns = rs ? 2/pow(rs,4) - 2 : 1e6 (raytrace.cpp:143-144) and the sRGB texel table
//     fmin(1, pow(c/255, 2.2)) (raytrace.cpp:47-53) are evaluated with the host libm,
//     the same calls the reference makes per shading point
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "yrt_render.h"

namespace yrt {
namespace {

float as_float(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
float as_float(int i) { return as_float((uint32_t)i); }

f4 node_lo(const bvh_node& n, uint32_t start) { return {n.bbox.min.x, n.bbox.min.y, n.bbox.min.z, as_float(start)}; }
f4 node_hi(const bvh_node& n) {
    uint32_t c = (uint32_t)n.count | (n.isleaf ? leaf_bit : 0u);
    return {n.bbox.max.x, n.bbox.max.y, n.bbox.max.z, as_float(c)};
}

void check(hipError_t e, const char* what) {
    if (e == hipErrorOutOfMemory) throw device_oom(std::string(what) + ": " + hipGetErrorString(e));
    if (e != hipSuccess) throw device_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct arena_builder {
    struct section {
        const void* src;
        size_t bytes;
        size_t offset;
    };
    std::vector<section> sections;
    size_t total = 0;
    size_t add(const void* src, size_t bytes) {
        size_t off = total;
        sections.push_back({src, bytes, off});
        total += (bytes + 255) & ~size_t(255);
        if (bytes == 0) total += 256;  // keep every pointer distinct and valid
        return off;
    }
};

// 4-wide collapse of a binary BVH for the any-hit walk: a wide node
// holds the children of a binary node X with every INNER child replaced by its two
// children, so one visit tests up to four boxes two levels below X. The boxes, the
// leaves and the primitive order are the reference's; only the inner boxes that are
// skipped are not tested. For an any-hit query that changes nothing: a box test is
// monotone in the box (a box inside another passes only if the outer one passes,
// NaN slabs included, trace_common.h box_hit), so every leaf reached here is one the
// reference reaches too, and the answer of intersect_any does not depend on the order
// in which the leaves are tested.
// Record (8 x f4, 128 bytes): lo.x[4] lo.y[4] lo.z[4] hi.x[4] hi.y[4] hi.z[4], then
// per slot the reference (wide node index, or first leaf slot + `leaf_base`) and the
// info (0 empty slot, 1 inner, count | leaf_bit for a leaf).
// A binary tree over the LEAVES of a reference BVH, built with binned SAH, for the
// any-hit walk only. Its leaves are the reference's leaves (same boxes, same primitive
// slots); its inner boxes are unions of leaf boxes, so each one contains every leaf
// below it. A box test is monotone in the box (NaN slabs included), so a leaf's own box
// passing implies every ancestor's passes -- in this tree and in the reference's alike:
// the set of leaves a ray reaches is the same in both trees, and so is the any-hit
// answer, which does not depend on the order. What changes is how many inner boxes the
// walk tests to get there. (The closest-hit walk keeps the reference tree: its tie-break
// depends on the order.)
struct sah_builder {
    struct item {
        bbox3f box;
        vec3f c;
        int leaf;  // reference node index
    };
    const bvh_tree& ref;
    std::vector<item> items;
    bvh_tree out;
    int max_depth = 0;

    static float area(const bbox3f& b) {
        const vec3f d = b.max - b.min;
        return d.x * d.y + d.y * d.z + d.z * d.x;
    }

    explicit sah_builder(const bvh_tree& t) : ref(t) {
        for (size_t i = 0; i < t.nodes.size(); i++)
            if (t.nodes[i].isleaf) {
                const bbox3f& b = t.nodes[i].bbox;
                items.push_back({b, (b.min + b.max) * 0.5f, (int)i});
            }
        out.leaf_prims = t.leaf_prims;
        if (items.empty()) return;
        out.nodes.reserve(2 * items.size());
        out.nodes.push_back({});
        build(0, 0, (int)items.size(), 1);
    }

    void build(int x, int b, int e, int depth) {
        max_depth = std::max(max_depth, depth);
        bbox3f box = invalid_bbox3f, cb = invalid_bbox3f;
        for (int i = b; i < e; i++) box = expand_bbox(box, items[i].box), cb = expand_bbox(cb, items[i].c);
        if (e - b == 1) {
            out.nodes[x] = ref.nodes[items[b].leaf];
            return;
        }
        // binned SAH over the leaf centroids, every axis
        constexpr int NB = 32;
        float best = INFINITY;
        int best_axis = -1, best_bin = 0;
        for (int a = 0; a < 3; a++) {
            const float lo = (&cb.min.x)[a], hi = (&cb.max.x)[a];
            if (!(hi > lo)) continue;
            bbox3f bb[NB];
            int bn[NB] = {};
            for (auto& q : bb) q = invalid_bbox3f;
            for (int i = b; i < e; i++) {
                int k = (int)((((&items[i].c.x)[a]) - lo) / (hi - lo) * NB);
                k = std::min(std::max(k, 0), NB - 1);
                bb[k] = expand_bbox(bb[k], items[i].box);
                bn[k]++;
            }
            float la[NB];
            int ln[NB];
            bbox3f acc = invalid_bbox3f;
            int n = 0;
            for (int k = 0; k < NB; k++) {
                acc = expand_bbox(acc, bb[k]);
                n += bn[k];
                la[k] = n ? area(acc) : 0.0f, ln[k] = n;
            }
            acc = invalid_bbox3f;
            n = 0;
            for (int k = NB - 1; k > 0; k--) {
                acc = expand_bbox(acc, bb[k]);
                n += bn[k];
                if (!n || !ln[k - 1]) continue;
                const float cost = la[k - 1] * (float)ln[k - 1] + area(acc) * (float)n;
                if (cost < best) best = cost, best_axis = a, best_bin = k;
            }
        }
        int mid;
        if (best_axis < 0) {  // coincident centroids: split the range in half
            mid = (b + e) / 2;
        } else {
            const float lo = (&cb.min.x)[best_axis], hi = (&cb.max.x)[best_axis];
            auto it = std::partition(items.begin() + b, items.begin() + e, [&](const item& q) {
                int k = (int)((((&q.c.x)[best_axis]) - lo) / (hi - lo) * NB);
                k = std::min(std::max(k, 0), NB - 1);
                return k < best_bin;
            });
            mid = (int)(it - items.begin());
            if (mid == b || mid == e) mid = (b + e) / 2;
        }
        const int c = (int)out.nodes.size();
        out.nodes.push_back({});
        out.nodes.push_back({});
        bvh_node& n = out.nodes[x];
        n.bbox = box;
        n.start = (uint32_t)c;
        n.count = 2;
        n.isleaf = 0;
        n.axis = (uint8_t)std::max(best_axis, 0);
        build(c, b, mid, depth + 1);
        build(c + 1, mid, e, depth + 1);
    }
};

struct wide_builder {
    std::vector<f4>& out;
    int max_depth = 0;

    // the slots of the wide node made from binary node x: x's children, each inner child
    // replaced by its own two children (a leaf root is its own single slot)
    std::vector<int> slots_of(const bvh_tree& t, int x) const {
        std::vector<int> slots;
        const bvh_node& n = t.nodes[x];
        auto area = [&](int i) {
            const bbox3f& b = t.nodes[i].bbox;
            const vec3f d = b.max - b.min;
            return d.x * d.y + d.y * d.z + d.z * d.x;
        };
        if (n.isleaf) {
            slots.push_back(x);
        } else {
            for (int c : {(int)n.start + 1, (int)n.start}) {  // the reference visits start+1 first
                const bvh_node& cn = t.nodes[c];
                if (cn.isleaf) {
                    slots.push_back(c);
                } else {
                    slots.push_back((int)cn.start + 1);
                    slots.push_back((int)cn.start);
                }
            }
        }
        // The any-hit walk enters the first passing slot and pops the others in slot
        // order; the order does not change any answer. Smallest surface area first
        // (A/B at c4: shadow -2.7 %; largest first +1.7 %).
        std::stable_sort(slots.begin(), slots.end(), [&](int a, int b) { return area(a) < area(b); });
        return slots;
    }

    int alloc() {
        const int me = (int)out.size() / 8;
        out.resize(out.size() + 8, f4{0, 0, 0, 0});
        return me;
    }

    // record `me` for `slots`; child(k) gives the record index of inner slot k
    template <class Child>
    void write(const bvh_tree& t, int me, const std::vector<int>& slots, uint32_t leaf_base, Child&& child) {
        float v[6][4];
        // child words (yrt_device.h wide_*): an inner child is its record's byte offset,
        // a leaf is leaf bit | count << 28 | first slot; an empty slot is a leaf with no
        // slots behind an inverted infinite box (no finite or infinite ray passes it; a
        // NaN ray, which passes every box, finds nothing there)
        uint32_t word[4] = {wide_leaf, wide_leaf, wide_leaf, wide_leaf};
        for (int k = 0; k < 4; k++) {
            if (k >= (int)slots.size()) {
                for (int a = 0; a < 3; a++) v[a][k] = INFINITY, v[3 + a][k] = -INFINITY;
                continue;
            }
            const bvh_node& s = t.nodes[slots[k]];
            v[0][k] = s.bbox.min.x, v[1][k] = s.bbox.min.y, v[2][k] = s.bbox.min.z;
            v[3][k] = s.bbox.max.x, v[4][k] = s.bbox.max.y, v[5][k] = s.bbox.max.z;
            if (s.isleaf) {
                const uint32_t first = s.start + leaf_base;
                if (first > wide_index_mask || s.count > 7)
                    throw unsupported_error("scene too large for the wide any-hit records");
                word[k] = wide_leaf | ((uint32_t)s.count << wide_count_shift) | first;
            } else {
                const size_t off = (size_t)child(k) * wide_record_bytes;
                if (off > wide_index_mask) throw unsupported_error("scene too large for the wide any-hit records");
                word[k] = (uint32_t)off;
            }
        }
        for (int a = 0; a < 6; a++) out[(size_t)me * 8 + a] = {v[a][0], v[a][1], v[a][2], v[a][3]};
        out[(size_t)me * 8 + 6] = {as_float((int)word[0]), as_float((int)word[1]), as_float((int)word[2]),
                                   as_float((int)word[3])};
        out[(size_t)me * 8 + 7] = {as_float((int)slots.size()), 0, 0, 0};
    }

    // depth first: a node's record, then its inner children's subtrees in slot order
    int emit(const bvh_tree& t, int x, uint32_t leaf_base, int depth) {
        max_depth = std::max(max_depth, depth);
        const std::vector<int> slots = slots_of(t, x);
        const int me = alloc();
        int idx[4] = {-1, -1, -1, -1};
        for (int k = 0; k < (int)slots.size(); k++)
            if (!t.nodes[slots[k]].isleaf) idx[k] = emit(t, slots[k], leaf_base, depth + 1);
        write(t, me, slots, leaf_base, [&](int k) { return idx[k]; });
        return me;
    }

    // breadth first: the records of the top levels come first (the part of the instance
    // tree the persistent any-hit kernel stages in LDS)
    int emit_bfs(const bvh_tree& t, int root, uint32_t leaf_base) {
        struct item {
            int x, me, depth;
        };
        std::vector<item> q = {{root, alloc(), 1}};
        for (size_t h = 0; h < q.size(); h++) {
            const item it = q[h];
            max_depth = std::max(max_depth, it.depth);
            const std::vector<int> slots = slots_of(t, it.x);
            int idx[4] = {-1, -1, -1, -1};
            for (int k = 0; k < (int)slots.size(); k++)
                if (!t.nodes[slots[k]].isleaf) {
                    idx[k] = alloc();
                    q.push_back({slots[k], idx[k], it.depth + 1});
                }
            write(t, it.me, slots, leaf_base, [&](int k) { return idx[k]; });
        }
        return q.front().me;
    }
};

}  // namespace

dev_camera make_dev_camera(const camera& c) {
    dev_camera d;
    d.ox = c.frame.o.x;
    d.oy = c.frame.o.y;
    d.oz = c.frame.o.z;
    d.xx = c.frame.x.x;
    d.xy = c.frame.x.y;
    d.xz = c.frame.x.z;
    vec3f ny = c.frame.y * -1;  // raytrace.cpp:18
    d.yx = ny.x;
    d.yy = ny.y;
    d.yz = ny.z;
    d.zx = c.frame.z.x;
    d.zy = c.frame.z.y;
    d.zz = c.frame.z.z;
    d.h = 2.0f * c.focus * std::tan(c.fovy / 2.0f);  // raytrace.cpp:21 (tanf)
    d.w = d.h * c.aspect;
    d.focus = c.focus;
    return d;
}

device_scene* device_scene_create(const scene& scn, int device) {
    if (!scn.has_bvh) throw std::invalid_argument("scene has no BVH (call build_bvh first)");
    if (scn.cameras.empty()) throw std::runtime_error("scene has no camera");
    // (a scene without instances uploads: its instance BVH is one empty leaf behind an
    // inverted box, which no ray enters -- the reference renders it black)

    // the kernels test an inner node's two children together (records start, start+1),
    // as make_node always builds them (scene.cpp:595-601)
    auto binary = [](const bvh_tree& t) {
        for (auto& n : t.nodes)
            if (!n.isleaf && n.count != 2) return false;
        return !t.nodes.empty();
    };
    if (!binary(scn.bvh)) throw unsupported_error("instance BVH is not binary (unsupported)");
    for (auto& s : scn.shapes)
        if (!binary(s.bvh)) throw unsupported_error("shape BVH of " + s.name + " is not binary (unsupported)");

    // the walks address records with 32-bit offsets (the s_load SGPR offset is an unsigned
    // 32-bit byte offset; the packed any-hit triangles' offset is a signed int): 48 B per
    // primitive slot (sprims), 36 B (aprims), 64 B / 80 B per instance slot (tinst / winst)
    {
        uint64_t nslots = 0;
        for (auto& s : scn.shapes) nslots += s.bvh.leaf_prims.size();
        const uint64_t ninst = scn.bvh.leaf_prims.size();
        if (nslots * 48 >= (1ull << 32) || nslots * 36 >= (1ull << 31))
            throw unsupported_error("scene too large: " + std::to_string(nslots) +
                                    " primitive slots exceed the walks' 32-bit record offsets");
        if (ninst * 16 * (uint64_t)std::max(4, winst_rows) >= (1ull << 32))
            throw unsupported_error("scene too large: " + std::to_string(ninst) +
                                    " instances exceed the walks' 32-bit record offsets");
    }

    auto ds = new device_scene();
    ds->device = device;
    ds->cameras = scn.cameras;
    ds->top_depth = bvh_max_depth(scn.bvh);
    for (auto& s : scn.shapes) ds->shape_depth = std::max(ds->shape_depth, bvh_max_depth(s.bvh));
    if (ds->top_depth + ds->shape_depth > traversal_stack_cap) {
        int td = ds->top_depth, sd = ds->shape_depth;
        delete ds;
        throw unsupported_error("BVH too deep for the kernel stacks (instance " + std::to_string(td) +
                                 " + shape " + std::to_string(sd) + " > " +
                                 std::to_string(traversal_stack_cap) + ")");
    }

    // ---- shapes: nodes, leaf-ordered primitives, elements, vertices ----
    std::vector<f4> snodes, sprims, vpos, vnorm;
    std::vector<f2> vuv;
    std::vector<i4> shapes, elems;
    std::vector<uint32_t> shape_prim_base;
    for (size_t si = 0; si < scn.shapes.size(); si++) {
        const shape& s = scn.shapes[si];
        int kinds = (!s.triangles.empty()) + (!s.lines.empty()) + (!s.points.empty());
        if (kinds > 1)
            throw unsupported_error("shape " + s.name + " mixes primitive types (unsupported)");
        int kind = !s.triangles.empty() ? kind_triangles
                   : !s.lines.empty()   ? kind_lines
                   : !s.points.empty()  ? kind_points
                                        : kind_empty;
        int node_base = (int)snodes.size() / 2;
        int prim_base = (int)sprims.size() / 3;
        int elem_base = (int)elems.size();
        int vert_base = (int)vpos.size();
        for (auto& n : s.bvh.nodes) {
            // leaves: absolute primitive slot; inner nodes: child index relative to the
            // shape's root (the traversal keeps shape-level stack entries root-relative)
            uint32_t start = n.isleaf ? n.start + prim_base : n.start;
            snodes.push_back(node_lo(n, start));
            snodes.push_back(node_hi(n));
        }
        for (int ei : s.bvh.leaf_prims) {
            if (kind == kind_triangles) {
                vec3i t = s.triangles[ei];
                vec3f v0 = s.pos[t.x], e1 = s.pos[t.y] - v0, e2 = s.pos[t.z] - v0;
                sprims.push_back({v0.x, v0.y, v0.z, as_float(ei)});
                sprims.push_back({e1.x, e1.y, e1.z, 0});
                sprims.push_back({e2.x, e2.y, e2.z, 0});
            } else if (kind == kind_lines) {
                vec2i l = s.lines[ei];
                vec3f v0 = s.pos[l.x], v1 = s.pos[l.y];
                sprims.push_back({v0.x, v0.y, v0.z, as_float(ei)});
                sprims.push_back({v1.x, v1.y, v1.z, s.radius[l.x]});
                sprims.push_back({s.radius[l.y], 0, 0, 0});
            } else {
                int p = s.points[ei];
                vec3f v = s.pos[p];
                sprims.push_back({v.x, v.y, v.z, as_float(ei)});
                sprims.push_back({s.radius[p], 0, 0, 0});
                sprims.push_back({0, 0, 0, 0});
            }
        }
        if (kind == kind_triangles)
            for (auto t : s.triangles) elems.push_back({t.x + vert_base, t.y + vert_base, t.z + vert_base, 0});
        else if (kind == kind_lines)
            for (auto l : s.lines) elems.push_back({l.x + vert_base, l.y + vert_base, -1, 0});
        else if (kind == kind_points)
            for (auto p : s.points) elems.push_back({p + vert_base, -1, -1, 0});
        for (size_t v = 0; v < s.pos.size(); v++) {
            vec3f p = s.pos[v];
            vec3f n = v < s.norm.size() ? s.norm[v] : vec3f{0, 0, 0};
            vec2f t = v < s.texcoord.size() ? s.texcoord[v] : vec2f{0, 0};
            vpos.push_back({p.x, p.y, p.z, 0});
            vnorm.push_back({n.x, n.y, n.z, 0});
            vuv.push_back({t.x, t.y});
        }
        shapes.push_back({node_base, kind, elem_base, vert_base});
        shape_prim_base.push_back((uint32_t)prim_base);
        ds->max_shape_nodes = std::max(ds->max_shape_nodes, s.bvh.nodes.size());
    }

    // ---- 4-wide collapse for the any-hit walk: instance level first, then shapes ----
    // over binned-SAH trees of the reference trees' leaves
    auto any_tree = [](const bvh_tree& t) {
        if (t.nodes.empty()) return t;
        sah_builder sb(t);
        return sb.out;
    };
    std::vector<f4> wnodes;
    wide_builder wb{wnodes};
    // instance-level wide records breadth first (the top levels lead: what LDS staging reads)
    const int wtop_root = wb.emit_bfs(any_tree(scn.bvh), 0, 0);
    const int wtop_depth = wb.max_depth;
    const int wtop_records = (int)wnodes.size() / 8;
    std::vector<int> wshape_root(scn.shapes.size());
    int wshape_depth = 0;
    for (size_t si = 0; si < scn.shapes.size(); si++) {
        wb.max_depth = 0;
        wshape_root[si] =
            scn.shapes[si].bvh.nodes.empty() ? -1 : wb.emit(any_tree(scn.shapes[si].bvh), 0, shape_prim_base[si], 1);
        wshape_depth = std::max(wshape_depth, wb.max_depth);
    }
    // instances of an empty shape enter a wide node with no slots
    const int wempty = (int)wnodes.size() / 8;
    wnodes.resize(wnodes.size() + 8, f4{0, 0, 0, 0});
    for (int a = 0; a < 3; a++) wnodes[(size_t)wempty * 8 + a] = {INFINITY, INFINITY, INFINITY, INFINITY};
    for (int a = 3; a < 6; a++) wnodes[(size_t)wempty * 8 + a] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    {
        const float e = as_float((int)wide_leaf);
        wnodes[(size_t)wempty * 8 + 6] = {e, e, e, e};
    }
    for (auto& r : wshape_root)
        if (r < 0) r = wempty;
    if (wnodes.size() / 8 * wide_record_bytes >= (1u << 30))
        throw unsupported_error("scene too large for the wide any-hit records");
    // the wide walk pushes at most three siblings per visit
    ds->wide_ok = 3 * (wtop_depth + wshape_depth) + 2 <= 64;

    // ---- instance level: nodes + instances permuted into leaf order ----
    std::vector<f4> tnodes, tinst, winst;
    std::vector<std::array<double, 6>> iboxd;  // per instance slot: its world box (lo, hi), no margin
    std::vector<int> tinst_id;
    for (auto& n : scn.bvh.nodes) {
        tnodes.push_back(node_lo(n, n.start));
        tnodes.push_back(node_hi(n));
    }
    // spine records for the closest-hit walk: node X's record followed by those of its
    // child start+1, that child's child start+1, ... (spine_len nodes, 32 bytes each):
    // the nodes the reference tests back to back after X when each one passes
    auto pairs = [](const std::vector<f4>& nodes, size_t first, size_t count, size_t base) {
        std::vector<f4> out;
        out.reserve(count * 2 * spine_len);
        for (size_t x = first; x < first + count; x++) {
            size_t y = x;
            bool live = true;
            for (int j = 0; j < spine_len; j++) {
                if (!live) {
                    out.push_back({0, 0, 0, 0});
                    out.push_back({0, 0, 0, 0});
                    continue;
                }
                f4 lo = nodes[2 * y];
                const f4 hi = nodes[2 * y + 1];
                uint32_t cl, start;
                memcpy(&cl, &hi.w, 4);
                memcpy(&start, &lo.w, 4);
                if (!(cl & leaf_bit)) {
                    // an inner node's child: the byte offset of its spine record (from the
                    // level's first record), the walks' load offset as is
                    const uint64_t off = (uint64_t)start * spine_record_bytes;
                    if (off >= (1ull << 31)) throw unsupported_error("scene too large for the spine records");
                    lo.w = as_float((int)off);
                }
                out.push_back(lo);
                out.push_back(hi);
                if (cl & leaf_bit)
                    live = false;
                else
                    y = base + start + 1;
            }
        }
        return out;
    };
    // The instance level's records are renumbered breadth first, sibling pairs kept
    // adjacent (the walks find child start+1's record right after start's): the top levels
    // of the tree lead the array, so k_primary_persist can stage its first records in LDS
    // (YRT_PRIMARY_LDS_RECORDS). Only the record numbering changes; the tree, and so the
    // walk's order of tests, is the reference's.
    std::vector<f4> tpair;
    std::vector<int> tcut;
    {
        const size_t nn = tnodes.size() / 2;
        std::vector<uint32_t> bfs(nn, 0), order;  // old index -> breadth-first index, and back
        order.reserve(nn);
        if (nn) order.push_back(0);
        for (size_t q = 0; q < order.size(); q++) {
            uint32_t cl, start;
            memcpy(&cl, &tnodes[2 * order[q] + 1].w, 4);
            memcpy(&start, &tnodes[2 * order[q]].w, 4);
            if (cl & leaf_bit) continue;
            if ((size_t)start + 1 >= nn) throw std::runtime_error("instance BVH child out of range");
            bfs[start] = (uint32_t)order.size(), order.push_back(start);
            bfs[start + 1] = (uint32_t)order.size(), order.push_back(start + 1);
        }
        if (order.size() != nn) throw std::runtime_error("instance BVH has unreachable nodes");
        std::vector<f4> renum(tnodes.size());
        for (size_t n = 0; n < nn; n++) {
            f4 lo = tnodes[2 * order[n]];
            const f4 hi = tnodes[2 * order[n] + 1];
            uint32_t cl, start;
            memcpy(&cl, &hi.w, 4);
            memcpy(&start, &lo.w, 4);
            if (!(cl & leaf_bit)) lo.w = as_float((int)bfs[start]);
            renum[2 * n] = lo, renum[2 * n + 1] = hi;
        }
        tpair = pairs(renum, 0, nn, 0);
        // the camera lists' starting frontier (wavefront.hip k_camera_lists): the nodes of the
        // tree's top cut_depth levels' cut -- every node at depth cut_depth, and every leaf above
        // it -- in the reference's DFS order (child start+1 before start, scene.cpp:446-479), as
        // byte offsets of their records in trel; at most 2^cut_depth entries
        std::vector<std::pair<uint32_t, int>> st;  // (node, depth)
        if (nn) st.push_back({0u, 0});
        while (!st.empty()) {
            const auto [n, d] = st.back();
            st.pop_back();
            uint32_t cl, start;
            memcpy(&cl, &renum[2 * n + 1].w, 4);
            memcpy(&start, &renum[2 * n].w, 4);
            if ((cl & leaf_bit) || d == camera_cut_depth) {
                tcut.push_back((int)(n * (uint32_t)spine_record_bytes));
                continue;
            }
            st.push_back({start, d + 1});      // visited second
            st.push_back({start + 1, d + 1});  // visited first, as the reference does
        }
    }
    std::vector<f4> spair;
    for (size_t si = 0; si < scn.shapes.size(); si++) {
        const size_t nb = (size_t)shapes[si].x, nn = scn.shapes[si].bvh.nodes.size();
        std::vector<f4> p = pairs(snodes, nb, nn, nb);
        spair.insert(spair.end(), p.begin(), p.end());
    }
    if (scn.materials.size() > (size_t)mat_index_mask + 1)
        throw unsupported_error("scene too large (materials > 2^24, unsupported)");
    // each material's shadow class (yrt_device.h mat_class_shift; wavefront.hip light_term_zero)
    std::vector<uint32_t> mat_class(scn.materials.size(), 0);
    for (size_t k = 0; k < scn.materials.size(); k++) {
        const material& m = scn.materials[k];
        const float rs = m.rs;
        const float ns = (rs) ? 2 / std::pow(rs, 4.0f) - 2 : 1e6f;  // raytrace.cpp:144, as in mats below
        const float lim = 1048576.0f;                                 // 2^20
        auto small = [&](vec3f c) { return std::fabs(c.x) <= lim && std::fabs(c.y) <= lim && std::fabs(c.z) <= lim; };
        if (!small(m.kd) || !small(m.ks)) continue;  // (NaN fails too)
        if (m.ks.x == 0.0f && m.ks.y == 0.0f && m.ks.z == 0.0f) {
            if (ns >= 0.0f && ns <= 3.402823466e+38f) mat_class[k] = 1;
        } else {
            for (int c = mat_class_max; c >= 2; c--)
                if (ns >= mat_class_ns(c)) {
                    mat_class[k] = (uint32_t)c;
                    break;
                }
        }
    }
    for (int ii : scn.bvh.leaf_prims) {
        const instance& ist = scn.instances[ii];
        if (ist.mat < 0 || ist.mat >= (int)scn.materials.size())
            throw std::runtime_error("instance " + ist.name + " has no material");
        const frame3f& f = ist.frame;
        // the frame's rotation rows bitwise equal to the identity's: the instance-local
        // direction is then the same for every such instance (the walks compute it once)
        auto bits = [](float v) {
            uint32_t u;
            memcpy(&u, &v, 4);
            return u;
        };
        const bool ident = bits(f.x.x) == 0x3f800000u && bits(f.x.y) == 0 && bits(f.x.z) == 0 && bits(f.y.x) == 0 &&
                           bits(f.y.y) == 0x3f800000u && bits(f.y.z) == 0 && bits(f.z.x) == 0 && bits(f.z.y) == 0 &&
                           bits(f.z.z) == 0x3f800000u;
        if (ist.shp >= (1 << 30)) throw unsupported_error("scene too large (shapes >= 2^30, unsupported)");
        // .w: the shape index | identity rotation << 30
        tinst.push_back({f.x.x, f.x.y, f.x.z, as_float((int)((uint32_t)ist.shp | (ident ? inst_identity_bit : 0u)))});
        // .w: the shape's wide root (record byte offset) | kind << 30 (the any-hit walk's entry)
        const uint32_t wr = (uint32_t)wshape_root[ist.shp] * (uint32_t)wide_record_bytes;
        tinst.push_back({f.y.x, f.y.y, f.y.z, as_float((int)(wr | ((uint32_t)shapes[ist.shp].y << 30)))});
        tinst_id.push_back(ii);
        tinst.push_back({f.z.x, f.z.y, f.z.z, as_float((int)((uint32_t)ist.mat | mat_class[ist.mat] << mat_class_shift))});
        // .w of the last row: the shape's root node and primitive kind, so a traversal
        // entering the instance needs no dependent fetch of the shape record
        const i4 sh = shapes[ist.shp];
        if (sh.x >= (1 << 30)) throw unsupported_error("scene too large (shape nodes >= 2^30, unsupported)");
        tinst.push_back({f.o.x, f.o.y, f.o.z, as_float((int)((uint32_t)sh.x | ((uint32_t)sh.y << 30)))});
        // any-hit copy with the shape's root box (an empty shape: a box no finite ray passes)
        const shape& sp = scn.shapes[ist.shp];
        bbox3f rb = {{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
        if (!sp.bvh.nodes.empty()) rb = sp.bvh.nodes[0].bbox;
        static_assert(winst_rows == 5, "winst layout (yrt_device.h)");
        const f4* t = &tinst[tinst.size() - 4];
        winst.push_back(t[0]);
        winst.push_back(t[1]);
        winst.push_back({t[2].x, t[2].y, t[2].z, rb.min.x});
        winst.push_back({t[3].x, t[3].y, t[3].z, rb.min.y});
        winst.push_back({rb.min.z, rb.max.x, rb.max.y, rb.max.z});
        // the instance's world box (dev_scene_view ibox): the points w whose instance-space
        // image transform_point_inverse(f, w) = R^T (w - o) lies in the root box are
        // o + (R^T)^-1 l, so the root box's corners go through (R^T)^-1, in double (the margin
        // is added below, once the scene's extent is known). Only for a frame whose axes are
        // orthonormal to 2^-20: the walks reuse the world tmax as the instance-space tmax
        // along the renormalised local direction, so a scaled frame stretches the segment a
        // ray tests in its space (vmath.h:275-278); those instances keep NaN boxes, which no
        // plane separates
        {
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            const double R[3][3] = {{f.x.x, f.y.x, f.z.x}, {f.x.y, f.y.y, f.z.y}, {f.x.z, f.y.z, f.z.z}};  // columns: axes
            bool ortho = true;
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    double g = 0.0;  // (R^T R)_ij
                    for (int k = 0; k < 3; k++) g += R[k][i] * R[k][j];
                    ortho = ortho && std::fabs(g - (i == j ? 1.0 : 0.0)) <= std::ldexp(1.0, -20);
                }
            const double det = R[0][0] * (R[1][1] * R[2][2] - R[1][2] * R[2][1]) -
                               R[0][1] * (R[1][0] * R[2][2] - R[1][2] * R[2][0]) +
                               R[0][2] * (R[1][0] * R[2][1] - R[1][1] * R[2][0]);
            double Mi[3][3];  // (R^T)^-1 = the cofactor matrix of R over det(R)
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
                    Mi[i][j] = (R[i1][j1] * R[i2][j2] - R[i1][j2] * R[i2][j1]) / det;
                }
            const bool empty = !(rb.min.x <= rb.max.x && rb.min.y <= rb.max.y && rb.min.z <= rb.max.z);
            const bool nan = std::isnan(rb.min.x) || std::isnan(rb.min.y) || std::isnan(rb.min.z) ||
                             std::isnan(rb.max.x) || std::isnan(rb.max.y) || std::isnan(rb.max.z) || !ortho ||
                             !std::isfinite(det) || !std::isfinite(f.o.x) || !std::isfinite(f.o.y) ||
                             !std::isfinite(f.o.z);
            if (nan) {
                for (int a = 0; a < 3; a++) lo[a] = hi[a] = NAN;
            } else if (!empty) {
                const double o[3] = {f.o.x, f.o.y, f.o.z};
                for (int c = 0; c < 8; c++) {
                    const double l[3] = {(c & 1) ? rb.max.x : rb.min.x, (c & 2) ? rb.max.y : rb.min.y,
                                         (c & 4) ? rb.max.z : rb.min.z};
                    for (int a = 0; a < 3; a++) {
                        const double w = o[a] + Mi[a][0] * l[0] + Mi[a][1] * l[1] + Mi[a][2] * l[2];
                        lo[a] = std::min(lo[a], w), hi[a] = std::max(hi[a], w);
                    }
                }
            }
            iboxd.push_back({lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
        }
    }
    // the world boxes' margin: 2^-14 of four times the scene's extent (a bound on the list
    // builders' points: hit points, lights and the camera of a usual view), ~1000x the
    // rounding of an instance transform and slab test at that scale; the builders' own
    // cone / hull margins (1e-3 + 3e-5 of their coordinates) come on top
    std::vector<f4> ibox;
    {
        double M = 0.0;
        for (auto& b : iboxd)
            for (double c : b)
                if (std::isfinite(c)) M = std::max(M, std::fabs(c));
        const double eps = (4.0 * M + 1.0) * std::ldexp(1.0, -14);
        auto down = [](double x) {
            float v = (float)x;
            if ((double)v > x) v = std::nextafter(v, -INFINITY);
            return v;
        };
        auto up = [](double x) {
            float v = (float)x;
            if ((double)v < x) v = std::nextafter(v, INFINITY);
            return v;
        };
        for (auto& b : iboxd) {
            f4 lo = {down(b[0] - eps), down(b[1] - eps), down(b[2] - eps), 0.0f};
            f4 hi = {up(b[3] + eps), up(b[4] + eps), up(b[5] + eps), 0.0f};
            for (int a = 0; a < 6; a++)
                if (std::isnan(b[a])) lo = {NAN, NAN, NAN, 0.0f}, hi = {NAN, NAN, NAN, 0.0f};
            ibox.push_back(lo);
            ibox.push_back(hi);
        }
    }

    // ---- materials, lights, textures ----
    std::vector<f4> mats, lights;
    for (auto& m : scn.materials) {
        float rs = m.rs;
        float ns = (rs) ? 2 / std::pow(rs, 4.0f) - 2 : 1e6f;  // raytrace.cpp:144
        int flags = (m.kr.x > 0.0f || m.kr.y > 0.0f || m.kr.z > 0.0f) ? mat_reflective : 0;
        if (flags & mat_reflective) ds->reflective = true;
        for (int t : {m.kd_txt, m.ks_txt}) {
            if (t >= (int)scn.textures.size() || (t >= 0 && scn.textures[t].pixels.empty()))
                throw std::runtime_error("material " + m.name + " references a missing texture");
        }
        mats.push_back({m.kd.x, m.kd.y, m.kd.z, ns});
        mats.push_back({m.ks.x, m.ks.y, m.ks.z, as_float(m.kd_txt)});
        mats.push_back({m.kr.x, m.kr.y, m.kr.z, as_float(m.ks_txt)});
        mats.push_back({m.ke.x, m.ke.y, m.ke.z, as_float(flags)});
    }
    for (auto& ist : scn.instances) {
        if (ist.mat < 0) continue;
        vec3f ke = scn.materials[ist.mat].ke;
        if (!(ke.x > 0.0f && ke.y > 0.0f && ke.z > 0.0f)) continue;
        const shape& s = scn.shapes[ist.shp];
        if (s.pos.empty()) throw std::runtime_error("light " + ist.name + " has no vertex");
        const frame3f& f = ist.frame;
        vec3f p0 = s.pos.front();
        lights.push_back({f.x.x, f.x.y, f.x.z, 0});
        lights.push_back({f.y.x, f.y.y, f.y.z, 0});
        lights.push_back({f.z.x, f.z.y, f.z.z, 0});
        lights.push_back({f.o.x, f.o.y, f.o.z, 0});
        lights.push_back({p0.x, p0.y, p0.z, 0});
        lights.push_back({ke.x, ke.y, ke.z, 0});
    }
    std::vector<uint32_t> texels;
    std::vector<i4> texinfo;
    for (auto& t : scn.textures) {
        texinfo.push_back({(int)texels.size(), t.width, t.height, 0});
        for (auto& p : t.pixels)
            texels.push_back((uint32_t)p.x | (uint32_t)p.y << 8 | (uint32_t)p.z << 16 | (uint32_t)p.w << 24);
    }
    std::vector<float> srgb(256);
    for (int c = 0; c < 256; c++) {
        float r = (float)(unsigned char)c;
        srgb[c] = std::fmin(1.0f, std::pow(r / 255.0f, 2.2f));  // raytrace.cpp:51
    }

    // ---- upload ----
    arena_builder ab;
    size_t o_tnodes = ab.add(tnodes.data(), tnodes.size() * sizeof(f4));
    size_t o_tinst = ab.add(tinst.data(), tinst.size() * sizeof(f4));
    size_t o_snodes = ab.add(snodes.data(), snodes.size() * sizeof(f4));
    size_t o_sprims = ab.add(sprims.data(), sprims.size() * sizeof(f4));
    // the any-hit walk's triangles: v0, e1, e2 of every sprims slot as 9 packed floats
    // (one s_load_dwordx8 + s_load_dword, 9 SGPRs instead of 12; other kinds: zeros)
    std::vector<float> aprims(9 * (sprims.size() / 3), 0.0f);
    for (size_t i = 0; i < sprims.size() / 3; i++) {
        const f4* r = &sprims[3 * i];
        const float v[9] = {r[0].x, r[0].y, r[0].z, r[1].x, r[1].y, r[1].z, r[2].x, r[2].y, r[2].z};
        for (int q = 0; q < 9; q++) aprims[9 * i + q] = v[q];
    }
    size_t o_aprims = ab.add(aprims.data(), aprims.size() * sizeof(float));
    size_t o_shapes = ab.add(shapes.data(), shapes.size() * sizeof(i4));
    size_t o_elems = ab.add(elems.data(), elems.size() * sizeof(i4));
    size_t o_vpos = ab.add(vpos.data(), vpos.size() * sizeof(f4));
    size_t o_vnorm = ab.add(vnorm.data(), vnorm.size() * sizeof(f4));
    size_t o_vuv = ab.add(vuv.data(), vuv.size() * sizeof(f2));
    size_t o_mats = ab.add(mats.data(), mats.size() * sizeof(f4));
    size_t o_lights = ab.add(lights.data(), lights.size() * sizeof(f4));
    size_t o_texels = ab.add(texels.data(), texels.size() * sizeof(uint32_t));
    size_t o_texinfo = ab.add(texinfo.data(), texinfo.size() * sizeof(i4));
    size_t o_srgb = ab.add(srgb.data(), srgb.size() * sizeof(float));
    size_t o_wnodes = ab.add(wnodes.data(), wnodes.size() * sizeof(f4));
    size_t o_winst = ab.add(winst.data(), winst.size() * sizeof(f4));
    size_t o_tpair = ab.add(tpair.data(), tpair.size() * sizeof(f4));
    size_t o_trel = ab.add(tpair.data(), tpair.size() * sizeof(f4));  // rewritten per render
    size_t o_spair = ab.add(spair.data(), spair.size() * sizeof(f4));
    size_t o_tinst_id = ab.add(tinst_id.data(), tinst_id.size() * sizeof(int));
    size_t o_ibox = ab.add(ibox.data(), ibox.size() * sizeof(f4));
    size_t o_tcut = ab.add(tcut.data(), tcut.size() * sizeof(int));

    try {
        check(hipSetDevice(device), "hipSetDevice");
        check(hipMalloc(&ds->arena, ab.total), "hipMalloc(scene arena)");
        {
            int ncu = 0;
            if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
                ds->num_cus = (ncu + 7) / 8 * 8;  // the persistent grids are dealt over 8 XCDs
        }
        ds->arena_bytes = ab.total;
        for (auto& s : ab.sections)
            if (s.bytes)
                check(hipMemcpy((char*)ds->arena + s.offset, s.src, s.bytes, hipMemcpyHostToDevice),
                      "hipMemcpy(scene)");
        // the copies ran on the null stream; a caller's non-blocking stream is not ordered
        // after them, so the upload completes here
        check(hipDeviceSynchronize(), "hipDeviceSynchronize(scene upload)");
    } catch (...) {
        device_scene_destroy(ds);
        throw;
    }
    char* base = (char*)ds->arena;
    dev_scene_view& v = ds->view;
    v.tnodes = (const f4*)(base + o_tnodes);
    v.tinst = (const f4*)(base + o_tinst);
    v.snodes = (const f4*)(base + o_snodes);
    v.sprims = (const f4*)(base + o_sprims);
    v.aprims = (const float*)(base + o_aprims);
    v.shapes = (const i4*)(base + o_shapes);
    v.elems = (const i4*)(base + o_elems);
    v.vpos = (const f4*)(base + o_vpos);
    v.vnorm = (const f4*)(base + o_vnorm);
    v.vuv = (const f2*)(base + o_vuv);
    v.mats = (const f4*)(base + o_mats);
    v.lights = (const f4*)(base + o_lights);
    v.texels = (const uint32_t*)(base + o_texels);
    v.texinfo = (const i4*)(base + o_texinfo);
    v.srgb = (const float*)(base + o_srgb);
    v.wnodes = (const f4*)(base + o_wnodes);
    v.winst = (const f4*)(base + o_winst);
    v.tpair = (const f4*)(base + o_tpair);
    ds->trel = (f4*)(base + o_trel);
    v.spair = (const f4*)(base + o_spair);
    v.tinst_id = (const int*)(base + o_tinst_id);
    v.ibox = ibox.empty() ? nullptr : (const f4*)(base + o_ibox);
    v.tcut = (const int*)(base + o_tcut);
    v.ntcut = (int)tcut.size();
    v.inst_masks = !ibox.empty() && tinst.size() / 4 < ((size_t)1 << 21) ? 1 : 0;
    v.wtop_root = wtop_root * wide_record_bytes;
    v.nwtop = wtop_records;
    v.wide = ds->wide_ok ? 1 : 0;
    v.nlights = (int)lights.size() / 6;
    v.ntextures = (int)texinfo.size();
    ds->nlights = v.nlights;
    v.ntnodes = (int)tnodes.size() / 2;
    ds->ntnodes = tnodes.size() / 2;
    ds->narrow_stack = ds->ntnodes < 65536 && ds->max_shape_nodes < 65536;
    ds->nsnodes = snodes.size() / 2;
    ds->nsprims = sprims.size() / 3;
    ds->ninst = tinst.size() / 4;
#ifdef YRT_DEBUG_BOUNDS
    v.nsnodes = (int)ds->nsnodes;
    v.nsprims = (int)ds->nsprims;
    v.ninst = (int)ds->ninst;
    v.nwnodes = (int)wnodes.size() / 8;
#endif
    return ds;
}

int phase_timer::begin(int phase, hipStream_t s) {
    if (!on) return -1;
    if (used >= phase_of.size()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess) return -1;
        if (hipEventCreate(&b) != hipSuccess) {
            (void)hipEventDestroy(a);
            return -1;
        }
        pool.push_back(a);
        pool.push_back(b);
        phase_of.push_back(0);
    }
    int idx = (int)used++;
    phase_of[idx] = phase;
    (void)hipEventRecord(pool[2 * idx], s);
    return idx;
}

void phase_timer::end(int idx, hipStream_t s) {
    if (idx >= 0) (void)hipEventRecord(pool[2 * idx + 1], s);
}

void phase_timer::collect(float* ms, int* launches) {
    for (int p = 0; p < phase_count; p++) {
        ms[p] = 0;
        launches[p] = 0;
    }
    for (size_t i = 0; i < used; i++) {
        float t = 0;
        (void)hipEventSynchronize(pool[2 * i + 1]);
        if (hipEventElapsedTime(&t, pool[2 * i], pool[2 * i + 1]) == hipSuccess) ms[phase_of[i]] += t;
        launches[phase_of[i]]++;
    }
}

void phase_timer::destroy() {
    for (auto e : pool) (void)hipEventDestroy(e);
    pool.clear();
    phase_of.clear();
    used = 0;
}

void device_scene_destroy(device_scene* ds) {
    if (!ds) return;
    (void)hipSetDevice(ds->device);
    ds->timer.destroy();
    if (ds->arena) (void)hipFree(ds->arena);
    if (ds->work) (void)hipFree(ds->work);
    if (ds->level_count_ev) (void)hipEventDestroy(ds->level_count_ev);
    if (ds->level_count_host) (void)hipHostFree(ds->level_count_host);
    if (ds->list_stats_ev) (void)hipEventDestroy(ds->list_stats_ev);
    if (ds->list_stats_host) (void)hipHostFree(ds->list_stats_host);
    delete ds;
}

}  // namespace yrt
