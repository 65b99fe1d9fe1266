// bvh_build.cpp -- host BVH builder restating build_bvh (src/scene.cpp:509-658).
//
// The kernels replay the reference's traversal order, so the node topology,
// numbering and leaf primitive order must be identical to the reference's:
//   * primitive bounds: points, then lines, then triangles, each with its own
//     element index (scene.cpp:525-550); radius-padded for points/lines
//   * instance bounds: bbox_to_world(frame, shape root bbox) (scene.cpp:554-565)
//   * make_node: bbox union; split only when > 4 prims; children allocated as a
//     consecutive pair at the end of the node array, left subtree first
//     (scene.cpp:572-603)
//   * split_prims: largest centroid extent (ties x, then y), midpoint of the
//     centroid box, in-place two-sided (Hoare) partition with the same swap
//     sequence as std::partition on a bidirectional range (scene.cpp:607-639);
//     equal_num uses an nth_element median (not used by raytrace, main() passes false)
// tests/test_library.py::test_bvh_matches_reference compares the serialised nodes with the reference's byte-for-byte.
#include <algorithm>
#include <stdexcept>

#include "yrt_scene.h"

namespace yrt {
namespace {

struct bound_prim {
    bbox3f bbox;
    vec3f center;
    int pid;
};

bbox3f padded(const bbox3f& b, vec3f p, float r) {
    return expand_bbox(b, bbox3f{p - vec3f{r, r, r}, p + vec3f{r, r, r}});
}

float axis_of(vec3f v, int a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; }

bool split_prims(std::vector<bound_prim>& prims, int start, int end, bool equal_num, int& axis,
                 int& mid) {
    bbox3f cb = invalid_bbox3f;
    for (int i = start; i < end; i++) cb = expand_bbox(cb, prims[i].center);
    vec3f size = cb.max - cb.min;
    if (size == vec3f{0, 0, 0}) return false;
    if (size.x >= size.y && size.x >= size.z)
        axis = 0;
    else if (size.y >= size.x && size.y >= size.z)
        axis = 1;
    else
        axis = 2;
    if (equal_num) {
        mid = (start + end) / 2;
        int a = axis;
        std::nth_element(prims.begin() + start, prims.begin() + mid, prims.begin() + end,
                         [a](const bound_prim& x, const bound_prim& y) {
                             return axis_of(x.center, a) < axis_of(y.center, a);
                         });
        return true;
    }
    float half = axis_of((cb.min + cb.max) / 2, axis);
    auto pred = [&](int i) { return axis_of(prims[i].center, axis) < half; };
    // two-sided partition: advance from the front past elements that belong left,
    // retreat from the back past elements that belong right, swap, repeat
    int first = start, last = end;
    for (;;) {
        while (first != last && pred(first)) first++;
        if (first == last) break;
        last--;
        while (first != last && !pred(last)) last--;
        if (first == last) break;
        std::swap(prims[first], prims[last]);
        first++;
    }
    mid = first;
    return true;
}

void make_node(bvh_tree& bvh, int nid, std::vector<bound_prim>& prims, int start, int end,
               bool equal_num, int depth) {
    if (depth > 4096) throw std::runtime_error("bvh build: degenerate split recursion");
    bbox3f b = invalid_bbox3f;
    for (int i = start; i < end; i++) b = expand_bbox(b, prims[i].bbox);
    bool split = false;
    int axis = -1, mid = -1;
    if (end - start > 4) split = split_prims(prims, start, end, equal_num, axis, mid);
    if (split && (mid <= start || mid >= end)) {
        // the reference recurses forever here (assert compiled out, scene.cpp:592);
        // surface it as an error instead of a stack overflow
        throw std::runtime_error("bvh build: empty midpoint split (degenerate centroids)");
    }
    bvh.nodes[nid].bbox = b;
    if (!split) {
        bvh.nodes[nid].isleaf = 1;
        bvh.nodes[nid].start = (uint32_t)start;
        bvh.nodes[nid].count = (uint16_t)(end - start);
    } else {
        int first = (int)bvh.nodes.size();
        bvh.nodes[nid].isleaf = 0;
        bvh.nodes[nid].axis = (uint8_t)axis;
        bvh.nodes[nid].start = (uint32_t)first;
        bvh.nodes[nid].count = 2;
        bvh.nodes.push_back({});
        bvh.nodes.push_back({});
        make_node(bvh, first, prims, start, mid, equal_num, depth + 1);
        make_node(bvh, first + 1, prims, mid, end, equal_num, depth + 1);
    }
}

bvh_tree build_tree(std::vector<bound_prim>& prims, bool equal_num) {
    bvh_tree bvh;
    bvh.nodes.reserve(prims.size() * 2);
    bvh.nodes.push_back({});
    make_node(bvh, 0, prims, 0, (int)prims.size(), equal_num, 0);
    bvh.nodes.shrink_to_fit();
    bvh.leaf_prims.resize(prims.size());
    for (size_t i = 0; i < prims.size(); i++) bvh.leaf_prims[i] = prims[i].pid;
    return bvh;
}

void build_shape_bvh(shape& s, bool equal_num) {
    std::vector<bound_prim> prims;
    for (int ei = 0; ei < (int)s.points.size(); ei++) {
        int e = s.points[ei];
        bbox3f b = padded(invalid_bbox3f, s.pos[e], s.radius[e]);
        prims.push_back({b, (b.min + b.max) / 2.0f, ei});
    }
    for (int ei = 0; ei < (int)s.lines.size(); ei++) {
        vec2i e = s.lines[ei];
        bbox3f b = padded(invalid_bbox3f, s.pos[e.x], s.radius[e.x]);
        b = padded(b, s.pos[e.y], s.radius[e.y]);
        prims.push_back({b, (b.min + b.max) / 2.0f, ei});
    }
    for (int ei = 0; ei < (int)s.triangles.size(); ei++) {
        vec3i e = s.triangles[ei];
        bbox3f b = padded(invalid_bbox3f, s.pos[e.x], 0);
        b = padded(b, s.pos[e.y], 0);
        b = padded(b, s.pos[e.z], 0);
        prims.push_back({b, (b.min + b.max) / 2.0f, ei});
    }
    s.bvh = build_tree(prims, equal_num);
}

}  // namespace

void build_bvh(scene& scn, bool equal_num) {
    for (auto& s : scn.shapes) {
        if (!s.points.empty() && s.radius.size() < s.pos.size())
            throw std::runtime_error("shape " + s.name + ": points without radius");
        if (!s.lines.empty() && s.radius.size() < s.pos.size())
            throw std::runtime_error("shape " + s.name + ": lines without radius");
        build_shape_bvh(s, equal_num);
    }
    std::vector<bound_prim> prims;
    for (int ii = 0; ii < (int)scn.instances.size(); ii++) {
        const auto& ist = scn.instances[ii];
        bbox3f b = bbox_to_world(ist.frame, scn.shapes[ist.shp].bvh.nodes[0].bbox);
        prims.push_back({b, (b.min + b.max) / 2.0f, ii});
    }
    scn.bvh = build_tree(prims, equal_num);
    scn.has_bvh = true;
}

int bvh_max_depth(const bvh_tree& bvh) {
    if (bvh.nodes.empty()) return 0;
    int best = 0;
    std::vector<std::pair<int, int>> st = {{0, 1}};
    while (!st.empty()) {
        auto [n, d] = st.back();
        st.pop_back();
        best = std::max(best, d);
        const auto& node = bvh.nodes[n];
        if (!node.isleaf)
            for (int c = 0; c < node.count; c++) st.push_back({(int)node.start + c, d + 1});
    }
    return best;
}

}  // namespace yrt
