// bvh_gpu.hip -- build_bvh (src/scene.cpp:509-658) with the tree construction on the
// GPU, producing the reference's nodes byte for byte (bvh_build.cpp is the host twin).
//
// The O(N log N) part -- per node: the union of its primitives' boxes, the centroid box,
// the split axis and midpoint, and the in-place partition -- runs level by level on the
// device, one workgroup per node of the level. The O(N) parts stay on the host: the
// primitive and instance bounds (the same yrt_math.h code as the host builder) and the
// final node numbering.
//
// Exactness:
//  * boxes: the reference folds expand_bbox over a node's primitives in order, with ?:
//    selects (smin(a, b) = a < b ? a : b): among equal minima the LAST one wins (so a
//    -0/+0 tie is order dependent) and a NaN sticks only until a later element replaces
//    it. A thread folds a contiguous run in order and the workgroup combines the runs in
//    index order with the fold's own composition law: a run is summarised by (w, has_nan)
//    -- w the value the run leaves when it starts from any acc, unless acc < w and the run
//    holds no NaN -- which composes associatively, so the result is the sequential fold's
//    bit for bit, signed zeros and NaNs included.
//  * partition: split_prims' two-sided (Hoare) partition swaps the k-th element from the
//    left that belongs right with the k-th element from the right that belongs left, for
//    every k, and moves nothing else; the workgroup ranks both kinds with prefix counts
//    and performs exactly those swaps.
//  * numbering: make_node allocates a child pair when it splits a node, then builds the
//    left subtree, then the right one: the pair of the i-th split node in that pre-order
//    is nodes 2i+1, 2i+2. The host computes the pre-order ranks from the level lists.
//  equal_num (nth_element, never used by raytrace: main() passes false) is not supported.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "yrt_scene.h"

namespace yrt {
namespace {

struct bprim {  // bound_prim (scene.cpp:500-505)
    float bmin[3], bmax[3], c[3];
    int pid;
};

struct seg {        // one node of the current level
    int start, end; // its primitives
    int parent;     // index of the parent in the previous level's node list, -1 for a root
    int side;       // 0: the parent's left child (start), 1: right (start + 1)
};

struct node_out {
    float bmin[3], bmax[3];
    int start, end, mid;  // mid: the split (inner nodes)
    int axis;             // -1: leaf
};

// a run of the min fold (w, has_nan); max is the same with >
struct run {
    float w;
    int nan;
};
template <bool MAX>
__device__ __forceinline__ bool before(float a, float b) {
    return MAX ? a > b : a < b;
}
template <bool MAX>
__device__ __forceinline__ run combine(run l, run r) {
    if (r.nan) return r;
    return {before<MAX>(l.w, r.w) ? l.w : r.w, l.nan};
}
template <bool MAX>
__device__ __forceinline__ float apply(float acc, run s) {
    return s.nan ? s.w : (before<MAX>(acc, s.w) ? acc : s.w);
}

constexpr int WG = 256;

// in-order reduction of six runs (min.xyz, max.xyz) over [b, e): each thread folds a
// contiguous piece, the pieces are combined in thread order
template <bool CENTER>
__device__ void box_of(const bprim* P, int b, int e, float out_min[3], float out_max[3], run (&sh)[6][WG]) {
    const int n = e - b, t = threadIdx.x;
    const int per = (n + WG - 1) / WG;
    const int lo = b + t * per, hi = min(e, lo + per);
    run r[6];
    for (int a = 0; a < 6; a++) r[a] = {__builtin_nanf(""), 0};
    bool any = false;
    for (int i = lo; i < hi; i++) {
        for (int a = 0; a < 3; a++) {
            const float vmn = CENTER ? P[i].c[a] : P[i].bmin[a];
            const float vmx = CENTER ? P[i].c[a] : P[i].bmax[a];
            const run xn = {vmn, vmn != vmn}, xx = {vmx, vmx != vmx};
            r[a] = any ? combine<false>(r[a], xn) : xn;
            r[3 + a] = any ? combine<true>(r[3 + a], xx) : xx;
        }
        any = true;
    }
    // an empty piece is the identity: mark it so the combine below skips it
    for (int a = 0; a < 6; a++) sh[a][t] = any ? r[a] : run{0.0f, -1};
    __syncthreads();
    for (int stride = 1; stride < WG; stride *= 2) {
        if ((t % (2 * stride)) == 0 && t + stride < WG) {
            for (int a = 0; a < 6; a++) {
                const run l = sh[a][t], rr = sh[a][t + stride];
                if (rr.nan < 0) continue;
                if (l.nan < 0) {
                    sh[a][t] = rr;
                    continue;
                }
                sh[a][t] = a < 3 ? combine<false>(l, rr) : combine<true>(l, rr);
            }
        }
        __syncthreads();
    }
    // the reference folds from invalid_bbox3f (vmath.h): min from +flt_max, max from -flt_max
    for (int a = 0; a < 3; a++) {
        out_min[a] = apply<false>(flt_max, sh[a][0]);
        out_max[a] = apply<true>(-flt_max, sh[3 + a][0]);
    }
    __syncthreads();
}

// exclusive prefix count of flags over the workgroup in thread order; returns the total
__device__ int scan_count(int flag, int& before_me, int (&sh)[WG]) {
    const int t = threadIdx.x;
    sh[t] = flag;
    __syncthreads();
    for (int off = 1; off < WG; off *= 2) {
        const int v = t >= off ? sh[t - off] : 0;
        __syncthreads();
        sh[t] += v;
        __syncthreads();
    }
    before_me = sh[t] - flag;
    const int total = sh[WG - 1];
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(WG) void k_split_level(bprim* P, const seg* segs, int nsegs, node_out* out,
                                                    int* left_false, int* right_true, int* err) {
    __shared__ run box_sh[6][WG];
    __shared__ int cnt_sh[WG];
    const int s = blockIdx.x;
    if (s >= nsegs) return;
    const seg g = segs[s];
    const int t = threadIdx.x;
    float bmn[3], bmx[3];
    box_of<false>(P, g.start, g.end, bmn, bmx, box_sh);
    node_out o;
    for (int a = 0; a < 3; a++) o.bmin[a] = bmn[a], o.bmax[a] = bmx[a];
    o.start = g.start, o.end = g.end, o.mid = -1, o.axis = -1;
    const int n = g.end - g.start;
    if (n > 4) {
        float cmn[3], cmx[3];
        box_of<true>(P, g.start, g.end, cmn, cmx, box_sh);
        const float sx = cmx[0] - cmn[0], sy = cmx[1] - cmn[1], sz = cmx[2] - cmn[2];
        if (!(sx == 0 && sy == 0 && sz == 0)) {  // vec3f == {0,0,0} (split_prims)
            const int axis = (sx >= sy && sx >= sz) ? 0 : (sy >= sx && sy >= sz) ? 1 : 2;
            const float half = (cmn[axis] + cmx[axis]) / 2;  // axis_of((min + max) / 2, axis)
            // T = elements that belong left; the partition point is start + T
            int total = 0;
            for (int base = g.start; base < g.end; base += WG) {
                const int i = base + t;
                int dummy;
                total += scan_count(i < g.end && P[i].c[axis] < half, dummy, cnt_sh);
            }
            const int mid = g.start + total;
            // rank the right-belonging elements of [start, mid) from the left and the
            // left-belonging elements of [mid, end) from the right
            int nf = 0, nt = 0;
            for (int base = g.start; base < mid; base += WG) {
                const int i = base + t;
                const int f = (i < mid && !(P[i].c[axis] < half)) ? 1 : 0;
                int k;
                const int c = scan_count(f, k, cnt_sh);
                if (f) left_false[g.start + nf + k] = i;
                nf += c;
            }
            for (int base = g.end - 1; base >= mid; base -= WG) {
                const int i = base - t;
                const int f = (i >= mid && P[i].c[axis] < half) ? 1 : 0;
                int k;
                const int c = scan_count(f, k, cnt_sh);
                if (f) right_true[g.start + nt + k] = i;
                nt += c;
            }
            __syncthreads();
            if (nf != nt) {
                if (t == 0) atomicOr(err, 1);
                return;
            }
            for (int k = t; k < nf; k += WG) {
                const int a = left_false[g.start + k], b = right_true[g.start + k];
                const bprim x = P[a];
                P[a] = P[b];
                P[b] = x;
            }
            if (mid <= g.start || mid >= g.end) {
                if (t == 0) atomicOr(err, 2);  // the reference recurses forever here
                return;
            }
            o.mid = mid, o.axis = axis;
        }
    }
    if (t == 0) out[s] = o;
}

void check(hipError_t e, const char* what) {
    if (e == hipErrorOutOfMemory) throw device_oom(std::string(what) + ": " + hipGetErrorString(e));
    if (e != hipSuccess) throw device_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
struct dbuf {
    T* p = nullptr;
    explicit dbuf(size_t n) { check(hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)), "hipMalloc(bvh build)"); }
    ~dbuf() {
        if (p) (void)hipFree(p);
    }
};

bprim make_prim(const bbox3f& b, int pid) {
    bprim p;
    const vec3f c = (b.min + b.max) / 2.0f;
    p.bmin[0] = b.min.x, p.bmin[1] = b.min.y, p.bmin[2] = b.min.z;
    p.bmax[0] = b.max.x, p.bmax[1] = b.max.y, p.bmax[2] = b.max.z;
    p.c[0] = c.x, p.c[1] = c.y, p.c[2] = c.z;
    p.pid = pid;
    return p;
}

bbox3f padded(const bbox3f& b, vec3f p, float r) {
    return expand_bbox(b, bbox3f{p - vec3f{r, r, r}, p + vec3f{r, r, r}});
}

// build the trees whose primitives are prims[roots[r].start, roots[r].end) together;
// returns one bvh_tree per root (leaf_prims = the partitioned pids)
std::vector<bvh_tree> build_trees(std::vector<bprim>& prims, const std::vector<std::pair<int, int>>& roots,
                                  int device, float* kernel_ms) {
    std::vector<bvh_tree> trees(roots.size());
    const size_t n = prims.size();
    check(hipSetDevice(device), "hipSetDevice");
    dbuf<bprim> d_prims(n);
    dbuf<int> d_lf(n), d_rt(n), d_err(1);
    dbuf<seg> d_segs(n + roots.size());
    dbuf<node_out> d_out(n + roots.size());
    check(hipMemcpy(d_prims.p, prims.data(), n * sizeof(bprim), hipMemcpyHostToDevice), "hipMemcpy");
    check(hipMemset(d_err.p, 0, sizeof(int)), "hipMemset");
    hipEvent_t e0, e1;
    check(hipEventCreate(&e0), "hipEventCreate");
    check(hipEventCreate(&e1), "hipEventCreate");
    check(hipEventRecord(e0, nullptr), "hipEventRecord");
    // level by level; levels[L][i] = the i-th node of level L
    std::vector<std::vector<seg>> lsegs;
    std::vector<std::vector<node_out>> lnodes;
    std::vector<seg> cur;
    for (auto& r : roots) cur.push_back({r.first, r.second, -1, 0});
    std::vector<int> root_of_first(roots.size());
    while (!cur.empty()) {
        check(hipMemcpy(d_segs.p, cur.data(), cur.size() * sizeof(seg), hipMemcpyHostToDevice), "hipMemcpy");
        hipLaunchKernelGGL(k_split_level, dim3((unsigned)cur.size()), dim3(WG), 0, nullptr, d_prims.p, d_segs.p,
                           (int)cur.size(), d_out.p, d_lf.p, d_rt.p, d_err.p);
        check(hipGetLastError(), "k_split_level");
        std::vector<node_out> outs(cur.size());
        check(hipMemcpy(outs.data(), d_out.p, outs.size() * sizeof(node_out), hipMemcpyDeviceToHost), "hipMemcpy");
        int err = 0;
        check(hipMemcpy(&err, d_err.p, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy");
        if (err & 2) throw std::runtime_error("bvh build: empty midpoint split (degenerate centroids)");
        if (err) throw std::runtime_error("bvh build: partition count mismatch");
        std::vector<seg> next;
        for (size_t i = 0; i < cur.size(); i++)
            if (outs[i].axis >= 0) {
                next.push_back({outs[i].start, outs[i].mid, (int)i, 0});
                next.push_back({outs[i].mid, outs[i].end, (int)i, 1});
            }
        lsegs.push_back(std::move(cur));
        lnodes.push_back(std::move(outs));
        cur = std::move(next);
    }
    check(hipEventRecord(e1, nullptr), "hipEventRecord");
    check(hipMemcpy(prims.data(), d_prims.p, n * sizeof(bprim), hipMemcpyDeviceToHost), "hipMemcpy");
    check(hipEventSynchronize(e1), "hipEventSynchronize");
    float ms = 0;
    check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (kernel_ms) *kernel_ms = ms;

    // ---- numbering (host, O(nodes)): pre-order ranks of the split nodes ----
    const int L = (int)lnodes.size();
    std::vector<std::vector<int>> inner(L), rank(L), child(L);  // child: index of the left child in level L+1
    for (int l = 0; l < L; l++) {
        inner[l].assign(lnodes[l].size(), 0);
        rank[l].assign(lnodes[l].size(), 0);
        child[l].assign(lnodes[l].size(), -1);
    }
    for (int l = 1; l < L; l++)
        for (size_t i = 0; i < lsegs[l].size(); i++)
            if (lsegs[l][i].side == 0) child[l - 1][lsegs[l][i].parent] = (int)i;
    for (int l = L - 1; l >= 0; l--)  // split nodes in each subtree
        for (size_t i = 0; i < lnodes[l].size(); i++)
            if (lnodes[l][i].axis >= 0) {
                const int c = child[l][i];
                inner[l][i] = 1 + inner[l + 1][c] + inner[l + 1][c + 1];
            }
    std::vector<int> tree_of(lnodes[0].size());
    for (size_t r = 0; r < lnodes[0].size(); r++) tree_of[r] = (int)r, rank[0][r] = 0;
    std::vector<std::vector<int>> tree(L), index(L);
    tree[0] = tree_of;
    index[0].assign(lnodes[0].size(), 0);
    for (size_t r = 0; r < roots.size(); r++) trees[r].nodes.assign(1 + 2 * (size_t)inner[0][r], bvh_node{});
    for (int l = 0; l < L; l++) {
        if (l + 1 < L) {
            tree[l + 1].assign(lnodes[l + 1].size(), 0);
            index[l + 1].assign(lnodes[l + 1].size(), 0);
        }
        for (size_t i = 0; i < lnodes[l].size(); i++) {
            const node_out& o = lnodes[l][i];
            bvh_node& bn = trees[tree[l][i]].nodes[index[l][i]];
            bn.bbox = {{o.bmin[0], o.bmin[1], o.bmin[2]}, {o.bmax[0], o.bmax[1], o.bmax[2]}};
            const int rootstart = roots[tree[l][i]].first;
            if (o.axis < 0) {
                bn.isleaf = 1;
                bn.start = (uint32_t)(o.start - rootstart);
                bn.count = (uint16_t)(o.end - o.start);
                continue;
            }
            const int c = child[l][i];
            const int first = 1 + 2 * rank[l][i];
            bn.isleaf = 0;
            bn.axis = (uint8_t)o.axis;
            bn.start = (uint32_t)first;
            bn.count = 2;
            // pre-order: the left child right after this node, the right one after the
            // left subtree
            rank[l + 1][c] = rank[l][i] + 1;
            rank[l + 1][c + 1] = rank[l][i] + 1 + inner[l + 1][c];
            tree[l + 1][c] = tree[l + 1][c + 1] = tree[l][i];
            index[l + 1][c] = first;
            index[l + 1][c + 1] = first + 1;
        }
    }
    for (size_t r = 0; r < roots.size(); r++) {
        auto& lp = trees[r].leaf_prims;
        lp.resize(roots[r].second - roots[r].first);
        for (int i = roots[r].first; i < roots[r].second; i++) lp[i - roots[r].first] = prims[i].pid;
    }
    return trees;
}

}  // namespace

void build_bvh_gpu(scene& scn, bool equal_num, int device, float* kernel_ms) {
    if (equal_num) throw unsupported_error("build_bvh on the GPU: equal_num (nth_element splits) is not supported");
    // ---- shapes: the primitive bounds of build_bvh(shape*) (scene.cpp:522-550), then all
    // shape trees in one level-synchronous build ----
    std::vector<bprim> prims;
    std::vector<std::pair<int, int>> roots;
    for (auto& s : scn.shapes) {
        if (!s.points.empty() && s.radius.size() < s.pos.size())
            throw std::runtime_error("shape " + s.name + ": points without radius");
        if (!s.lines.empty() && s.radius.size() < s.pos.size())
            throw std::runtime_error("shape " + s.name + ": lines without radius");
        const int b = (int)prims.size();
        for (int ei = 0; ei < (int)s.points.size(); ei++) {
            const int e = s.points[ei];
            prims.push_back(make_prim(padded(invalid_bbox3f, s.pos[e], s.radius[e]), ei));
        }
        for (int ei = 0; ei < (int)s.lines.size(); ei++) {
            const vec2i e = s.lines[ei];
            bbox3f bb = padded(invalid_bbox3f, s.pos[e.x], s.radius[e.x]);
            prims.push_back(make_prim(padded(bb, s.pos[e.y], s.radius[e.y]), ei));
        }
        for (int ei = 0; ei < (int)s.triangles.size(); ei++) {
            const vec3i e = s.triangles[ei];
            bbox3f bb = padded(invalid_bbox3f, s.pos[e.x], 0);
            bb = padded(bb, s.pos[e.y], 0);
            prims.push_back(make_prim(padded(bb, s.pos[e.z], 0), ei));
        }
        roots.push_back({b, (int)prims.size()});
    }
    // a shape without primitives is one empty leaf (make_node on an empty range)
    std::vector<std::pair<int, int>> built;
    std::vector<size_t> which;
    for (size_t i = 0; i < roots.size(); i++)
        if (roots[i].first < roots[i].second) built.push_back(roots[i]), which.push_back(i);
    float ms_shapes = 0, ms_inst = 0;
    std::vector<bvh_tree> st = built.empty() ? std::vector<bvh_tree>{} : build_trees(prims, built, device, &ms_shapes);
    for (size_t i = 0; i < scn.shapes.size(); i++) {
        bvh_tree empty;
        empty.nodes.assign(1, bvh_node{});
        empty.nodes[0].bbox = invalid_bbox3f;
        empty.nodes[0].isleaf = 1;
        scn.shapes[i].bvh = std::move(empty);
    }
    for (size_t k = 0; k < which.size(); k++) scn.shapes[which[k]].bvh = std::move(st[k]);
    // ---- instances (scene.cpp:554-565) ----
    std::vector<bprim> ip;
    for (int ii = 0; ii < (int)scn.instances.size(); ii++) {
        const auto& ist = scn.instances[ii];
        ip.push_back(make_prim(bbox_to_world(ist.frame, scn.shapes[ist.shp].bvh.nodes[0].bbox), ii));
    }
    if (ip.empty()) {  // no instances: one empty leaf, as make_node on an empty range
        bvh_tree empty;
        empty.nodes.assign(1, bvh_node{});
        empty.nodes[0].bbox = invalid_bbox3f;
        empty.nodes[0].isleaf = 1;
        scn.bvh = std::move(empty);
    } else {
        std::vector<bvh_tree> it = build_trees(ip, {{0, (int)ip.size()}}, device, &ms_inst);
        scn.bvh = std::move(it[0]);
    }
    scn.has_bvh = true;
    if (kernel_ms) *kernel_ms = ms_shapes + ms_inst;
}

}  // namespace yrt
