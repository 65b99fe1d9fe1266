// packet_trace.h -- wave-coherent ("packet") traversal of the reference's two-level
// BVH: the 64 rays of a wave walk the tree together.
//
// Each stack entry is a node plus the mask of lanes that reached it (the lanes
// whose parent box test passed). Popping an entry, every lane of its mask tests
// the node's box with ITS OWN ray and current tmax; the lanes that pass continue
// into the node. The order of the walk is the reference's DFS order (pop; slab
// test; inner node pushes start then start+1, so start+1 is visited first;
// instance leaves enter their instances in slot order; shape leaves test their
// primitives in slot order), so every lane sees exactly the node tests, in exactly
// the order and with exactly the tmax, of intersect_bvh for its ray
// (src/scene.cpp:386-479) -- closest-hit tie-breaking included. Lanes only idle on
// nodes that other lanes of the wave need.
//
// Why on CDNA4: the node index, the node record, the instance frame and the
// primitive record of a step are wave-uniform, so they are scalar loads into SGPRs
// (one request per wave, no per-lane stack, no address VGPRs); the loop control is
// uniform, so there is no exec-mask divergence at all; per-lane state is just the
// ray, the local ray and the hit record. Rays of one wave are 64 samples of one
// pixel (or an 8x8 pixel tile), so the union of their paths is barely larger than
// one path.
//
// Contract: must be called by every lane of the wave in uniform control flow;
// lanes with valid == false take no part (they get no hit).
#pragma once

#include "trace_common.h"

namespace yrt {

// per-wave stack in LDS: entry s = {node, lane mask}
struct wave_stack {
    int* node;
    unsigned long long* mask;
};

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ unsigned long long uniform64(unsigned long long x) {
    unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x);
    unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
    return (unsigned long long)hi << 32 | lo;
}
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }

template <bool ANY, bool COUNT>
__device__ __forceinline__ bool packet_trace(const dev_scene_view& S, ray3 wray, bool valid, hit_record& hr,
                                             wave_stack st, work_counts& wc) {
    const int lane = threadIdx.x & 63;
    const unsigned long long me = 1ull << lane;
    // a NaN tmin/tmax fails every slab test of the reference: such a ray never enters a node
    const unsigned long long live = ballot(valid && !is_nan(wray.tmin) && !is_nan(wray.tmax));
    bool hit = false;
    if (!live) return false;
    const vec3f winvd = {1.0f / wray.d.x, 1.0f / wray.d.y, 1.0f / wray.d.z};
    vec3f lo_o = wray.o, ld = wray.d, linvd = winvd;  // local ray of the current instance
    float ltmax = wray.tmax;
    unsigned long long done = 0;       // any-hit: lanes that already found their hit
    unsigned long long inst_mask = 0;  // lanes entering the current instance leaf
    int level = 0, sp = 0, base = 0, root = 0, kind = 0, inst_next = 0, inst_end = 0, cur_slot = -1;
    int node = 0;
    unsigned long long mask = live;
    for (;;) {
        // ---- every lane of `mask` tests `node` with its own ray ----
        const f4* nb = level ? S.snodes + 2 * (root + node) : S.tnodes + 2 * node;
        const float4 lo = ld4(nb), hi = ld4(nb + 1);
        bool pass;
        if (level)
            pass = !is_nan(ltmax) && box_hit(lo_o, linvd, wray.tmin, ltmax, lo, hi);
        else
            pass = !is_nan(wray.tmax) && box_hit(wray.o, winvd, wray.tmin, wray.tmax, lo, hi);
        if (COUNT && (mask & me)) wc.box++;
        const unsigned long long pm = ballot(pass) & mask;
        bool descend = false;
        if (pm) {
            const int start = uniform(ibits(lo.w));
            const uint32_t cl = (uint32_t)uniform((int)ubits(hi.w));
            const int count = (int)(cl & 0xffffu);
            if (!(cl & leaf_bit)) {
                // push start, continue with start+1 (the reference pops start+1 first)
                if (lane == 0) {
                    st.node[sp] = start;
                    st.mask[sp] = pm;
                }
                sp++;
                node = start + 1;
                mask = pm;
                descend = true;
            } else if (level == 0) {
                inst_next = start;
                inst_end = start + count;
                inst_mask = pm;
                level = 1;
                base = sp;
            } else {
                const bool in = (pm & me) != 0;
                ray3 tr = {lo_o, ld, wray.tmin, ltmax};
                bool leaf_hit = false;
                for (int i = start; i < start + count; i++) {
                    const f4* pr = S.sprims + 3 * i;
                    const float4 a = ld4(pr), b = ld4(pr + 1), c = ld4(pr + 2);
                    if (!in) continue;
                    if (COUNT) wc.prim++;
                    float t;
                    vec4f ew;
                    bool h;
                    if (kind == kind_triangles)
                        h = tri_hit(tr, xyz(a), xyz(b), xyz(c), t, ew);
                    else if (kind == kind_lines)
                        h = line_hit(tr, xyz(a), xyz(b), b.w, c.x, t, ew);
                    else
                        h = point_hit(tr, xyz(a), b.x, t, ew);
                    if (ANY && h) {
                        leaf_hit = true;
                        break;
                    }
                    if (h) {
                        tr.tmax = t;
                        hr.slot = cur_slot;
                        hr.ei = ibits(a.w);
                        hr.ew = ew;
                        hr.dist = t;
                        leaf_hit = true;
                    }
                }
                if (leaf_hit) hit = true;
                if (ANY) {
                    done |= ballot(leaf_hit);
                    if (!(live & ~done)) return hit;
                } else {
                    // the reference sets tray.tmax = dist once the shape returns a hit;
                    // nothing reads the world tmax before that, so updating it here is equivalent
                    ltmax = tr.tmax;
                    if (leaf_hit) wray.tmax = tr.tmax;
                }
            }
        }
        if (descend) continue;
        // ---- next: the next instance of the current leaf, or pop ----
        bool found = false;
        while (!found) {
            if (level == 1 && sp == base) {
                if (inst_next < inst_end) {
                    // enter instance k: transform_ray_inverse (vmath.h:275-278), every lane
                    const int k = inst_next++;
                    const f4* ti = S.tinst + 4 * k;
                    const float4 fx = ld4(ti), fy = ld4(ti + 1), fz = ld4(ti + 2), fo = ld4(ti + 3);
                    const frame3f f = {xyz(fx), xyz(fy), xyz(fz), xyz(fo)};
                    lo_o = transform_point_inverse(f, wray.o);
                    ld = transform_direction_inverse(f, wray.d);
                    linvd = {1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z};
                    ltmax = wray.tmax;
                    const int4 sh = ld4(S.shapes + uniform(ibits(fx.w)));
                    root = uniform(sh.x);
                    kind = uniform(sh.y);
                    cur_slot = k;
                    node = 0;
                    mask = inst_mask & ~done;
                    if (COUNT && (mask & me)) wc.inst++;
                    found = mask != 0;
                    continue;
                }
                level = 0;
            }
            if (sp == 0) return hit;
            sp--;
            node = uniform(st.node[sp]);
            mask = uniform64(st.mask[sp]) & ~done;
            found = mask != 0;
        }
    }
}

}  // namespace yrt
