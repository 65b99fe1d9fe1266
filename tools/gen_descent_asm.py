"""Generate yocto_raytracing_amd/csrc/descent_asm.h: the closest hit's descent loop
(packet_trace.h first_descend, maskless stack) as one inline-assembly block per ray octant
and record kind, so that the scalar unit issues only what the walk needs.

    python tools/gen_descent_asm.py        (rewrites the header; build.py does not run it)

Why assembly: compiled, each spine record's two lane-mask tests are `s_and_b64` followed by
an `s_cmp_lg_u64` of the result against 0 -- the AND already sets SCC, but the backend does
not fold the compare for 64-bit masks -- and each push recomputes the stack slot into `m0`
from the stack pointer. Here the branches read the AND's SCC, and the second push of a
record advances `m0` itself: 8 scalar instructions per record instead of 11.

The block is the same computation as first_descend<OCT, false, REL, 0, false>: the slab test
of intersect_check_bbox (scene.cpp:371-382) with the octant's swaps resolved (box_oct), the
reference's DFS (child start+1 first), the walk's stack in the lanes of one VGPR
(v_writelane / v_readlane at the stack pointer) and pops tested with the level's available
lanes (inner_pop_avail). It clobbers s16-s31 (the spine record) and writes VCC, M0 and SCC.
Hazard spacing: the record's SGPRs are read by the VALU after `s_waitcnt` and one `s_nop`, as
the compiler spaces its own scalar loads; a popped node offset (written by `v_readlane`)
reaches the next `s_load` after further scalar instructions.
"""
from __future__ import annotations

from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "yocto_raytracing_amd" / "csrc" / "descent_asm.h"

# the spine record in s16-s31: node A (the popped / continued node X) then node B (X's
# child start+1): {lo.xyz, word} {hi.xyz, count|leaf}
REC = {
    0: {"lo": ("s16", "s17", "s18"), "hi": ("s20", "s21", "s22"), "word": "s19", "cnt": "s23"},
    1: {"lo": ("s24", "s25", "s26"), "hi": ("s28", "s29", "s30"), "word": "s27", "cnt": "s31"},
}


def box(k: int, oct_: int, rel: bool) -> list[str]:
    """the slab test of record node k into VCC (box_oct<OCT> with o = the ray origin, or the
    records relative to it when rel)"""
    r = REC[k]
    o = ("%[ox]", "%[oy]", "%[oz]")
    c = ("%[cx]", "%[cy]", "%[cz]")
    lines = []
    near, far = [], []
    for a in range(3):
        neg = (oct_ >> a) & 1
        n_src, f_src = (r["hi"][a], r["lo"][a]) if neg else (r["lo"][a], r["hi"][a])
        near.append(n_src)
        far.append(f_src)
    # t0 = near x, t1 = far x, t2 = near y, t3 = far y, t4 = near z, t5 = far z
    t = ["%[t0]", "%[t1]", "%[t2]", "%[t3]", "%[t4]", "%[t5]"]
    for a in range(3):
        for j, src in enumerate((near[a], far[a])):
            dst = t[2 * a + j]
            if rel:
                lines.append(f"v_mul_f32 {dst}, {src}, {c[a]}")
            else:
                lines.append(f"v_sub_f32 {dst}, {src}, {o[a]}")
                lines.append(f"v_mul_f32 {dst}, {dst}, {c[a]}")
    # fmaxf(fmaxf(fmaxf(t0x, t0y), t0z), tmin) and fminf(fminf(fminf(t1x, t1y), t1z), tmax)
    lines.append("v_max_f32 %[t0], %[t0], %[t2]")
    lines.append("v_min_f32 %[t1], %[t1], %[t3]")
    lines.append("v_max3_f32 %[t0], %[t0], %[t4], %[tmin]")
    lines.append("v_min3_f32 %[t1], %[t1], %[t5], %[tmax]")
    lines.append("v_mul_f32 %[t1], 0x3f800002, %[t1]")  # tmax *= 1.00000024f
    lines.append("v_cmp_le_f32 vcc, %[t0], %[t1]")
    return lines


def body(oct_: int, rel: bool) -> list[str]:
    r0, r1 = REC[0], REC[1]
    L = []
    L.append(".Lyd_loop%=:")
    L.append("s_load_dwordx16 s[16:31], %[pb], %[node]")
    L.append("s_waitcnt lgkmcnt(0)")
    L.append("s_nop 0")
    L += box(0, oct_, rel)
    L.append("s_and_b64 %[mask], vcc, %[mask]")  # SCC = some lane passes X
    L.append("s_cbranch_scc0 .Lyd_pop%=")
    L.append(f"s_cmp_lt_i32 {r0['cnt']}, 0")  # X a leaf
    L.append("s_cbranch_scc1 .Lyd_leaf0%=")
    L.append("s_mov_b32 m0, %[sp]")  # push X's child start for the lanes that passed X
    L.append(f"v_writelane_b32 %[stk], {r0['word']}, m0")
    L += box(1, oct_, rel)
    L.append("s_and_b64 %[mask], vcc, %[mask]")  # SCC = some lane passes R (X's child start+1)
    L.append("s_cbranch_scc0 .Lyd_pop1%=")
    L.append(f"s_cmp_lt_i32 {r1['cnt']}, 0")  # R a leaf
    L.append("s_cbranch_scc1 .Lyd_leaf1%=")
    L.append("s_add_u32 m0, m0, 1")  # push R's child start
    L.append(f"v_writelane_b32 %[stk], {r1['word']}, m0")
    L.append("s_add_u32 %[sp], %[sp], 2")
    L.append(f"s_add_u32 %[node], {r1['word']}, 64")  # on at R's child start+1
    L.append("s_branch .Lyd_loop%=")
    L.append(".Lyd_pop1%=:")
    L.append("s_add_u32 %[sp], %[sp], 1")
    L.append(".Lyd_pop%=:")  # mask is 0 here
    L.append("s_cmp_le_i32 %[sp], %[floor]")
    L.append("s_cbranch_scc1 .Lyd_end%=")
    L.append("s_sub_u32 %[sp], %[sp], 1")
    L.append("v_readlane_b32 %[node], %[stk], %[sp]")
    L.append("s_mov_b64 %[mask], %[avail]")
    L.append("s_nop 3")
    L.append("s_branch .Lyd_loop%=")
    L.append(".Lyd_leaf0%=:")
    L.append(f"s_mov_b32 %[node], {r0['word']}")
    L.append(f"s_mov_b32 %[cl], {r0['cnt']}")
    L.append("s_branch .Lyd_end%=")
    L.append(".Lyd_leaf1%=:")
    L.append("s_add_u32 %[sp], %[sp], 1")
    L.append(f"s_mov_b32 %[node], {r1['word']}")
    L.append(f"s_mov_b32 %[cl], {r1['cnt']}")
    L.append(".Lyd_end%=:")
    return L


def emit(oct_: int, rel: bool) -> str:
    lines = "\n".join(f'        "{x}\\n"' for x in body(oct_, rel))
    o_in = "" if rel else ', [ox] "v"(o.x), [oy] "v"(o.y), [oz] "v"(o.z)'
    clob = ", ".join(f'"s{i}"' for i in range(16, 32))
    return f"""template <>
struct descent_asm<{oct_}, {str(rel).lower()}> {{
    static __device__ __forceinline__ void run(const f4* pb, vec3f o, vec3f ci, float tmin, float tmax, int floor,
                                               unsigned long long avail, int& node, unsigned long long& mask, int& sp,
                                               int& stk, uint32_t& cl) {{
        float t0, t1, t2, t3, t4, t5;
        asm volatile(
{lines}
            : [node] "+s"(node), [mask] "+s"(mask), [sp] "+s"(sp), [stk] "+v"(stk), [cl] "+s"(cl), [t0] "=&v"(t0),
              [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4), [t5] "=&v"(t5)
            : [pb] "s"(pb), [cx] "v"(ci.x), [cy] "v"(ci.y), [cz] "v"(ci.z), [tmin] "v"(tmin), [tmax] "v"(tmax),
              [floor] "s"(floor), [avail] "s"(avail){o_in}
            : {clob}, "vcc", "m0", "scc");
    }}
}};
"""


def main():
    parts = [
        "// descent_asm.h -- GENERATED by tools/gen_descent_asm.py (do not edit): the closest hit's\n"
        "// descent loop in one asm block per octant and record kind (first_descend, YRT_DESCENT_ASM;\n"
        "// the generator's docstring says what it computes and why).\n"
        "#pragma once\n\n"
        "#include \"trace_common.h\"\n\n"
        "namespace yrt {\n\n"
        "template <int OCT, bool REL>\nstruct descent_asm;\n\n"
    ]
    for rel in (True, False):
        for oct_ in range(8):
            parts.append(emit(oct_, rel))
            parts.append("\n")
    parts.append("}  // namespace yrt\n")
    OUT.write_text("".join(parts))
    print(OUT)


if __name__ == "__main__":
    main()
