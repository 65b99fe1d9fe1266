"""Generate yocto_raytracing_amd/csrc/wide_asm.h: the any-hit walk's 4-wide descent loop
(packet_trace.h wide_descend / wide_step, records through the scalar cache, exact slab tests)
as one inline-assembly block per ray octant.

    python tools/gen_wide_asm.py        (rewrites the header; build.py does not run it)

Why assembly: the compiled step spends ~20 scalar instructions per wide record, and the any
hit is bound by scalar issue (SALU ~0.74 of peak). Around the slot selection (already asm in
wide_step) the compiler adds compares of the selected mask against 0, copies of the asm's
results through readfirstlane, a leaf test of a copy and the loop's own bookkeeping. Here one
block runs the loop: the record load, the slab tests of the node's slots (slots 2 and 3 only
when the node has them), the ballot ANDs, the selection (the lowest passing slot goes on,
the others are pushed highest first so that they pop in slot order), the leaf test of the
next item, and the pops (stack entries keep their lane masks: a popped 4-wide entry is not
tested again, so its mask is the result of its box test at the parent).

The computation is wide_descend<OCT, 0>'s with YRT_ANY_CONSERVATIVE off: the same slab
tests (box_oct), the same order. The block clobbers s16-s31 and s36-s55 (the record, the slot
masks), VCC, M0 and SCC. It exits with mask != 0 and cur a leaf word, or mask = 0 when the level is done.
"""
from __future__ import annotations

from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "yocto_raytracing_amd" / "csrc" / "wide_asm.h"

# record rows: lo.x[4] lo.y[4] lo.z[4] hi.x[4] in s16-s31 (x16), hi.y[4] hi.z[4] in s36-s43
# (x8), word[4] in s44-s47 (x4); s32-s35 are left alone (s32/s33 are the stack and frame
# pointers of a kernel that has a stack, as the YRT_DEBUG_BOUNDS build's printf gives it)
LO = [(16 + k, 20 + k, 24 + k) for k in range(4)]
HI = [(28 + k, 36 + k, 40 + k) for k in range(4)]
WORD = [44 + k for k in range(4)]
MASK = [(48 + 2 * k, 49 + 2 * k) for k in range(4)]  # slot k's lanes: s[48+2k : 49+2k]


def s(i: int) -> str:
    return f"s{i}"


def m(k: int) -> str:
    lo, hi = MASK[k]
    return f"s[{lo}:{hi}]"


def box(k: int, oct_: int) -> list[str]:
    o = ("%[ox]", "%[oy]", "%[oz]")
    c = ("%[cx]", "%[cy]", "%[cz]")
    t = ["%[t0]", "%[t1]", "%[t2]", "%[t3]", "%[t4]", "%[t5]"]
    L = []
    for a in range(3):
        neg = (oct_ >> a) & 1
        near, far = (HI[k][a], LO[k][a]) if neg else (LO[k][a], HI[k][a])
        for j, src in enumerate((near, far)):
            dst = t[2 * a + j]
            L.append(f"v_sub_f32 {dst}, {s(src)}, {o[a]}")
            L.append(f"v_mul_f32 {dst}, {dst}, {c[a]}")
    L.append("v_max_f32 %[t0], %[t0], %[t2]")
    L.append("v_min_f32 %[t1], %[t1], %[t3]")
    L.append("v_max3_f32 %[t0], %[t0], %[t4], %[tmin]")
    L.append("v_min3_f32 %[t1], %[t1], %[t5], %[tmax]")
    L.append("v_mul_f32 %[t1], 0x3f800002, %[t1]")
    L.append("v_cmp_le_f32 vcc, %[t0], %[t1]")
    L.append(f"s_and_b64 {m(k)}, vcc, %[mask]")
    return L


def push(j: int) -> list[str]:
    lo, hi = MASK[j]
    return [
        "s_mov_b32 m0, %[sp]",
        f"v_writelane_b32 %[sw], {s(WORD[j])}, m0",
        f"v_writelane_b32 %[sl], {s(lo)}, m0",
        f"v_writelane_b32 %[sh], {s(hi)}, m0",
        "s_add_u32 %[sp], %[sp], 1",
    ]


def body(oct_: int) -> list[str]:
    L = [".Lyw_loop%=:"]
    L.append("s_load_dwordx16 s[16:31], %[wb], %[cur]")
    L.append("s_load_dwordx8 s[36:43], %[wb], %[cur] offset:0x40")
    L.append("s_load_dwordx4 s[44:47], %[wb], %[cur] offset:0x60")
    L.append("s_waitcnt lgkmcnt(0)")
    L.append("s_nop 0")
    L += box(0, oct_)
    L += box(1, oct_)
    L.append(f"s_mov_b64 {m(2)}, 0")
    L.append(f"s_mov_b64 {m(3)}, 0")
    # slots 2 and 3 exist unless their word is an empty slot's (wide_leaf exactly)
    L.append(f"s_cmp_eq_u32 {s(WORD[2])}, 0x80000000")
    L.append("s_cbranch_scc1 .Lyw_skip2%=")
    L += box(2, oct_)
    L.append(".Lyw_skip2%=:")
    L.append(f"s_cmp_eq_u32 {s(WORD[3])}, 0x80000000")
    L.append("s_cbranch_scc1 .Lyw_sel%=")
    L += box(3, oct_)
    # the selection (wide_step's chain): A(k) looks for the highest passing slot; B(j, k)
    # knows candidate j and tests slot k < j; a passing k pushes j and becomes the candidate
    L.append(".Lyw_sel%=:")
    L.append(f"s_cmp_lg_u64 {m(3)}, 0")
    L.append("s_cbranch_scc1 .Lyw_b32%=")
    L.append(f"s_cmp_lg_u64 {m(2)}, 0")
    L.append("s_cbranch_scc1 .Lyw_b21%=")
    L.append(f"s_cmp_lg_u64 {m(1)}, 0")
    L.append("s_cbranch_scc1 .Lyw_b10%=")
    L.append(f"s_cmp_lg_u64 {m(0)}, 0")
    L.append("s_cbranch_scc1 .Lyw_fin0%=")
    L.append("s_branch .Lyw_pop%=")  # no slot passes
    for j in (3, 2, 1):
        for k in range(j - 1, -1, -1):
            L.append(f".Lyw_b{j}{k}%=:")
            L.append(f"s_cmp_lg_u64 {m(k)}, 0")
            nxt = f".Lyw_b{j}{k - 1}%=" if k > 0 else f".Lyw_fin{j}%="
            L.append(f"s_cbranch_scc0 {nxt}")
            L += push(j)
            L.append(f"s_branch .Lyw_b{k}{k - 1}%=" if k > 0 else ".Lyw_fin0_br%=")
    # (b{k}{k-1} for k = 0 does not exist: a push of j at k = 0 continues at fin0)
    L = [x if x != ".Lyw_fin0_br%=" else "s_branch .Lyw_fin0%=" for x in L]
    for j in (3, 2, 1, 0):
        L.append(f".Lyw_fin{j}%=:")
        L.append(f"s_mov_b64 %[mask], {m(j)}")
        L.append(f"s_mov_b32 %[cur], {s(WORD[j])}")
        L.append(f"s_cmp_lt_i32 {s(WORD[j])}, 0")  # a leaf: wide_leaf is the sign bit
        L.append("s_cbranch_scc1 .Lyw_end%=")
        L.append("s_branch .Lyw_loop%=")
    # pops: entries above the floor until one still has lanes
    L.append(".Lyw_pop%=:")
    L.append("s_cmp_le_i32 %[sp], %[floor]")
    L.append("s_cbranch_scc1 .Lyw_exit0%=")
    L.append("s_sub_u32 %[sp], %[sp], 1")
    L.append(f"v_readlane_b32 {s(MASK[0][0])}, %[sl], %[sp]")
    L.append(f"v_readlane_b32 {s(MASK[0][1])}, %[sh], %[sp]")
    L.append("v_readlane_b32 %[cur], %[sw], %[sp]")
    L.append(f"s_andn2_b64 %[mask], {m(0)}, %[done]")
    L.append("s_cbranch_scc0 .Lyw_pop%=")
    L.append("s_cmp_lt_i32 %[cur], 0")
    L.append("s_cbranch_scc1 .Lyw_end%=")
    L.append("s_nop 3")
    L.append("s_branch .Lyw_loop%=")
    L.append(".Lyw_exit0%=:")
    L.append("s_mov_b64 %[mask], 0")
    L.append(".Lyw_end%=:")
    return L


def emit(oct_: int) -> str:
    lines = "\n".join(f'        "{x}\\n"' for x in body(oct_))
    clob = ", ".join(f'"s{i}"' for i in list(range(16, 32)) + list(range(36, 56)))
    return f"""template <>
struct wide_asm<{oct_}> {{
    static __device__ __forceinline__ void run(const f4* wb, vec3f o, vec3f ci, float tmin, float tmax, int floor,
                                               unsigned long long done, uint32_t& cur, unsigned long long& mask,
                                               int& sp, int& sw, int& sl, int& sh) {{
        float t0, t1, t2, t3, t4, t5;
        asm volatile(
{lines}
            : [cur] "+s"(cur), [mask] "+s"(mask), [sp] "+s"(sp), [sw] "+v"(sw), [sl] "+v"(sl), [sh] "+v"(sh),
              [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4), [t5] "=&v"(t5)
            : [wb] "s"(wb), [ox] "v"(o.x), [oy] "v"(o.y), [oz] "v"(o.z), [cx] "v"(ci.x), [cy] "v"(ci.y),
              [cz] "v"(ci.z), [tmin] "v"(tmin), [tmax] "v"(tmax), [floor] "s"(floor), [done] "s"(done)
            : {clob}, "vcc", "m0", "scc");
    }}
}};
"""


def main():
    parts = [
        "// wide_asm.h -- GENERATED by tools/gen_wide_asm.py (do not edit): the any-hit walk's 4-wide\n"
        "// descent loop in one asm block per octant (wide_descend, YRT_WIDE_ASM; the generator's\n"
        "// docstring says what it computes and why).\n"
        "#pragma once\n\n"
        "#include \"trace_common.h\"\n\n"
        "namespace yrt {\n\n"
        "template <int OCT>\nstruct wide_asm;\n\n"
    ]
    for oct_ in range(8):
        parts.append(emit(oct_))
        parts.append("\n")
    parts.append("}  // namespace yrt\n")
    OUT.write_text("".join(parts))
    print(OUT)


if __name__ == "__main__":
    main()
