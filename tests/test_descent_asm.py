"""descent_asm.h and wide_asm.h are generated: the committed headers must be what
tools/gen_descent_asm.py and tools/gen_wide_asm.py write (the walks' parity tests run the
committed headers), and their blocks must keep the shape the generators' docstrings describe."""
import importlib.util
import re

from helpers import ROOT

HDR = ROOT / "yocto_raytracing_amd" / "csrc" / "descent_asm.h"


def _gen(name="gen_descent_asm"):
    spec = importlib.util.spec_from_file_location(name, ROOT / "tools" / f"{name}.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_header_is_generated(tmp_path, monkeypatch):
    gen = _gen()
    out = tmp_path / "descent_asm.h"
    monkeypatch.setattr(gen, "OUT", out)
    gen.main()
    assert out.read_text() == HDR.read_text(), "descent_asm.h differs from tools/gen_descent_asm.py's output"


def test_blocks_per_octant_and_kind():
    text = HDR.read_text()
    specs = re.findall(r"struct descent_asm<(\d), (true|false)>", text)
    assert sorted(specs) == sorted((str(o), r) for r in ("true", "false") for o in range(8))


def test_scalar_work_per_record():
    # the hot path of one spine record (both children pass, neither a leaf): two mask ANDs,
    # two leaf tests, the m0 set and advance, and the stack pointer and node adds -- 8 SALU,
    # no compare of a mask against 0
    gen = _gen()
    for rel in (True, False):
        for oct_ in range(8):
            body = gen.body(oct_, rel)
            hot = body[: body.index("s_branch .Lyd_loop%=") + 1]
            salu = [x for x in hot if x.startswith("s_") and not x.startswith(("s_load", "s_waitcnt", "s_nop", "s_branch", "s_cbranch"))]
            assert len(salu) == 8, salu
            assert not any(x.startswith("s_cmp_lg_u64") for x in hot)
            assert sum(x.startswith("v_writelane_b32") for x in hot) == 2
            # the REL records hold (bound - o): no subtraction
            assert any(x.startswith("v_sub_f32") for x in hot) == (not rel)


WIDE = ROOT / "yocto_raytracing_amd" / "csrc" / "wide_asm.h"


def test_wide_header_is_generated(tmp_path, monkeypatch):
    gen = _gen("gen_wide_asm")
    out = tmp_path / "wide_asm.h"
    monkeypatch.setattr(gen, "OUT", out)
    gen.main()
    assert out.read_text() == WIDE.read_text(), "wide_asm.h differs from tools/gen_wide_asm.py's output"


def test_wide_selection_pops_in_slot_order():
    # the chain pushes every passing slot above the lowest, highest first (so they pop in
    # slot order), and pops keep the entries' lane masks (ANDed with the lanes not done)
    gen = _gen("gen_wide_asm")
    for oct_ in range(8):
        body = gen.body(oct_)
        assert sum(x.startswith("v_writelane_b32 %[sw]") for x in body) == 6  # b32 b31 b30 b21 b20 b10
        assert "s_andn2_b64 %[mask], s[48:49], %[done]" in body
        assert sum(x.startswith("v_cmp_le_f32") for x in body) == 4
        # slots 2 and 3 are tested only when present (an empty slot's word is wide_leaf exactly)
        assert body.count("s_cmp_eq_u32 s46, 0x80000000") == 1 and body.count("s_cmp_eq_u32 s47, 0x80000000") == 1
        # never the stack / frame pointers
        assert not any(re.search(r"\bs3[23]\b|s\[3[23]:", x) for x in body)
