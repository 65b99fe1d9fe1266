"""descent_asm.h is generated: the committed header must be what tools/gen_descent_asm.py
writes (the walk's parity tests run the committed header), and its blocks must keep the
shape the generator's docstring describes."""
import importlib.util
import re

from helpers import ROOT

HDR = ROOT / "yocto_raytracing_amd" / "csrc" / "descent_asm.h"


def _gen():
    spec = importlib.util.spec_from_file_location("gen_descent_asm", ROOT / "tools" / "gen_descent_asm.py")
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
