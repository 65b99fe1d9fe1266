"""Build-only checks of the compile-time knobs that survive in the device code.

The product is built with every knob at its default (yocto_raytracing_amd/build.py).
The knobs that remain are either tunables with a measured default (register
budgets, block sizes, XCD run lengths, the persistent-grid threshold) or kept
variants the ledger refers to (LDS staging of the top 4-wide records, the north
star's "hot node tiles in LDS") and the three diagnostic builds. None of them is
compiled by the normal build, so each non-default setting is compiled here for
gfx950 (device code only) to keep it from rotting. A knob added to the sources
without an entry below fails test_every_knob_is_listed.
"""
import concurrent.futures as cf
import os
import re
import subprocess

import pytest

from helpers import ROOT

CSRC = ROOT / "yocto_raytracing_amd" / "csrc"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# knob -> the non-default defines compiled here
VARIANTS = {
    "YRT_SHADOW_LDS_RECORDS": ["-DYRT_SHADOW_LDS_RECORDS=341"],
    "YRT_DEBUG_BOUNDS": ["-DYRT_DEBUG_BOUNDS"],
    "YRT_WIDE_STATS": ["-DYRT_WIDE_STATS"],
    "YRT_LIST_TIMING": ["-DYRT_LIST_TIMING"],
    "YRT_TAIL_STATS": ["-DYRT_TAIL_STATS"],
    "YRT_NT_STREAMS": ["-DYRT_NT_STREAMS=0"],
    "YRT_SHARED_TAIL": ["-DYRT_SHARED_TAIL=0"],
    "YRT_BUNDLE_SORT": ["-DYRT_BUNDLE_SORT=1"],
    "YRT_BUNDLE_SUPER": ["-DYRT_BUNDLE_SUPER=0"],
    "YRT_TRACE_WAVES": ["-DYRT_TRACE_WAVES=7"],
    "YRT_SHADOW_WAVES": ["-DYRT_SHADOW_WAVES=6"],
    "YRT_SHADE_WAVES": ["-DYRT_SHADE_WAVES=5"],
    "YRT_SHADE_LDS_SRGB": ["-DYRT_SHADE_LDS_SRGB=0"],
    "YRT_PRIMARY_REL": ["-DYRT_PRIMARY_REL=0"],
    "YRT_FOLD_PREFETCH": ["-DYRT_FOLD_PREFETCH=1"],
    "YRT_HIT16": ["-DYRT_HIT16=1"],
    "YRT_SHADOW_BUNDLES": ["-DYRT_SHADOW_BUNDLES=0"],
    "YRT_CAMERA_LISTS": ["-DYRT_CAMERA_LISTS=0"],
    "YRT_CAMERA_LIST_MAX": ["-DYRT_CAMERA_LIST_MAX=12", "-DYRT_CAMERA_CUT_DEPTH=3"],
    "YRT_BUNDLE_ITEMS": ["-DYRT_BUNDLE_ITEMS=16", "-DYRT_BUNDLE_MIN_TOP=0"],
    "YRT_SKIP_UNUSED_V": ["-DYRT_SKIP_UNUSED_V=0"],
    "YRT_SHADE_LEVEL_WAVES": ["-DYRT_SHADE_LEVEL_WAVES=7"],
    "YRT_PRIMARY_LDS_RECORDS": ["-DYRT_PRIMARY_LDS_RECORDS=1023"],
    "YRT_PRIMARY_WAVES": ["-DYRT_PRIMARY_WAVES=6", "-DYRT_PRIMARY_SP_BLOCK=768"],
    "YRT_FAST_NORMALIZE": ["-DYRT_FAST_NORMALIZE=0"],
    # round 5: the conservative inner-slot test of the any-hit walk (both forms lost)
    # and the shadow-ray cull (on by default)
    "YRT_ANY_CONSERVATIVE": ["-DYRT_ANY_CONSERVATIVE=1"],
    "YRT_SHADOW_CULL": ["-DYRT_SHADOW_CULL=0"],
    "YRT_INSTANCE_MASKS": ["-DYRT_INSTANCE_MASKS=0"],
    "YRT_LISTS_MIN_SPP": ["-DYRT_LISTS_MIN_SPP=1"],
    # round 6: the closest hit's one-exit descent and pop, the camera lists' top cut, the fused
    # bundle lists, and the diagnostic (inexact) f32 pow of the f64-path A/B
    "YRT_DESCENT_ONE_EXIT": ["-DYRT_DESCENT_ONE_EXIT=0", "-DYRT_POP_ONE_EXIT=0"],
    "YRT_CAMERA_CUT_DEPTH": ["-DYRT_CAMERA_CUT_DEPTH=0"],
    "YRT_BUNDLE_FUSED": ["-DYRT_BUNDLE_FUSED=1"],
    "YRT_DIAG_POW_F32": ["-DYRT_DIAG_POW_F32"],
    # the closest hit's stack with lane masks (the round-5 form; off: inner_pop_avail)
    "YRT_STACK_MASKS": ["-DYRT_STACK_MASKS=1"],
    # the compiled descent loop instead of descent_asm.h's
    "YRT_DESCENT_ASM": ["-DYRT_DESCENT_ASM=0"],
    "YRT_WIDE_ASM": ["-DYRT_WIDE_ASM=0"],
    # the any-hit grid's items as (block, light) pairs (the round-5 form; on: every light per item)
    "YRT_SHADOW_ITEM_LIGHTS": ["-DYRT_SHADOW_ITEM_LIGHTS=0", "-DYRT_SHADOW_ITEM_RUN=8"],
    # round-5 register-pressure A/B (k_primary_persist), one knob per change
    "YRT_R5_LANE": ["-DYRT_R5_LANE=0", "-DYRT_R5_UORIG=0", "-DYRT_R5_VCONST=0", "-DYRT_R5_IDXLANE=0", "-DYRT_R5_SURF=0"],
    "YRT_LEVEL_SEGMENTS": ["-DYRT_LEVEL_SEGMENTS=32"],
    "YRT_PRIMARY_BLOCK": ["-DYRT_PRIMARY_BLOCK=256", "-DYRT_SHADOW_BLOCK=256", "-DYRT_SHADOW_BLOCK_CHUNK=64",
                          "-DYRT_SHADOW_LIGHT_MINOR=16", "-DYRT_XCD_CHUNK_PRIMARY=64",
                          "-DYRT_SHADOW_PERSIST_MIN_ITEMS=0", "-DYRT_PRIMARY_PERSIST_MIN_ITEMS=1000000",
                          "-DYRT_PRIMARY_BLOCK_CHUNK=64"],
}
# knobs covered by another entry's defines
COVERED = {"YRT_SHADOW_ITEM_RUN", "YRT_POP_ONE_EXIT", "YRT_R5_UORIG", "YRT_R5_VCONST", "YRT_R5_IDXLANE", "YRT_R5_SURF", "YRT_BUNDLE_MIN_TOP", "YRT_PRIMARY_SP_BLOCK", "YRT_SHADOW_BLOCK", "YRT_SHADOW_BLOCK_CHUNK", "YRT_SHADOW_LIGHT_MINOR", "YRT_XCD_CHUNK_PRIMARY",
           "YRT_SHADOW_PERSIST_MIN_ITEMS", "YRT_PRIMARY_PERSIST_MIN_ITEMS", "YRT_PRIMARY_BLOCK_CHUNK"}


def _knobs_in_sources():
    found = set()
    for p in list(CSRC.glob("*.h")) + list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")):
        found |= set(re.findall(r"#\s*if(?:n?def)?\s+(YRT_[A-Z0-9_]+)", p.read_text()))
    return found


def test_every_knob_is_listed():
    knobs = _knobs_in_sources()
    assert knobs, "no knobs found"
    missing = knobs - set(VARIANTS) - COVERED
    assert not missing, f"knobs without a build-only variant: {sorted(missing)}"
    stale = (set(VARIANTS) | COVERED) - knobs
    assert not stale, f"listed knobs no longer in the sources: {sorted(stale)}"


def _compile(defs):
    cmd = [HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", f"-I{CSRC}", f"-I{ROOT / 'include'}", "-mllvm",
           "-structurizecfg-skip-uniform-regions=true", "-fno-slp-vectorize", "--offload-arch=gfx950",
           "--offload-device-only", "-c", str(CSRC / "wavefront.hip"), "-o", os.devnull, *defs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return defs, r.returncode, r.stderr[-3000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_non_default_knobs_compile():
    with cf.ThreadPoolExecutor(max_workers=min(len(VARIANTS), max(1, (os.cpu_count() or 2) - 1))) as ex:
        results = list(ex.map(_compile, VARIANTS.values()))
    failed = [(d, err) for d, rc, err in results if rc != 0]
    assert not failed, "\n".join(f"{d}:\n{err}" for d, err in failed)
