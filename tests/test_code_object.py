"""Register budgets of the timed kernels, read from the shipped library's gfx950 code objects
(the AMDHSA metadata note: yocto_raytracing_amd/codeid.py kernel_resources).

The traversal kernels run at 8 waves per SIMD, i.e. within 64 VGPRs and 78 SGPRs. A VGPR the
compiler cannot fit goes to scratch: a vector-memory round trip per spill site inside walks
that already wait a third of their cycles, and scratch lines that L2 writes back to HBM
(round 4's k_primary_persist with the camera lists spilled 23 VGPRs, 88 bytes per lane, and
wrote 2.67 GB per c4 frame more than its surface stream). SGPR spills go to VGPR lanes
(v_writelane / v_readlane) and are only bounded here. A change that brings scratch back to a
timed kernel fails this test before it reaches the GPU.
"""
import re

import pytest

from helpers import ROOT

LIB = ROOT / "yocto_raytracing_amd" / "libyrt.so"

# timed kernel (what it is) -> mangled-name pattern, and ceilings:
# (VGPR spills, private bytes per lane, SGPR spills[, static LDS bytes])
# The SGPR-spill ceilings are today's counts (ratcheted: a change that adds spills to a walk
# fails here and has to say why in DESIGN.md)
TIMED = {
    "k_primary_persist<uint, 0, list> (c4 closest hit)": (r"k_primary_persistIjLi0ELb1EE", 0, 0, 24),
    "k_primary_persist<uint, 0, tree> (lists off)": (r"k_primary_persistIjLi0ELb0EE", 0, 0, 24),
    # (28: the one-exit pop of round 6 is shared with the wide step -- two SGPR spills more than
    # its old form there, shadow phase unchanged in the A/B, profiles/r6/ab/r6b_ab_c4.txt)
    "k_shadow_persist<0> (c4 any hit)": (r"k_shadow_persistILi0EE", 0, 0, 32),
    "k_shade<fused, occ4> (c4 shading + per-pixel sum)": (r"k_shadeILb0ELb1ELi256ELb1EE", 0, 0, 16),
    "k_shade<level, occ4> (c3 mirror levels)": (r"k_shadeILb0ELb0ELi256ELb1EE", 0, 0, 52),
    "k_bounce<packet> (c3 mirror rays)": (r"k_bounceILb0ELb1EjEE", 0, 0, 36),
    "k_camera_lists": (r"k_camera_lists", 0, 0, 0),
    # (the list builders' 28 private bytes: a 7-float slot record indexed per lane, not spills)
    "k_bundle_lists": (r"k_bundle_listsILb0EE", 0, 28, 0),
    "k_bundle_super": (r"k_bundle_super", 0, 28, 0),
    # the LDS-staged walks (yrt_scene_set_lds_staging): 511 camera-relative spine records
    # (32 KiB) beside the parked 1/d, and 85 wide records; two 1024-thread blocks per CU must
    # still fit the CU's 160 KiB of LDS, i.e. at most 80 KiB per block
    "k_primary_persist<uint, 511, tree> (LDS staging)": (r"k_primary_persistIjLi511ELb0EE", 0, 0, 26, 80 * 1024),
    "k_shadow_persist<85> (LDS staging)": (r"k_shadow_persistILi85EE", 0, 0, 18, 80 * 1024),
}


@pytest.fixture(scope="module")
def resources():
    if not LIB.exists():
        from yocto_raytracing_amd import build

        build.build_library()
    from yocto_raytracing_amd.codeid import kernel_resources

    return kernel_resources(LIB)


@pytest.mark.parametrize("what", list(TIMED))
def test_timed_kernel_register_budget(resources, what):
    pat, vsp_max, priv_max, ssp_max, *lds_max = TIMED[what]
    hits = {k: v for k, v in resources.items() if re.search(pat, k)}
    assert len(hits) == 1, (what, sorted(hits))
    (name, r), = hits.items()
    print(what, r)
    assert r["vgpr_spill"] <= vsp_max, (what, r)
    assert r["private"] <= priv_max, (what, r)
    assert r["sgpr_spill"] <= ssp_max, (what, r)
    if lds_max:
        assert r["lds"] <= lds_max[0], (what, r)


def test_traversal_kernels_fit_eight_waves(resources):
    """the walks' register budget: 8 waves per SIMD hold at most 64 VGPRs each (512 per lane
    slot of a SIMD on gfx950)"""
    for pat in (r"k_primary_persistIjLi0ELb1EE", r"k_shadow_persistILi0EE"):
        (name, r), = {k: v for k, v in resources.items() if re.search(pat, k)}.items()
        assert r["vgpr"] <= 64 and r["sgpr"] <= 80, (name, r)
