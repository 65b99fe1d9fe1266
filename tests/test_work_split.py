"""The persistent grids' work split (wavefront.hip: head_items / chunk_fetch / split_item,
YRT_SHARED_TAIL): every item of a launch is taken exactly once -- the per-XCD head in whole
runs and whole block chunks, the shared tail in image order -- for the run and chunk sizes
the kernels are compiled with. A host model of the device index arithmetic (no GPU)."""
import random
import re
from math import gcd

import pytest

from helpers import ROOT

SRC = (ROOT / "yocto_raytracing_amd" / "csrc" / "wavefront.hip").read_text()


def knob(name):
    return int(re.search(rf"#define {name} (\d+)", SRC).group(1))


def covered(n_items, run, cs, div):
    """positions each XCD's blocks take, then the shared tail's, mapped to items"""
    g = 8 * (run // gcd(run, cs) * cs)
    head = (n_items - n_items // div) // g * g if div else 0
    limit = head // 8
    seen = [0] * n_items
    for xcd in range(8):
        k = 0
        while k * cs + cs <= limit:  # chunk_fetch: the XCD's own counter while its share lasts
            for o in range(cs):
                q = k * cs + o
                item = ((q // run) * 8 + xcd) * run + q % run
                assert item < head
                seen[item] += 1
            k += 1
    t = 0
    while head + t * cs < n_items:  # the shared counter: flagged positions, head + index
        for o in range(cs):
            if head + t * cs + o < n_items:
                seen[head + t * cs + o] += 1
        t += 1
    return seen


@pytest.mark.parametrize("grid", ["primary", "shadow"])
def test_every_item_taken_once(grid):
    div = knob("YRT_SHARED_TAIL")
    assert div > 0
    if grid == "primary":
        run, cs = knob("YRT_XCD_CHUNK_PRIMARY"), knob("YRT_PRIMARY_BLOCK_CHUNK")
    else:
        run, cs = knob("YRT_SHADOW_LIGHT_MINOR"), knob("YRT_SHADOW_BLOCK_CHUNK")
    rng = random.Random(7)
    sizes = [0, 1, 63, 64, 2047, 2048, 2049, 3072, 3073, 32768, 32769, 259200, 777600]
    sizes += [rng.randint(1, 400_000) for _ in range(12)]
    for n in sizes:
        seen = covered(n, run, cs, div)
        assert all(v == 1 for v in seen), (grid, n)
