"""Code identity of a built library: the sha256 of its gfx950 code objects.

Committed profiler counters (profiles/issue_counters.json, pmc_traffic.json) are
stamped with the identity of the library they were collected from; bench.py reports
an issue-rate roofline only when the library it just timed has the same identity, so
a counter file can never be paired with a kernel it did not measure. Host-side tool
(objcopy + clang-offload-bundler); nothing here touches the GPU.
"""
from __future__ import annotations

import hashlib
import re
import subprocess
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path) -> list:
    """the gfx950 code objects bundled in the .hip_fatbin section of an object or a
    library (a linked library holds one bundle per device source, concatenated)"""
    out = []
    with tempfile.TemporaryDirectory() as td:
        fat = Path(td) / "fatbin"
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", str(path), str(Path(td) / "scratch")],
                       check=True, capture_output=True)
        data = fat.read_bytes()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for k in range(len(starts) - 1):
            one = Path(td) / f"b{k}"
            co = Path(td) / f"co{k}"
            one.write_bytes(data[starts[k]:starts[k + 1]])
            subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={one}",
                            f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
            out.append(co.read_bytes())
    if not out:
        raise ValueError(f"{path}: no gfx950 code object")
    return out


def code_identity(path) -> str:
    """sha256 over the gfx950 code objects of `path`, in bundle order"""
    h = hashlib.sha256()
    for co in code_objects(Path(path)):
        h.update(hashlib.sha256(co).digest())
    return h.hexdigest()


_RES_KEYS = {"vgpr_count": "vgpr", "sgpr_count": "sgpr", "vgpr_spill_count": "vgpr_spill",
             "sgpr_spill_count": "sgpr_spill", "private_segment_fixed_size": "private",
             "group_segment_fixed_size": "lds", "max_flat_workgroup_size": "block"}


def kernel_resources(path) -> dict:
    """per kernel symbol of the gfx950 code objects in `path`: its register counts, spills,
    private (scratch) bytes per lane and static LDS bytes, from the code object's
    AMDHSA metadata note (llvm-readelf --notes)"""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(Path(path))):
            p = Path(td) / f"co{k}"
            p.write_bytes(co)
            notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(p)], check=True,
                                   capture_output=True, text=True).stdout
            # one YAML mapping per kernel under amdhsa.kernels, each starting with "  - ."
            for block in re.split(r"\n  - (?=\.)", notes)[1:]:
                m = re.search(r"^\s*\.name:\s+(\S+)", block, re.M)
                if not m:
                    continue
                res = {}
                for key, short in _RES_KEYS.items():
                    v = re.search(rf"^\s*\.{key}:\s+(\d+)", block, re.M)
                    if v:
                        res[short] = int(v.group(1))
                out[m.group(1)] = res
    return out
