"""Build variants of libyrt.so that differ only in compile-time defines of the
kernels, for in-process A/B timing (tools/ab_variants.py).

    python tools/build_variants.py w7:-DYRT_TRACE_WAVES=7 lds85:-DYRT_SHADOW_LDS_RECORDS=85

writes yocto_raytracing_amd/variants/libyrt_<name>.so (git-ignored, travels to the GPU box).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "yocto_raytracing_amd"
sys.path.insert(0, str(PKG))
import build as b  # noqa: E402


def main(argv):
    b.build_library()
    out_dir = PKG / "variants"
    out_dir.mkdir(exist_ok=True)
    jobs, libs = [], []
    for spec in argv:
        name, _, defs = spec.partition(":")
        defines = [d for d in defs.split(",") if d]
        vdir = out_dir / name
        vdir.mkdir(exist_ok=True)
        objs = []
        for src in b.SOURCES:  # host and device code both see the defines
            o = vdir / (Path(src).stem + ".o")
            if src.endswith(".hip"):
                cmd = [b.HIPCC, *b.COMMON, *b.DEVICE_FLAGS, *defines, f"--offload-arch={b.ARCH}", "-c", str(b.CSRC / src), "-o", str(o)]
            else:
                cmd = [b.CLANGXX, *b.COMMON, *b.HOST_DEFS, *defines, "-c", str(b.CSRC / src), "-o", str(o)]
            jobs.append(cmd)
            objs.append(o)
        libs.append((out_dir / f"libyrt_{name}.so", objs))

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(" ".join(map(str, cmd)) + "\n" + r.stderr[-4000:])

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(run, jobs))
    for lib, objs in libs:
        subprocess.run([b.HIPCC, "-shared", "-fPIC", f"--offload-arch={b.ARCH}", "-o", str(lib), *map(str, objs), *b.LINK_LIBS],
                       check=True)
        print(lib)


if __name__ == "__main__":
    main(sys.argv[1:])
