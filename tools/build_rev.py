"""Build libyrt.so from the sources of a git revision, for in-process A/B against the
working tree (tools/ab_variants.py):

    python tools/build_rev.py HEAD r4        # -> yocto_raytracing_amd/variants/libyrt_r4.so

The revision's csrc/ and include/ are exported with `git archive` into a scratch
directory and compiled with the working tree's build flags (build.py).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "yocto_raytracing_amd"
sys.path.insert(0, str(PKG))
import build as b  # noqa: E402


def main(argv):
    rev, name, defines = argv[0], argv[1], argv[2:]
    out = PKG / "variants" / f"libyrt_{name}.so"
    out.parent.mkdir(exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        arc = subprocess.run(["git", "-C", str(ROOT), "archive", rev, "yocto_raytracing_amd/csrc", "include"],
                             check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", td], input=arc, check=True)
        csrc, inc = Path(td) / "yocto_raytracing_amd" / "csrc", Path(td) / "include"
        common = [f for f in b.COMMON if not f.startswith("-I")] + [f"-I{csrc}", f"-I{inc}"]
        jobs, objs = [], []
        for src in b.SOURCES:
            o = Path(td) / (Path(src).stem + ".o")
            if src.endswith(".hip"):
                cmd = [b.HIPCC, *common, *b.DEVICE_FLAGS, *defines, f"--offload-arch={b.ARCH}", "-c", str(csrc / src), "-o", str(o)]
            else:
                cmd = [b.CLANGXX, *common, *b.HOST_DEFS, *defines, "-c", str(csrc / src), "-o", str(o)]
            jobs.append(cmd)
            objs.append(o)

        def run(cmd):
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode:
                raise RuntimeError(" ".join(map(str, cmd)) + "\n" + r.stderr[-4000:])

        with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            list(ex.map(run, jobs))
        subprocess.run([b.HIPCC, "-shared", "-fPIC", f"--offload-arch={b.ARCH}", "-o", str(out), *map(str, objs),
                        *b.LINK_LIBS], check=True)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1:])
