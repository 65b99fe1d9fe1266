"""In-tree build of the native library (libyrt.so), the CLI and the test oracle.

hipcc drives everything (no cmake): host C++ and the gfx950 kernels are compiled
with -ffp-contract=off so that no a*b+c is fused anywhere on the hot path (the
reference's x86-64 build has no FMA). Objects are rebuilt only when
a source or header is newer.

    python yocto_raytracing_amd/build.py            # library + CLI
    python yocto_raytracing_amd/build.py --oracle   # + oracle/liboracle.so (+ oracle/_ref if present)
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
LIB = PKG / "libyrt.so"
CLI = PKG / "yrt_raytrace"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CLANGXX = os.environ.get("YRT_CXX", "/opt/rocm/lib/llvm/bin/clang++")
ARCH = os.environ.get("YRT_OFFLOAD_ARCH", "gfx950")

SOURCES = ["obj_loader.cpp", "png.cpp", "scene_io.cpp", "bvh_build.cpp",
           "device_scene.cpp", "capi.cpp", "render.hip", "wavefront.hip"]
COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          f"-I{CSRC}", f"-I{ROOT / 'include'}"]


HOST_DEFS = ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
# device code: leave wave-uniform regions unstructurized. Every branch of the BVH walks
# is on an SGPR value; structurizing them adds flow variables and exec-mask juggling
# (SALU) to every traversal step (A/B at c4: primary -2 %, shadow -4 %).
DEVICE_FLAGS = ["-mllvm", "-structurizecfg-skip-uniform-regions=true"]


def _headers():
    return list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h*"))


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def build_library(verbose: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    hdrs = _headers()
    jobs = []
    objs = []
    for src in SOURCES:
        s = CSRC / src
        o = BUILD / (s.stem + ".o")
        objs.append(o)
        if _stale(o, [s, *hdrs]):
            if src.endswith(".hip"):
                cmd = [HIPCC, *COMMON, *DEVICE_FLAGS, f"--offload-arch={ARCH}", "-c", str(s), "-o", str(o)]
            else:  # host-only C++: same clang, no offload
                cmd = [CLANGXX, *COMMON, *HOST_DEFS, "-c", str(s), "-o", str(o)]
            jobs.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for r in ex.map(_run, jobs):
            if verbose:
                print(r.stderr, end="")
    if _stale(LIB, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(LIB), *map(str, objs), "-lz"])
    cli_src = CSRC / "cli.cpp"
    if cli_src.exists() and _stale(CLI, [cli_src, LIB, *hdrs]):
        _run([CLANGXX, *COMMON, *HOST_DEFS, str(cli_src), "-o", str(CLI),
              f"-L{PKG}", "-lyrt", "-Wl,-rpath,$ORIGIN"])
    return LIB


def build_oracle() -> None:
    """Test infrastructure only: the C restatement, and the reference build when present."""
    _run(["make", "-C", str(ROOT / "oracle"), "liboracle.so"])
    if Path("/root/reference/src/raytrace.cpp").exists():
        _run(["make", "-C", str(ROOT / "oracle"), "-j8", "ref"])


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    build_library(verbose="-v" in argv)
    print(f"built {LIB}")
    if "--oracle" in argv:
        build_oracle()
        print("built oracle")


if __name__ == "__main__":
    main()
