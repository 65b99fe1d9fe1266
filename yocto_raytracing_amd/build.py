"""In-tree build of the native library (libyrt.so), the CLI and the test oracle.

hipcc drives everything (no cmake): host C++ and the gfx950 kernels are compiled
with -ffp-contract=off so that no a*b+c is fused anywhere on the hot path (the
reference's x86-64 build has no FMA). Objects are rebuilt when a
source or header is newer or the compile command (flags, -D knobs) changed.

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
           "device_scene.cpp", "capi.cpp", "multi.cpp", "render.hip", "wavefront.hip", "bvh_gpu.hip"]
COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          f"-I{CSRC}", f"-I{ROOT / 'include'}"]


HOST_DEFS = ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
LINK_LIBS = ["-lz", "-ldl", "-lpthread"]
# device code: leave wave-uniform regions unstructurized. Every branch of the BVH walks
# is on an SGPR value; structurizing them adds flow variables and exec-mask juggling
# (SALU) to every traversal step (A/B at c4: primary -2 %, shadow -4 %).
DEVICE_FLAGS = ["-mllvm", "-structurizecfg-skip-uniform-regions=true",
                # no SLP packing of adjacent f32 adds/muls into v_pk_*_f32: packed f32 does
                # not issue faster here and lengthens the dependent chains (A/B at c4:
                # primary -3 %, shadow -6.7 %, frame 32.7 -> 31.1 ms; identical images)
                "-fno-slp-vectorize"]


def _headers():
    return list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h*"))


def _stale(out: Path, deps, cmd=None) -> bool:
    """out is missing, older than a dependency, or was built by a different command
    (flags, -D knobs, compiler): the command is kept in a stamp file next to it"""
    if not out.exists():
        return True
    if cmd is not None:
        stamp = out.with_name(out.name + ".cmd")
        if not stamp.exists() or stamp.read_text() != " ".join(map(str, cmd)):
            return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _stamp(out: Path, cmd) -> None:
    out.with_name(out.name + ".cmd").write_text(" ".join(map(str, cmd)))


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
        if src.endswith(".hip"):
            cmd = [HIPCC, *COMMON, *DEVICE_FLAGS, f"--offload-arch={ARCH}", "-c", str(s), "-o", str(o)]
        else:  # host-only C++: same clang, no offload
            cmd = [CLANGXX, *COMMON, *HOST_DEFS, "-c", str(s), "-o", str(o)]
        if _stale(o, [s, *hdrs], cmd):
            jobs.append((o, cmd))

    def job(item):
        o, cmd = item
        r = _run(cmd)
        _stamp(o, cmd)
        return r

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for r in ex.map(job, jobs):
            if verbose:
                print(r.stderr, end="")
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(LIB), *map(str, objs), *LINK_LIBS]
    if _stale(LIB, objs, link):
        _run(link)
        _stamp(LIB, link)
    cli_src = CSRC / "cli.cpp"
    cli = [CLANGXX, *COMMON, *HOST_DEFS, str(cli_src), "-o", str(CLI), f"-L{PKG}", "-lyrt", "-Wl,-rpath,$ORIGIN"]
    if cli_src.exists() and _stale(CLI, [cli_src, LIB, *hdrs], cli):
        _run(cli)
        _stamp(CLI, cli)
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
