"""The gfx950 code object inside a built object or library, and its disassembly.

    python tools/isa_dump.py yocto_raytracing_amd/libyrt.so            # code identity (sha256)
    python tools/isa_dump.py --isa OUT.txt yocto_raytracing_amd/_build/wavefront.o

The disassembly is normalised (addresses, encodings and branch-target offsets
stripped) so that two builds can be diffed: a refactor that only removes
compile-time variants must leave every default kernel's instructions unchanged.
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _codeid():
    # by path: importing the package would load libyrt.so (and torch)
    import importlib.util

    spec = importlib.util.spec_from_file_location("yrt_codeid", ROOT / "yocto_raytracing_amd" / "codeid.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_C = _codeid()
LLVM, code_identity, code_objects = _C.LLVM, _C.code_identity, _C.code_objects


def disassemble(co: bytes) -> str:
    with tempfile.TemporaryDirectory() as td:
        p = Path(td) / "co"
        p.write_bytes(co)
        r = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", "--no-leading-addr", str(p)],
                           check=True, capture_output=True, text=True)
    out = []
    for line in r.stdout.splitlines():
        line = re.sub(r"//.*$", "", line).rstrip()
        line = re.sub(r"<[^>]*\+0x[0-9a-f]+>", "<L>", line)  # branch targets inside a function
        if line and not line.startswith(str(p)):
            out.append(line)
    return "\n".join(out) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--isa", help="write the normalised disassembly here")
    a = ap.parse_args(argv)
    print(code_identity(Path(a.path)))
    if a.isa:
        Path(a.isa).write_text("".join(disassemble(co) for co in code_objects(Path(a.path))))


if __name__ == "__main__":
    sys.exit(main())
