"""Summarise rocprofv3 counter CSVs into the two files bench.py reads.

    python tools/pmc_summary.py --key instance10000-1920x1080-s8-n1-wavefront \
        --csv gpurun_out/T/p*/p*_counter_collection.csv --source profiles/r2/T \
        --traffic profiles/pmc_traffic.json --issue profiles/issue_counters.json

Per timed kernel (COUNT=false, first template argument) and per launch:
* traffic: HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024. On gfx950 FETCH_SIZE
  reports half the bytes of wide coalesced streaming reads (16 B/lane) and WRITE_SIZE is
  exact for 16-B stores (MI355X_MICROARCH.md, HBM section); separate --pmc passes.
* issue: the SQ_* / GRBM_* / SQC_* counters as collected (chip totals per launch), plus
  derived rates: clock cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs);
  SALU busy = SQ_INSTS_SALU / (256 CUs x cycles) (one scalar unit per CU, one issue per
  clock); VALU busy = SQ_INSTS_VALU / (256 x 4 SIMDs x cycles / 2) (a wave64 VALU
  instruction takes two clocks on a SIMD-32); scalar-cache hit rate.
Every entry is stamped with the code identity (yocto_raytracing_amd/codeid.py) of the
library the counters were collected from (--lib): bench.py pairs committed counters
only with a timed library of the same identity.
Entries are merged into the existing files (same key = replaced).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import importlib.util
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def code_identity(lib: Path) -> str:
    spec = importlib.util.spec_from_file_location("yrt_codeid", ROOT / "yocto_raytracing_amd" / "codeid.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.code_identity(lib)

PHASE_OF = {"k_primary": "primary", "k_primary_persist": "primary", "k_shadow": "shadow",
            "k_shadow_persist": "shadow", "k_shade": "shade", "k_bounce": "bounce",
            "k_fold_children": "fold", "k_accumulate": "accumulate", "render_kernel": "megakernel",
            "k_relative_records": "lists", "k_chunk_setup": "lists", "k_bundle_super": "lists", "k_camera_lists": "lists", "k_bundle_lists": "lists", "k_list_stats": "lists"}


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(k_\w+|render_kernel|trace_kernel)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def per_launch(paths) -> dict:
    """{phase: {counter: mean value per dispatch}, "_kernels": {phase: [kernel names]}} over
    the timed kernels of each phase (a reflective frame's shadow phase has one persistent
    level-0 launch and one grid-stride launch per mirror level: their mean per launch is
    what bench.py's per-launch time is set against)"""
    vals = collections.defaultdict(float)
    launches = collections.defaultdict(set)
    kernels = collections.defaultdict(set)
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if re.match(r"\w+<true", k):  # COUNT=true: the instrumented twin
                continue
            phase = PHASE_OF.get(k.split("<")[0])
            if not phase:
                continue
            kernels[phase].add(k)
            vals[(phase, r["Counter_Name"])] += float(r["Counter_Value"])
            launches[(phase, r["Counter_Name"])].add((path, r["Dispatch_Id"]))
    out = collections.defaultdict(dict)
    for (ph, c), v in vals.items():
        out[ph][c] = v / max(1, len(launches[(ph, c)]))
    out["_kernels"] = {ph: sorted(ks) for ph, ks in kernels.items()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", required=True, help="{scene}-{W}x{H}-s{spp axis}-n{ranks}-{algorithm}")
    ap.add_argument("--csv", nargs="+", required=True)
    ap.add_argument("--source", default="", help="where the CSVs are committed")
    ap.add_argument("--traffic", default="profiles/pmc_traffic.json")
    ap.add_argument("--issue", default="profiles/issue_counters.json")
    ap.add_argument("--lib", default=str(ROOT / "yocto_raytracing_amd" / "libyrt.so"),
                    help="the library the counters were collected from (its code identity is stamped)")
    a = ap.parse_args()
    ident = code_identity(Path(a.lib))
    data = per_launch(a.csv)
    traffic = json.loads(Path(a.traffic).read_text()) if Path(a.traffic).exists() else {}
    issue = json.loads(Path(a.issue).read_text()) if Path(a.issue).exists() else {}
    names = data.pop("_kernels")
    for phase, c in sorted(data.items()):
        k = " + ".join(names.get(phase, [])) or phase
        key = f"{a.key}-{phase}"
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            f, w = c["FETCH_SIZE"], c["WRITE_SIZE"]
            traffic[key] = {"kernel": k, "fetch_size_kb": f, "write_size_kb": w,
                            "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024, "source": a.source,
                            "code_identity": ident,
                            "note": "2*FETCH_SIZE (gfx950 half-count on 16B/lane streams) + WRITE_SIZE, KB->B"}
        rec = {n: v for n, v in c.items() if n.startswith(("SQ_", "SQC_", "GRBM_"))}
        if "SQ_INSTS_SALU" in rec and "SQ_INSTS_VALU" in rec:
            rec = {"kernel": k, "source": a.source, "code_identity": ident, **rec}
            cyc = rec.get("GRBM_GUI_ACTIVE", 0) / 8
            if cyc:
                rec["cycles"] = cyc
                rec["salu_busy"] = rec["SQ_INSTS_SALU"] / (256 * cyc)
                rec["valu_busy"] = rec["SQ_INSTS_VALU"] * 2 / (256 * 4 * cyc)
            if rec.get("SQ_WAVES"):
                rec["salu_per_wave"] = rec["SQ_INSTS_SALU"] / rec["SQ_WAVES"]
                rec["valu_per_wave"] = rec["SQ_INSTS_VALU"] / rec["SQ_WAVES"]
            h, m = rec.get("SQC_DCACHE_HITS"), rec.get("SQC_DCACHE_MISSES")
            if h is not None and m is not None and h + m:
                rec["sqc_dcache_hit_rate"] = h / (h + m)
            issue[key] = rec
    Path(a.traffic).write_text(json.dumps(traffic, indent=1, sort_keys=True) + "\n")
    Path(a.issue).write_text(json.dumps(issue, indent=1, sort_keys=True) + "\n")
    print(json.dumps({k: v for k, v in issue.items() if k.startswith(a.key)}, indent=1))


if __name__ == "__main__":
    main()
