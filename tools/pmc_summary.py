"""Summarise rocprofv3 counter CSVs into per-kernel HBM traffic per launch.

    python tools/pmc_summary.py --key instance10000-r1080-s8-n1-wavefront \
        --fetch gpurun_out/p3/p3_counter_collection.csv \
        --write gpurun_out/p4/p4_counter_collection.csv \
        [--kernel-trace gpurun_out/ks/ks_kernel_stats.csv] > profiles/pmc_traffic.json

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads (16 B/lane), and
WRITE_SIZE is exact for 16-B stores (MI355X_MICROARCH.md, HBM section); both come
from separate --pmc passes. Only the un-instrumented (COUNT=false, first template argument) kernels are kept.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re

PHASE_OF = {"k_primary": "primary", "k_shadow": "shadow", "k_shade": "shade", "k_bounce": "bounce",
            "k_fold_children": "fold", "k_accumulate": "accumulate", "render_kernel": "megakernel"}


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(k_\w+|render_kernel|trace_kernel)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def per_launch(path: str, counter: str) -> dict:
    vals = collections.defaultdict(float)
    launches = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        if re.match(r"\w+<true", k):  # COUNT=true: the instrumented twin
            continue
        vals[k] += float(r["Counter_Value"])
        launches[k].add(r["Dispatch_Id"])
    return {k: vals[k] / max(1, len(launches[k])) for k in vals}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--merge", help="existing json to extend")
    a = ap.parse_args()
    fetch = per_launch(a.fetch, "FETCH_SIZE")
    write = per_launch(a.write, "WRITE_SIZE")
    out = json.load(open(a.merge)) if a.merge else {}
    for k in sorted(set(fetch) | set(write)):
        base = k.split("<")[0]
        phase = PHASE_OF.get(base)
        if not phase:
            continue
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        out[f"{a.key}-{phase}"] = {
            "kernel": k, "fetch_size_kb": f, "write_size_kb": w,
            "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
            "note": "2*FETCH_SIZE (gfx950 half-count on 16B/lane streams) + WRITE_SIZE, KB->B",
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
