"""Per-kernel table of rocprofv3 counter CSVs (mean per dispatch).

    python tools/pmc_table.py FILE.csv [FILE2.csv ...] [--match k_shadow]
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("files", nargs="+")
ap.add_argument("--match", default="k_")
a = ap.parse_args()
vals = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in a.files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("yrt::(anonymous namespace)::", "").replace("void ", "")
        k = re.sub(r"\(.*", "", k)
        if a.match not in k:
            continue
        vals[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for (k, c) in sorted(vals):
    print(f"{k:45s} {c:28s} {vals[(k, c)] / len(disp[(k, c)]):16.4e}")
