"""Median per-dispatch PMC values per kernel from rocprofv3 --pmc csv files (dev tool).
Usage: python3 tools/pmc_table.py DIR [DIR...] [--match SUBSTR]"""
import collections
import csv
import glob
import statistics
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
if match in args:
    args.remove(match)
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args:
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match not in k:
                continue
            vals[k[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print("==", k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {statistics.median(v):16.0f}  (n={len(v)})")
