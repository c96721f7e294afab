"""Per-dispatch HBM bytes of the gate GEMM from rocprofv3 --pmc CSVs (dev tool).
gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE (KB) reports half the bytes of
16-B-per-lane streaming reads -> x2; WRITE_SIZE (KB) is exact for 16-B stores and
uncalibrated for the 4-B epilogue stores this kernel issues (reported as measured).
usage: python tools/pmc_summary.py FETCH_CSV WRITE_CSV OUT_JSON [KERNEL_SUBSTRING]"""
import csv
import json
import statistics
import sys


MATCH = sys.argv[4] if len(sys.argv) > 4 else "conv_gemm_b16_kernel"


def per_dispatch(path, counter):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if MATCH in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.setdefault(r.get("Dispatch_Id", len(vals)), 0.0)
                vals[r.get("Dispatch_Id", len(vals))] += float(r["Counter_Value"])
    return list(vals.values())


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
# the gate GEMM is the largest conv_gemm dispatch of the run (the pack/warm-up launches of
# other shapes read far less): keep dispatches within 50 % of the maximum
fk = [v for v in fetch if v > 0.5 * max(fetch)]
wk = [v for v in write if v > 0.5 * max(write)]
out = dict(kernel=f"{MATCH} (mgc DiffNet gate GEMM, M=30720 N=512 K=1024)",
           dispatches=len(fk), fetch_kb_median=statistics.median(fk),
           write_kb_median=statistics.median(wk),
           hbm_read_bytes_per_launch=2 * 1024 * statistics.median(fk),
           hbm_write_bytes_per_launch=1024 * statistics.median(wk))
out["hbm_bytes_per_launch"] = out["hbm_read_bytes_per_launch"] + out["hbm_write_bytes_per_launch"]
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
