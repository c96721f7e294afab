"""Sum rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over the dispatches between the two marker
kernels of tools/step_pmc.py and divide by its step count: HBM bytes per training step.
gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of 16-B-per-
lane streaming reads (x2); WRITE_SIZE is exact for 16-B stores (narrower accesses are
uncalibrated, so the figure is an estimate for the few kernels that issue them).
usage: python tools/step_pmc_sum.py FETCH_CSV WRITE_CSV OUT_JSON [STEPS]"""
import csv
import json
import re
import sys

STEPS = int(sys.argv[4]) if len(sys.argv) > 4 else 4


def between_markers(path, counter):
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            e = rows.setdefault(d, [r["Kernel_Name"], 0.0])
            e[1] += float(r["Counter_Value"])
    ids = sorted(rows)
    marks = [d for d in ids if "spin" in rows[d][0].lower() or "sleep" in rows[d][0].lower()]
    assert len(marks) >= 2, f"marker kernels not found ({len(marks)})"
    a, b = marks[-2], marks[-1]
    inside = [rows[d] for d in ids if a < d < b]
    per_kernel = {}
    for name, v in inside:
        m = re.search(r"(\w+_kernel\w*|ensvs_\w+|\w+Kernel\w*)", name)
        k = m.group(1) if m else name[:60]
        per_kernel[k] = per_kernel.get(k, 0.0) + v
    return sum(v for _, v in inside), len(inside), per_kernel


fk, nf, fkern = between_markers(sys.argv[1], "FETCH_SIZE")
wk, nw, wkern = between_markers(sys.argv[2], "WRITE_SIZE")
out = {"steps": STEPS, "dispatches_per_step": nf / STEPS,
       "hbm_read_bytes_per_step": 2 * 1024 * fk / STEPS,
       "hbm_write_bytes_per_step": 1024 * wk / STEPS}
out["hbm_bytes_per_step"] = out["hbm_read_bytes_per_step"] + out["hbm_write_bytes_per_step"]
top = sorted(fkern, key=lambda k: -(2 * fkern[k] + wkern.get(k, 0.0)))[:15]
out["top_kernels_mb_per_step"] = {k: round((2 * fkern[k] + wkern.get(k, 0.0)) * 1024 / STEPS
                                           / 1e6, 1) for k in top}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
