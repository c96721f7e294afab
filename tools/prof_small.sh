set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_small -o run -- python3 tools/small_gemm_probe.py > gpurun_out/prof_small.log 2>&1
f=$(find gpurun_out/prof_small -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r["Kernel_Name"][:40], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r.get("Grid_Size", ""), r.get("Workgroup_Size","")) for r in rows]
# print consecutive groups of identical kernel names with avg duration
out = []
cur = None
for name, d, g, w in seq:
    key = (name, g, w)
    if cur and cur[0] == key:
        cur[1].append(d)
    else:
        if cur: out.append(cur)
        cur = [key, [d]]
out.append(cur)
for (name, g, w), ds in out:
    if len(ds) >= 5:
        print(f"{name:40s} grid={g:>8s} wg={w:>5s} n={len(ds):3d} avg={sum(ds)/len(ds)/1e3:7.2f} us min={min(ds)/1e3:7.2f}")
PY
