"""Timeline of one replayed training step from a rocprofv3 kernel trace (dev tool).

Takes the window between the last two masked-L1 launches (one step), then prints per
hardware queue its first/last kernel and busy time, and a coarse timeline in 1 ms bins:
for each bin, the busy fraction of each queue and the top kernel by time, so phases
where only latency-bound recurrences run (idle CUs) are visible.
  python3 tools/step_timeline.py TRACE_CSV
"""
import collections
import csv
import sys


def main(path, binus=1000.0):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                 .split("(")[0][:28], r["Queue_Id"]) for r in rows)
    loss = [k for k in ks if "masked_l1" in k[2]]
    # the fused schedule launches one masked-L1 per branch: steps start where a gap of
    # more than 1 ms precedes a masked-L1 cluster; take the window between the last two
    starts = [loss[0][0]] + [b[0] for a, b in zip(loss, loss[1:]) if b[0] - a[0] > 5_000_000]
    adam = [k for k in ks if k[2].startswith("adam_kernel")]
    t1 = adam[-1][1]
    t0 = max(a[1] for a in adam if a[1] < t1 - 1_000_000)
    win = [k for k in ks if t0 <= k[0] < t1]
    wall = (t1 - t0) / 1e3
    print(f"step window {wall:.0f} us (adam to adam), {len(win)} kernels")
    qs = collections.defaultdict(list)
    for k in win:
        qs[k[3]].append(k)
    for q, v in sorted(qs.items()):
        busy = sum(e - s for s, e, *_ in v) / 1e3
        print(f"  queue {q}: {len(v):4d} kernels, first {(v[0][0] - t0) / 1e3:7.0f} last "
              f"{(max(e for _, e, *_ in v) - t0) / 1e3:7.0f} busy {busy:7.0f} us")
    nb = int(wall // binus) + 1
    occ = [collections.defaultdict(float) for _ in range(nb)]
    top = [collections.defaultdict(float) for _ in range(nb)]
    for s, e, n, q in win:
        a, b = (s - t0) / 1e3, (e - t0) / 1e3
        i = int(a // binus)
        while a < b and i < nb:
            hi = min(b, (i + 1) * binus)
            occ[i][q] += hi - a
            top[i][n] += hi - a
            a, i = hi, i + 1
    qn = sorted(qs)
    print("  bin(ms) " + " ".join(f"q{q:>3s}" for q in qn) + "  top kernels")
    for i in range(nb):
        t = sorted(top[i].items(), key=lambda kv: -kv[1])[:3]
        print(f"  {i:6d}  " + " ".join(f"{occ[i][q] / binus:4.2f}" for q in qn) + "  " +
              ", ".join(f"{n}:{v / binus:.2f}" for n, v in t))


if __name__ == "__main__":
    main(sys.argv[1])
