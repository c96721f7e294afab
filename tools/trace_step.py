"""Timeline of one replayed training step from a rocprofv3 kernel trace (dev tool): per
hardware queue (one per branch stream) the span, busy time and largest kernels of the step
between the last two Adam launches.   python tools/trace_step.py TRACE_CSV [step_from_end]"""
import collections
import csv
import re
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                     r["Kernel_Name"]))
rows.sort()
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
adam = [i for i, r in enumerate(rows) if "adam" in r[3]]
a, b = adam[-1 - k], adam[-k]
step = rows[a + 1:b + 1]
t0 = rows[a][1]
print(f"step span {(rows[b][1] - t0) / 1e3:.1f} us, {len(step)} kernels")


def short(n):
    m = re.search(r"(\w+_kernel)\w*(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


byq = collections.defaultdict(list)
for s, e, q, n in step:
    byq[q].append((s, e, n))
for q, ks in sorted(byq.items()):
    busy = 0
    last = 0
    for s, e, _ in sorted(ks):  # union of intervals
        s2 = max(s, last)
        if e > s2:
            busy += e - s2
        last = max(last, e)
    agg = collections.Counter()
    for s, e, n in ks:
        agg[short(n)] += e - s
    top = ", ".join(f"{n} {v / 1e3:.0f}" for n, v in agg.most_common(6))
    print(f"queue {q}: {len(ks)} kernels, [{(min(s for s, _, _ in ks) - t0) / 1e3:.0f}, "
          f"{(max(e for _, e, _ in ks) - t0) / 1e3:.0f}] us, busy {busy / 1e3:.0f} us | {top}")
