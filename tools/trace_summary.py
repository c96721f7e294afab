"""Summarise a rocprofv3 kernel trace of bench.py (dev tool).

Finds the last training step (the gap-separated cluster of kernels before the
gate-GEMM timing loop is hard to detect, so the caller passes the number of steps
and we take the window between the last two masked-L1 launches), and prints per
queue busy time and the top kernels, so the critical path of the concurrent
branch schedule is visible.

  python tools/trace_summary.py gpurun_out/prof/r_kernel_trace.csv
"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
           r.get("Queue_Id", "?")) for r in rows]
    ks.sort()
    loss = [k for k in ks if "masked_l1_kernel" in k[2]]
    if len(loss) < 2:
        print("need >= 2 steps")
        return
    t0, t1 = loss[-2][0], loss[-1][0]
    win = [k for k in ks if t0 <= k[0] < t1]
    wall = (t1 - t0) / 1e3
    print(f"one step (loss to loss): {wall:.0f} us, {len(win)} kernels")
    per_q = collections.defaultdict(float)
    per_name = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n, q in win:
        per_q[q] += (e - s) / 1e3
        short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        per_name[short][0] += (e - s) / 1e3
        per_name[short][1] += 1
    for q, b in sorted(per_q.items()):
        print(f"  queue {q}: busy {b:8.0f} us ({b / wall * 100:5.1f}% of wall)")
    # union of busy intervals = time at least one kernel runs
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"  GPU busy (any kernel): {busy / 1e3:.0f} us ({busy / 1e3 / wall * 100:.1f}%)")
    for n, (t, c) in sorted(per_name.items(), key=lambda kv: -kv[1][0])[:30]:
        print(f"  {t:8.0f} us {c:5d}x  {n[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])
