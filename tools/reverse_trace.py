"""Kernel time vs launch gaps of the last captured reverse diffusion in a rocprofv3 kernel
trace of tools/synth_probe.py (dev tool): the window spans the last K p_sample launches
(one DiffNet pass + p_sample per diffusion step, replayed from the graph on one stream).
  rocprofv3 --kernel-trace --output-format csv -d OUT -o syn -- python3 tools/synth_probe.py 1
  python tools/reverse_trace.py OUT/syn_kernel_trace.csv [K]
"""
import collections
import csv
import sys


def main(path, K=100):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
                 .split("(")[0], f'{r.get("Grid_Size_X", "?")}x{r.get("Grid_Size_Y", "?")}') for r in rows)
    ps = [i for i, k in enumerate(ks) if k[2].startswith("p_sample")]
    if len(ps) < K + 1:
        print("fewer than K + 1 p_sample launches")
        return
    lo, hi = ps[-K - 1] + 1, ps[-1] + 1
    win = ks[lo:hi]
    wall = (win[-1][1] - win[0][0]) / 1e3
    busy = sum(e - s for s, e, _, _ in win) / 1e3
    per = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n, g in win:
        per[(n, g)][0] += (e - s) / 1e3
        per[(n, g)][1] += 1
    print(f"last {K} diffusion steps: {wall / 1e3:.2f} ms wall, kernels {busy / 1e3:.2f} ms "
          f"({busy / wall * 100:.0f} %), {len(win)} launches, mean gap "
          f"{(wall - busy) / max(1, len(win) - 1):.2f} us")
    for (n, g), (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:20]:
        print(f"{t / 1e3:8.2f} ms {c:6d}x {t / c:7.2f} us  grid {g:>8}  {n[:70]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 100)
