"""Graph-replayed SeparateF0 (MODEL=main: the bench's main line) training steps for a
kernel trace (dev tool):
   rocprofv3 --kernel-trace --output-format csv -d DIR -o sf0 -- python3 tools/sf0_trace.py
then  python3 tools/sf0_trace.py --show DIR/sf0_kernel_trace.csv  prints, for the step between
the last two Adam launches, every queue's kernels in start order (ms from the step start,
duration, gap before) so the critical chain and the idle gaps between its launches show."""
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def show(path, min_us=15.0):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            m = re.search(r"(\w+_kernel)\w*(<[^>]*>)?", n)
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                         (m.group(1) + (m.group(2) or "")) if m else n[:40]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if r[3].startswith("adam_kernel")]
    a, b = adam[-2], adam[-1]
    step = rows[a + 1:b + 1]
    t0 = rows[a][1]
    print(f"step {(rows[b][1] - t0) / 1e6:.2f} ms, {len(step)} kernels")
    qs = {}
    for s, e, q, n in step:
        qs.setdefault(q, []).append((s, e, n))
    for q, ks in qs.items():
        busy = sum(e - s for s, e, _ in ks)
        print(f"\nqueue {q}: {len(ks)} kernels, {busy / 1e6:.2f} ms summed, "
              f"{(ks[-1][1] - ks[0][0]) / 1e6:.2f} ms span")
        last, small, small_us = ks[0][0], 0, 0.0
        for s, e, n in ks:
            d = (e - s) / 1e3
            if d < min_us:
                small += 1
                small_us += d
                last = max(last, e)
                continue
            gap = (s - last) / 1e3
            if small:
                print(f"{'':10s} ({small} short launches, {small_us:.0f} us)")
                small, small_us = 0, 0.0
            print(f"{(s - t0) / 1e6:9.3f} {d:8.1f} us gap {gap:7.1f}  {n}")
            last = max(last, e)


def run(steps=6):
    import torch
    from ensemble_svs_with_interactions_amd import configs, data
    from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep
    dev = torch.device("cuda:0")
    if os.environ.get("MODEL") == "main":  # the bench's main line (multi-track diffusion)
        torch.manual_seed(20250321)
        model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    else:
        torch.manual_seed(20250324)
        model = configs.instantiate(configs.multitrack_separate_f0(num_speakers=4)).to(dev)
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    P = int(os.environ.get("P", 30))
    T = int(os.environ.get("T", 1024))
    b = data.synthetic_batch(P, T, 1000 if os.environ.get("MODEL") == "main" else 4000)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    step = GraphedTrainStep(model, opt, g("x_main"), g("x_sub"), g("y_main"), g("spk_main"),
                            g("spk_sub"), b["lengths"].tolist(), warmup=1).step
    import time
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"{(time.time() - t) / steps * 1e3:.2f} ms per step")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--show":
        show(sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 15.0)
    else:
        run()
