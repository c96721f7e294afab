"""Per-branch kernel breakdown of one training step (dev tool).

Run mode: the step's branches (lf0 / mgc / bap / vuv, forward then backward) run
serially, each bracketed by a device synchronize and a 3 ms host sleep, so the kernel
trace shows one gap-separated cluster per branch region:
  rocprofv3 --kernel-trace --output-format csv -d OUT -o bk -- python3 tools/branch_kernels.py
Analysis mode:
  python tools/branch_kernels.py OUT/bk_kernel_trace.csv
prints, for the last step, each cluster's summed kernel time and its top kernels with
grid sizes, so the critical branch's time budget is visible.
"""
import collections
import csv
import os
import sys
import time

GAP_NS = 2_000_000


def analyse(path, top=25):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""),
                 r.get("Grid_Size", "?"), r.get("Workgroup_Size", "?")) for r in rows)
    clusters, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - max(c[1] for c in cur[-4:]) > GAP_NS:
            clusters.append(cur)
            cur = [k]
        else:
            cur.append(k)
    clusters.append(cur)
    # the last step: the 8 branch regions before the trailing optimizer cluster(s)
    big = [c for c in clusters if len(c) > 3]
    print(f"{len(clusters)} clusters; last 12 (kernels, span us, summed kernel us):")
    for c in clusters[-12:]:
        span = (c[-1][1] - c[0][0]) / 1e3
        busy = sum(e - s for s, e, *_ in c) / 1e3
        print(f"  {len(c):5d} {span:9.0f} {busy:9.0f}   first {c[0][2][:60]}")
    for idx, c in enumerate(big[-10:]):
        busy = sum(e - s for s, e, *_ in c) / 1e3
        agg = collections.defaultdict(lambda: [0.0, 0])
        for s, e, n, g, w in c:
            key = f"{n.split('(')[0][:60]} grid={g} wg={w}"
            agg[key][0] += (e - s) / 1e3
            agg[key][1] += 1
        print(f"\n=== cluster {idx - 10}: {len(c)} kernels, {busy:.0f} us kernel time, "
              f"span {(c[-1][1] - c[0][0]) / 1e3:.0f} us")
        for key, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
            print(f"  {t:8.0f} us {n:4d}x {t / n:8.1f}  {key}")


def run(P=30, T=1024, steps=2):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ensemble_svs_with_interactions_amd import configs, data, engine
    from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step

    class _gap:
        def __init__(self, ctx):
            self.ctx = ctx

        def __enter__(self):
            torch.cuda.synchronize()
            time.sleep(0.003)
            return self.ctx.__enter__()

        def __exit__(self, *exc):
            r = self.ctx.__exit__(*exc)
            torch.cuda.synchronize()
            time.sleep(0.003)
            return r

    orig = engine.Branches.on
    engine.Branches.on = lambda self, i: _gap(orig(self, i))
    engine.set_concurrency(False)
    engine.set_gemm_precision("bf16")
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    opt = FusedAdam(model)
    b = data.synthetic_batch(P, T, 3)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    args = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
            b["lengths"].tolist())
    for _ in range(steps):
        train_step(model, opt, *args)
        torch.cuda.synchronize()
        time.sleep(0.003)
    print("done", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        analyse(sys.argv[1])
    else:
        run()
