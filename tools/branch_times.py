"""Per-branch device time of the concurrent training step (dev tool).

Records HIP events around each branch region (engine.BRANCH_TIMES) and prints
each branch's fwd/bwd span, alone (serial schedule) and inside the concurrent
schedule, plus the step time.  python tools/branch_times.py [--pairs 30]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step  # noqa: E402

NAMES = {0: "lf0", 1: "mgc", 2: "bap", 3: "vuv"}


def run(conc, P, T, steps=3):
    engine.set_concurrency(conc)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    opt = FusedAdam(model)
    b = data.synthetic_batch(P, T, 3)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    args = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
            b["lengths"].tolist())
    for _ in range(2):
        train_step(model, opt, *args)
    torch.cuda.synchronize()
    engine.BRANCH_TIMES = []
    t0 = time.time()
    for _ in range(steps):
        train_step(model, opt, *args)
    torch.cuda.synchronize()
    step_ms = (time.time() - t0) / steps * 1e3
    rec = engine.BRANCH_TIMES
    engine.BRANCH_TIMES = None
    n = len(rec) // steps
    last = rec[-n:]  # last step: the branch regions (+ tagged single events)
    out = {}
    regions = [r for r in last if len(r) == 3]
    t_ref = regions[0][1]
    for k, (i, s, e) in enumerate(regions):
        phase = "fwd" if k < len(regions) // 2 and len(regions) == 8 else "bwd" if len(regions) == 8 else "br"
        out[f"{NAMES[i]}.{phase}.{k}"] = (f"{s.elapsed_time(e):.2f}"
                                          f"[{t_ref.elapsed_time(s):.1f}-{t_ref.elapsed_time(e):.1f}]")
    for r in last:
        if len(r) == 2:
            out[f"{r[0]}@{len(out)}"] = f"{t_ref.elapsed_time(r[1]):.1f}"
    return step_ms, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=30)
    ap.add_argument("--frames", type=int, default=1024)
    a = ap.parse_args()
    for conc in (False, True):
        ms, out = run(conc, a.pairs, a.frames)
        print(("concurrent" if conc else "serial    "), f"step {ms:.1f} ms |",
              "  ".join(f"{k} {v}" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    main()
