"""Weight-gradient split-count sweep (dev tool, not a test).

Times K.wgrad (kernel + split reduce, HIP events, back-to-back launches) on the bf16
weight-gradient shapes of the training step's census (M = 30 x 1024 frames) for a range of
row-split counts, against the split count kernels.wgrad picks.
python tools/wgrad_split_sweep.py [--iters 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib, kernels as K  # noqa: E402

SHAPES = [  # N, K, taps, dil, launches per step (census)
    (256, 256, 1, 1, 25),
    (256, 128, 1, 1, 12),
    (256, 64, 1, 1, 12),
    (256, 128, 3, 2, 10),
    (128, 128, 1, 1, 9),
    (512, 256, 3, 4, 20),
    (512, 128, 1, 1, 6),
    (1024, 256, 1, 1, 4),
]
SPLITS = [8, 16, 24, 32, 48, 64, 96, 128, 192, 256]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--splits", type=int, nargs="*", default=SPLITS)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, T = 30, 1024
    M = B * T
    for N, Kc, taps, dil, per_step in SHAPES:
        dst = torch.zeros(N, Kc, taps, device=dev)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        x = torch.randn(M, Kc, device=dev).to(torch.bfloat16)

        def run(splits):
            return lambda: K.wgrad(dy, N, x, Kc, B, T, T, N, Kc, taps, dil,
                                   -dil if taps > 1 else 0, _lib.PAD_ZERO, dst, Kc * taps, taps,
                                   1, splits=splits)
        ref = timeit(run(None), a.iters)
        row = [f"N{N} K{Kc}x{taps}: default {ref * 1e6:6.1f} us |"]
        best = (ref, None)
        for sp in a.splits:
            t = timeit(run(sp), a.iters)
            row.append(f"{sp}:{t * 1e6:.1f}")
            if t < best[0]:
                best = (t, sp)
        row.append(f"| best {best[1]} {best[0] * 1e6:.1f} us (x{per_step}/step)")
        print(" ".join(row), flush=True)


if __name__ == "__main__":
    main()
