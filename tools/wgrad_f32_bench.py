"""fp32-operand weight gradients of the training step (production bf16 staging) timed with
HIP events: the census's 'wgrad ... f' shapes at M = 30 x 1024 frames (dev tool).
    python tools/wgrad_f32_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L, kernels as K  # noqa: E402

SHAPES = [(256, 64, 1), (256, 128, 1), (256, 256, 1), (128, 128, 7), (512, 256, 1),
          (256, 256, 7), (128, 256, 7), (256, 512, 7), (512, 512, 1), (512, 128, 1)]


def main():
    dev = torch.device("cuda")
    B, T = 30, 1024
    M = B * T
    tot = 0.0
    for N, Kc, taps in SHAPES:
        x = torch.randn(M, Kc, device=dev)
        g = torch.randn(M, N, device=dev)
        dw = torch.zeros(N, Kc, taps, device=dev)
        pad = L.PAD_REFLECT if taps == 7 else L.PAD_ZERO

        def fn():
            K.wgrad(g, N, x, Kc, B, T, T, N, Kc, taps, 1, -(taps // 2), pad, dw, Kc * taps,
                    taps, 1, accum=True, dtype=L.DT_BF16)
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        tot += us
        mb = M * (N + Kc) * 4 / 1e6
        print(f"N={N:4d} K={Kc:4d}x{taps}  {us:7.1f} us  ({mb / us:5.2f} TB/s of fp32 operands)")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
