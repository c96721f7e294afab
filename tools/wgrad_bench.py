"""Weight-gradient GEMM microbenchmark (dev tool, not a test).

Times K.wgrad (kernel + split reduce) on the training step's weight-gradient shapes
(M = 30 x 1024 frames) with HIP events on the launch stream, bf16-operand and fp32-operand
variants.  python tools/wgrad_bench.py [--iters 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib, kernels as K  # noqa: E402

SHAPES = [  # name, N, K, taps, dil, ldy, ldx
    ("mgc dilated conv  N512 K256 x3", 512, 256, 3, 4, 512, 256),
    ("mgc w_o residual  N256 K256", 256, 256, 1, 1, 256, 256),
    ("mgc conditioner   N10240 K256", 10240, 256, 1, 1, 10240, 256),
    ("mgc w_o skip      N256 K5120", 256, 5120, 1, 1, 256, 5120),
    ("bap dilated conv  N256 K128 x3", 256, 128, 3, 2, 256, 128),
    ("enc conv k7       N256 K256 x7", 256, 256, 7, 1, 256, 256),
    ("lstm W_ih         N1024 K256", 1024, 256, 1, 1, 1024, 256),
]


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
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, T = 30, 1024
    M = B * T
    for name, N, Kc, taps, dil, ldy, ldx in SHAPES:
        flops = 2.0 * M * N * Kc * taps
        dst = torch.zeros(N, Kc, taps, device=dev)
        for dt in (torch.bfloat16, torch.float32):
            dy = torch.randn(M, ldy, device=dev).to(dt)
            x = torch.randn(M, ldx, device=dev).to(dt)
            f = lambda: K.wgrad(dy, ldy, x, ldx, B, T, T, N, Kc, taps, dil, -dil if taps > 1 else 0,  # noqa: E731
                                _lib.PAD_ZERO, dst, Kc * taps, taps, 1, accum=True)
            t = timeit(f, a.iters)
            print(f"{name:34s} {str(dt)[6:]:9s} {t * 1e6:8.1f} us  {flops / t / 1e12:7.1f} TFLOP/s",
                  flush=True)


if __name__ == "__main__":
    main()
