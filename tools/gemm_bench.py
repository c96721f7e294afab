"""GEMM engine microbenchmark on the GPU (dev tool, not a test).

Times ensvs_conv_gemm on the shapes the training step runs most (HIP events on
the launch stream) next to torch's bf16 matmul (hipBLASLt) on the same M, N, K
as a library anchor.  Usage: python tools/gemm_bench.py [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib, kernels as K  # noqa: E402
from ensemble_svs_with_interactions_amd import layers as Ly  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(iters):
        fn()
    e.record(st)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 1e3 / iters


def case(name, M, N, segs_spec, dtype, iters, epi=_lib.EPI_PLAIN, T=1024):
    """segs_spec: list of (K, taps, dil)."""
    dev = torch.device("cuda")
    B = M // T
    pb = K.PackedBuffer(dtype)
    segs, xs, Ktot = [], [], 0
    for (Kc, taps, dil) in segs_spec:
        w = torch.randn(N, Kc, taps, device=dev) * 0.02
        ref = pb.add(w, N, Kc, taps, Kc * taps, taps, 1)
        x = torch.randn(M, Kc, device=dev)
        xs.append((x, w))
        segs.append(K.Seg(x, Kc, Kc, ref, T, taps=taps, dil=dil, shift0=-(taps // 2) * dil))
        Ktot += Kc * taps
    pb.finalize(dev)
    pb.repack()
    extra = {}
    if epi == _lib.EPI_GATE:
        C = N // 2
        Y = torch.empty(M, C, device=dev)
        gf = torch.empty(M, N, device=dev)
        extra = dict(epi=epi, aux0=gf, ld0=N, C=C)
        ldy = C
    else:
        Y = torch.empty(M, N, device=dev)
        ldy = N
    fn = lambda: K.gemm(segs, B, T, N, pb, Y, ldy, **extra)  # noqa: E731
    sec = timeit(fn, iters)
    flops = 2.0 * M * N * Ktot
    a = torch.randn(M, Ktot, device=dev, dtype=torch.bfloat16)
    b = torch.randn(Ktot, N, device=dev, dtype=torch.bfloat16)
    ref_sec = timeit(lambda: torch.matmul(a, b), iters)
    return dict(case=name, dtype="bf16" if dtype == _lib.DT_BF16 else "f32", M=M, N=N, K=Ktot,
                us=round(sec * 1e6, 1), tflops=round(flops / sec / 1e12, 1),
                torch_bf16_us=round(ref_sec * 1e6, 1),
                torch_bf16_tflops=round(flops / ref_sec / 1e12, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    _lib.load()
    M = 30 * 1024
    rows = [
        case("gate_gemm(conv3+cond)", M, 512, [(256, 3, 2), (256, 1, 1)], _lib.DT_BF16, args.iters,
             epi=_lib.EPI_GATE),
        case("linear 256->512", M, 512, [(256, 1, 1)], _lib.DT_BF16, args.iters),
        case("linear 1024->1024", M, 1024, [(1024, 1, 1)], _lib.DT_BF16, args.iters),
        case("linear 2048->2048", M, 2048, [(2048, 1, 1)], _lib.DT_BF16, args.iters),
        case("conv7 2048->1024", M, 1024, [(2048, 7, 1)], _lib.DT_BF16, args.iters),
        case("linear 1024->1024 f32", M, 1024, [(1024, 1, 1)], _lib.DT_F32, args.iters),
    ]
    for r in rows:
        print(json.dumps(r), flush=True)
    _ = Ly


if __name__ == "__main__":
    main()
