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


def wcase(name, M, N, Kc, taps, dil, dtype, iters, T=1024):
    """Weight gradient dW[n, k, tap] = sum_m dY[m, n] X[src(m, tap), k]."""
    dev = torch.device("cuda")
    B = M // T
    dy = torch.randn(M, N, device=dev)
    x = torch.randn(M, Kc, device=dev)
    dw = torch.empty(N, Kc, taps, device=dev)
    fn = lambda: K.wgrad(dy, N, x, Kc, B, T, T, N, Kc, taps, dil, -(taps // 2) * dil,  # noqa
                         _lib.PAD_ZERO, dw, Kc * taps, taps, 1, dtype=dtype)
    sec = timeit(fn, iters)
    flops = 2.0 * M * N * Kc * taps
    return dict(case="wgrad " + name, dtype="bf16" if dtype == _lib.DT_BF16 else "f32", M=M, N=N,
                K=Kc * taps, us=round(sec * 1e6, 1), tflops=round(flops / sec / 1e12, 1))


def ccase(M, N, iters):
    dev = torch.device("cuda")
    y = torch.randn(M, N, device=dev)
    out = torch.empty(N, device=dev)
    sec = timeit(lambda: K.colsum(y, N, M, N, out), iters)
    return dict(case="colsum", M=M, N=N, us=round(sec * 1e6, 1),
                gbps=round(M * N * 4 / sec / 1e9, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    _lib.load()
    M = 30 * 1024
    rows = []
    for mode in ("reg", "glds2", "glds3"):
        K.BF16_ACT.update(on=mode != "reg", stages=int(mode[-1]) if mode != "reg" else 3,
                          min_reuse=1)
        for r in (case("gate_gemm(conv3+cond)", M, 512, [(256, 3, 2), (256, 1, 1)],
                       _lib.DT_BF16, args.iters, epi=_lib.EPI_GATE),
                  case("linear 256->512", M, 512, [(256, 1, 1)], _lib.DT_BF16, args.iters),
                  case("linear 512->256", M, 256, [(512, 1, 1)], _lib.DT_BF16, args.iters),
                  case("linear 1024->1024", M, 1024, [(1024, 1, 1)], _lib.DT_BF16, args.iters)):
            r["path"] = mode
            rows.append(r)
            print(json.dumps(r), flush=True)
    K.BF16_ACT.update(on=True, stages=3, min_reuse=2)
    x = torch.randn(M, 256, device="cuda")
    sec = timeit(lambda: K.cast_bf16(x, 256, 256, M), args.iters)
    print(json.dumps(dict(case="cast_bf16 30720x256", us=round(sec * 1e6, 1),
                          gbps=round(M * 256 * 6 / sec / 1e9, 1))), flush=True)
    rows = []
    rows += [
        wcase("gate conv3 256->512", M, 512, 256, 3, 2, _lib.DT_BF16, args.iters),
        wcase("linear 256->256", M, 256, 256, 1, 1, _lib.DT_BF16, args.iters),
        wcase("linear 1024->1024", M, 1024, 1024, 1, 1, _lib.DT_BF16, args.iters),
        wcase("conv7 2048->1024", M, 1024, 2048, 7, 1, _lib.DT_BF16, args.iters),
        ccase(M, 512, args.iters),
        ccase(M, 256, args.iters),
    ]
    for r in rows:
        print(json.dumps(r), flush=True)
    _ = Ly


if __name__ == "__main__":
    main()
