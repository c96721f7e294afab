"""The four-phase 256 x 256 GEMM kernel (ensvs_set_p8) against the engine's 128 x 128 kernel
and, as a library anchor, torch's bf16 matmul (hipBLASLt, bf16 output, no epilogue) on the same
M, N, K of the step's large shapes (dev tool): HIP-event time per launch and a bitwise check
against the 128 x 128 kernel.  (Round 6 until the hipBLASLt route was removed: a "blas" arm,
hipBLASLt with fp32 output and bias: profiles/r6_p8_bench.txt.)
   python tools/p8_bench.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L, kernels as K  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda")
T = 1024


def timeit(fn, iters=ITERS):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def case(name, M, N, spec, epi=L.EPI_PLAIN, bias=True, accum=False, relu_bf16=False):
    """spec: list of (K, taps, dil) bf16 segments."""
    g = torch.Generator(device=dev).manual_seed(1)
    pb = K.PackedBuffer(L.DT_BF16)
    segs, Kt = [], 0
    for (Kc, taps, dil) in spec:
        w = torch.randn(N, Kc, taps, device=dev, generator=g) * (1.0 / (Kc * taps) ** 0.5)
        ref = pb.add(w, N, Kc, taps, Kc * taps, taps, 1)
        x = torch.randn(M, Kc, device=dev, generator=g).to(torch.bfloat16)
        segs.append(K.Seg(x, Kc, Kc, ref, T, taps=taps, dil=dil, shift0=-(taps // 2) * dil))
        Kt += Kc * taps
    pb.finalize(dev)
    pb.repack()
    bv = torch.randn(N, device=dev, generator=g) if bias else None
    if epi == L.EPI_GATE:
        C = N // 2
        outs = [torch.empty(M, C, device=dev), torch.empty(M, N, device=dev, dtype=torch.bfloat16),
                torch.empty(M, C, device=dev, dtype=torch.bfloat16)]

        def fn():
            K.gemm(segs, M // T, T, N, pb, outs[0], C, epi=epi, aux0=outs[1], ld0=N, C=C,
                   ybf=outs[2], ybf_ld=C, keep_y=False, bias=bv)
    elif epi == L.EPI_RELU_MASK:
        outs = [torch.zeros(M, N, device=dev)]
        mask = torch.randn(M, N, device=dev, generator=g)

        def fn():
            K.gemm(segs, M // T, T, N, pb, outs[0], N, epi=epi, aux1=mask, ld1=N)
    elif relu_bf16:
        outs = [torch.zeros(M, N, device=dev), torch.zeros(M, N, device=dev, dtype=torch.bfloat16)]

        def fn():
            K.gemm(segs, M // T, T, N, pb, outs[0], N, bias=bv, relu=True, ybf=outs[1], ybf_ld=N)
    else:
        outs = [torch.zeros(M, N, device=dev)]

        def fn():
            K.gemm(segs, M // T, T, N, pb, outs[0], N, bias=bv, accum=accum)
    res = dict(case=name, M=M, N=N, K=Kt)
    flops = 2.0 * M * N * Kt
    ref = None
    for tag, p8 in (("eng128", 0), ("p8", 2), ("p8stag", 6), ("default", 7)):
        _lib_call("ensvs_set_p8", p8)
        for o in outs:
            o.zero_()
        fn()
        torch.cuda.synchronize()
        got = [o.clone() for o in outs]
        if ref is None:
            ref = got
        else:
            d = max(float((a.float() - b.float()).abs().max()) for a, b in zip(ref, got))
            res[f"{tag}_maxdiff"] = d
        us = timeit(fn)
        res[f"{tag}_us"] = round(us, 1)
        res[f"{tag}_tflops"] = round(flops / us / 1e6, 1)
    _lib_call("ensvs_set_p8", 6)
    a = torch.randn(M, Kt, device=dev, dtype=torch.bfloat16)
    b = torch.randn(Kt, N, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: torch.matmul(a, b))
    res["torch_us"] = round(us, 1)
    print(json.dumps(res), flush=True)


def _lib_call(name, *args):
    L.call(name, *args)


def none_case(name, M, N, spec):
    """The K loop alone (EPI_NONE: no output) on the 128 x 128 and four-phase kernels."""
    pb = K.PackedBuffer(L.DT_BF16)
    segs = []
    for (Kc, taps, dil) in spec:
        ref = pb.add(torch.randn(N, Kc, taps, device=dev) * 0.03, N, Kc, taps, Kc * taps, taps, 1)
        segs.append(K.Seg(torch.randn(M, Kc, device=dev).to(torch.bfloat16), Kc, Kc, ref, T,
                          taps=taps, dil=dil, shift0=-(taps // 2) * dil))
    pb.finalize(dev)
    pb.repack()
    Y = torch.empty(M, N, device=dev)
    res = dict(case=name + " (K loop only)", M=M, N=N, K=sum(k * t for k, t, _ in spec))
    for tag, p8 in (("eng128", 0), ("p8", 2), ("p8stag", 6), ("p8_noload", 10),
                    ("p8stag_noload", 14), ("p8stag_nomfma", 22)):
        _lib_call("ensvs_set_p8", p8)
        res[f"{tag}_us"] = round(timeit(lambda: K.gemm(segs, M // T, T, N, pb, Y, N,
                                                       epi=L.EPI_NONE)), 1)
    _lib_call("ensvs_set_p8", 6)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    L.load()
    M = 30 * 1024
    case("diffnet gate mgc", M, 512, [(256, 3, 4), (256, 1, 1)], epi=L.EPI_GATE)
    case("enc l0 proj 512->4096", M, 4096, [(512, 1, 1)])
    case("enc l1/2 proj 1024->4096", M, 4096, [(1024, 1, 1)])
    case("enc dgrad 2x2048->1024", M, 1024, [(2048, 1, 1), (2048, 1, 1)], bias=False)
    case("dec proj 512->2048", M, 2048, [(512, 1, 1)])
    case("dec dgrad 2x1024->512", M, 512, [(1024, 1, 1), (1024, 1, 1)], bias=False)
    case("mgc lstm proj 512->1024", M, 1024, [(512, 1, 1)])
    case("mgc enc conv k7 512->512", M, 512, [(512, 7, 1)])
    case("diffnet res 256->512", M, 512, [(256, 1, 1)])
    case("ff relu + bf16 copy 512->1024 (generic)", M, 1024, [(512, 1, 1)], relu_bf16=True)
    case("conv relu + bf16 copy k5 512->512 (generic)", M, 512, [(512, 5, 1)], relu_bf16=True)
    case("relu-mask dgrad 1024->1024 (generic)", M, 1024, [(1024, 1, 1)], epi=L.EPI_RELU_MASK,
         bias=False)
    none_case("enc l0 proj 512->4096", M, 4096, [(512, 1, 1)])
    none_case("enc dgrad 2x2048->1024", M, 1024, [(2048, 1, 1), (2048, 1, 1)])
