"""Gate-GEMM variants on the bench shape (dev tool): the training-step form (bf16 operands,
bf16 z only) at 2 / 3 pipeline stages, the same without the epilogue's outputs (PLAIN into
a scratch Y), and hipBLASLt's bf16 matmul on the same M, N, K as an anchor.
  python tools/gate_variants.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib, kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    _lib.load()
    dev = torch.device("cuda")
    P, T, C, E = 30, 1024, 256, 256
    M, N = P * T, 2 * C
    pb = K.PackedBuffer(_lib.DT_BF16)
    wd = torch.randn(N, C, 3, device=dev) * 0.02
    wc = torch.randn(N, E, 1, device=dev) * 0.02
    rd = pb.add(wd, N, C, 3, 3 * C, 3, 1)
    rc = pb.add(wc, N, E, 1, E, 1, 1)
    pb.finalize(dev)
    pb.repack()
    xb = torch.randn(M, C, device=dev).to(torch.bfloat16)
    cb = torch.randn(M, E, device=dev).to(torch.bfloat16)
    segs = [K.Seg(xb, C, C, rd, T, taps=3, dil=2, shift0=-2), K.Seg(cb, E, E, rc, T)]
    z = torch.empty(M, C, device=dev)
    zb = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    gf = torch.empty(M, N, device=dev)
    y = torch.empty(M, N, device=dev)
    bias = torch.zeros(N, device=dev)
    flops = 2.0 * M * N * (3 * C + E)
    for st in (2, 3):
        K.BF16_ACT["stages"] = st
        r = {}
        r["gate_train"] = timeit(lambda: K.gemm(segs, P, T, N, pb, z, C, epi=_lib.EPI_GATE,
                                                aux0=gf, ld0=N, C=C, ybf=zb, ybf_ld=C,
                                                keep_y=False, bias=bias), 50)
        r["gate_fp32z"] = timeit(lambda: K.gemm(segs, P, T, N, pb, z, C, epi=_lib.EPI_GATE,
                                                aux0=gf, ld0=N, C=C, bias=bias), 50)
        r["plain_fp32"] = timeit(lambda: K.gemm(segs, P, T, N, pb, y, N), 50)
        print(json.dumps({"stages": st, **{k: round(v * 1e6, 1) for k, v in r.items()},
                          "tflops_gate": round(flops / r["gate_train"] / 1e12, 1)}), flush=True)
    a = torch.randn(M, 3 * C + E, device=dev, dtype=torch.bfloat16)
    b = torch.randn(3 * C + E, N, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: torch.matmul(a, b), 50)
    print(json.dumps({"hipblaslt_bf16_out_us": round(t * 1e6, 1),
                      "tflops": round(flops / t / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
