"""The four-phase 256 x 256 kernel against the 128 x 128 kernel on the main step's short-K
N = 512 launches at 30 x 1024 frames (dev tool): HIP-event time per launch, bitwise check.
   python tools/p8_shortk_bench.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L, kernels as K  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda")
B, T = 30, 1024
M = B * T


def timeit(fn, iters=ITERS):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def run_case(name, fn, outs, flops):
    res = dict(case=name)
    ref = None
    for tag, mode in (("p8", 6), ("eng128", 4)):
        L.call("ensvs_set_p8", mode)
        for o in outs:
            o.zero_()
        fn()
        torch.cuda.synchronize()
        got = [o.clone() for o in outs]
        if ref is None:
            ref = got
        else:
            res[f"{tag}_maxdiff"] = max(float((a.float() - b.float()).abs().max())
                                        for a, b in zip(ref, got))
        us = timeit(fn)
        res[f"{tag}_us"] = round(us, 1)
        res[f"{tag}_tflops"] = round(flops / us / 1e6, 1)
    L.call("ensvs_set_p8", 6)
    print(json.dumps(res), flush=True)


def main():
    L.load()
    for Kc in (128, 256, 512):
        N = 512
        pb = K.PackedBuffer(L.DT_BF16)
        r = pb.add(torch.randn(N, Kc, 1, device=dev) * 0.05, N, Kc, 1, Kc, 1, 1)
        pb.finalize(dev)
        pb.repack()
        x = torch.randn(M, Kc, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev)
        bias = torch.randn(N, device=dev)
        run_case(f"plain N = 512 K = {Kc} (+ bias)", lambda: K.gemm(
            [K.Seg(x, Kc, Kc, r, T)], B, T, N, pb, y, N, bias=bias), [y], 2.0 * M * N * Kc)
        if Kc == 512:
            mask = torch.randn(M, N, device=dev)
            run_case("relu-mask N = 512 K = 512", lambda: K.gemm(
                [K.Seg(x, Kc, Kc, r, T)], B, T, N, pb, y, N, epi=L.EPI_RELU_MASK, aux1=mask,
                ld1=N), [y], 2.0 * M * N * Kc)


if __name__ == "__main__":
    main()
