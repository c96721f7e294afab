"""The main step's N = 128 GEMM launches at 30 x 1024 frames (240 tiles of 128 x 128: one
workgroup per CU) on the 128 x 128 kernel, the 64 x 64 kernel (ensvs_set_small(2)) and the
128 x 128 kernel with three LDS stages (dev tool): HIP-event time per launch and a bitwise
check.   python tools/n128_bench.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L, kernels as K  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda")
B, T, C = 30, 1024, 128
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
    return s.elapsed_time(e) / iters * 1e3  # us


def bf(*shape):
    return torch.randn(*shape, device=dev).to(torch.bfloat16)


def pack(ws):
    pb = K.PackedBuffer(L.DT_BF16)
    refs = [pb.add(w, w.shape[0], w.shape[1], w.shape[2], w.shape[1] * w.shape[2], w.shape[2], 1)
            for w in ws]
    pb.finalize(dev)
    pb.repack()
    return pb, refs


def arm(tag):
    L.call("ensvs_set_small", 2 if tag == "small64" else 1)
    K.BF16_ACT["stages"] = 3 if tag == "stages3" else 2


ARMS = ("eng128", "small64", "stages3")


def run_case(name, fn, outs, flops):
    res = dict(case=name)
    ref = None
    for tag in ARMS:
        arm(tag)
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
    arm("eng128")
    print(json.dumps(res), flush=True)


def main():
    L.load()
    x = bf(M, C)
    Y = torch.empty(M, C, device=dev)
    pb, (r7,) = pack([torch.randn(C, C, 7, device=dev) * 0.03])
    run_case("conv k7 128 -> 128 (PLAIN + bias)", lambda: K.gemm(
        [K.Seg(x, C, C, r7, T, taps=7, shift0=-3)], B, T, C, pb, Y, C,
        bias=torch.zeros(C, device=dev)), [Y], 2.0 * M * C * C * 7)
    x2 = bf(M, 2 * C)
    pb2, (r3,) = pack([torch.randn(C, 2 * C, 3, device=dev) * 0.03])
    dx = torch.randn(M, C, device=dev)
    run_case("dil dgrad N = 128 K = 256 x 3 (ADDSCALE)", lambda: K.gemm(
        [K.Seg(x2, 2 * C, 2 * C, r3, T, taps=3, dil=2, shift0=-2)], B, T, C, pb2, Y, C,
        epi=L.EPI_ADDSCALE, aux1=dx, ld1=C, alpha=0.7071), [Y], 2.0 * M * C * 2 * C * 3)
    a1, a2 = bf(M, 2 * C), bf(M, 2 * C)
    pb3, (q1, q2) = pack([torch.randn(C, 2 * C, 1, device=dev) * 0.03,
                          torch.randn(C, 2 * C, 1, device=dev) * 0.03])
    run_case("two segments N = 128 K = 256 + 256 (PLAIN)", lambda: K.gemm(
        [K.Seg(a1, 2 * C, 2 * C, q1, T), K.Seg(a2, 2 * C, 2 * C, q2, T)], B, T, C, pb3, Y, C),
        [Y], 2.0 * M * C * 4 * C)
    a3 = bf(M, 20 * C)
    pb4, (q4,) = pack([torch.randn(C, 20 * C, 1, device=dev) * 0.01])
    run_case("skip sum N = 128 K = 2560 (PLAIN)", lambda: K.gemm(
        [K.Seg(a3, 20 * C, 20 * C, q4, T)], B, T, C, pb4, Y, C), [Y], 2.0 * M * C * 20 * C)


if __name__ == "__main__":
    main()
