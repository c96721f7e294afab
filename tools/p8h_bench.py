"""The 128 x 256 GEMM kernel (ensvs_set_p8h) against the 128 x 128 kernel on the DiffNet's
N = 256 launches at 30 x 1024 frames (dev tool): HIP-event time per launch and a bitwise check.
   python tools/p8h_bench.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L, kernels as K  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda")
B, T, C, LL = 30, 1024, 256, 20
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


ARMS = (("eng128", "ensvs_set_p8h", 0), ("p8h", "ensvs_set_p8h", 2),
        ("p8_120tiles", "ensvs_set_p8_min_tiles", 96))


def run_case(name, fn, outs, flops):
    res = dict(case=name)
    ref = None
    for tag, sw, on in ARMS:
        L.call("ensvs_set_p8h", 0)
        L.call("ensvs_set_p8_min_tiles", 128)
        L.call(sw, on)
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
    L.call("ensvs_set_p8h", 1)
    L.call("ensvs_set_p8_min_tiles", 128)
    print(json.dumps(res), flush=True)


def main():
    L.load()
    # dilated-conv input gradient: dx' = dx / sqrt2 + conv^T(dpre) (ADDSCALE), bf16 copy, tile sums
    dpre = bf(M, LL * 2 * C)
    pb, (rd,) = pack([torch.randn(C, 2 * C, 3, device=dev) * 0.02])
    segs = [K.Seg(dpre, LL * 2 * C, 2 * C, rd, T, taps=3, dil=8, shift0=-8, xoff=3 * 2 * C)]
    dx = torch.randn(M, C, device=dev)
    xnew, xnewb = torch.empty(M, C, device=dev), torch.empty(M, C, device=dev,
                                                                 dtype=torch.bfloat16)
    cs = torch.empty(M // 128, LL * C, device=dev)
    run_case("dil dgrad ADDSCALE+csum", lambda: K.gemm(
        segs, B, T, C, pb, xnew, C, epi=L.EPI_ADDSCALE, aux1=dx, ld1=C, alpha=0.7071,
        ybf=xnewb, ybf_ld=C, csum=cs, csum_ld=LL * C, csum_off=3 * C), [xnew, xnewb, cs],
        2.0 * M * C * 6 * C)
    run_case("dil dgrad first block (PLAIN+csum)", lambda: K.gemm(
        segs, B, T, C, pb, xnew, C, ybf=xnewb, ybf_ld=C, csum=cs, csum_ld=LL * C,
        csum_off=3 * C), [xnew, xnewb, cs], 2.0 * M * C * 6 * C)
    # gate backward: [dx, dss] -> d(gate), d(filter) bf16 + tile sums (no fp32 copy)
    dxb, dssb = bf(M, C), bf(M, C)
    pb2, (r1, r2) = pack([torch.randn(C, C, 1, device=dev) * 0.06,
                          torch.randn(C, C, 1, device=dev) * 0.06])
    GF = bf(M, 2 * C)
    dpre_all = torch.empty(M, LL * 2 * C, device=dev)
    cs2 = torch.empty(M // 128, LL * 2 * C, device=dev)
    dpb = torch.empty(M, LL * 2 * C, device=dev, dtype=torch.bfloat16)
    run_case("gate bwd (GATE_BWD+csum, no fp32 y)", lambda: K.gemm(
        [K.Seg(dxb, C, C, r1, T), K.Seg(dssb, C, C, r2, T)], B, T, C, pb2, dpre_all,
        LL * 2 * C, yoff=3 * 2 * C, epi=L.EPI_GATE_BWD, aux1=GF, ld1=2 * C, C=C,
        ybf=dpb[:, 3 * 2 * C:], ybf_ld=LL * 2 * C, csum=cs2, csum_ld=LL * 2 * C,
        csum_off=3 * 2 * C, keep_y=False), [dpb, cs2], 2.0 * M * C * 2 * C)
    # forward residual half: x' = x / sqrt2 + W z + b (ADDSCALE), bf16 copy with the next add
    zb = bf(M, C)
    pb3, (r3, r4) = pack([torch.randn(C, C, 1, device=dev) * 0.06,
                          torch.randn(C, LL * C, 1, device=dev) * 0.01])
    x = torch.randn(M, C, device=dev)
    xn, xbn = torch.empty(M, C, device=dev), torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    ds = torch.randn(B, LL * C, device=dev)
    bias = torch.randn(C, device=dev)
    run_case("res fwd (ADDSCALE, bf16 copy + add)", lambda: K.gemm(
        [K.Seg(zb, C, C, r3, T)], B, T, C, pb3, xn, C, epi=L.EPI_ADDSCALE, aux1=x, ld1=C,
        alpha=0.7071, ybf=xbn, ybf_ld=C, ybf_radd=ds[:, C:], ybf_radd_ld=LL * C, bias=bias),
        [xn, xbn], 2.0 * M * C * C)
    # the skip sum over every block: K = L C
    zall = bf(M, LL * C)
    S = torch.empty(M, C, device=dev)
    run_case("skip sum (K = 5120, PLAIN)", lambda: K.gemm(
        [K.Seg(zall, LL * C, LL * C, r4, T)], B, T, C, pb3, S, C, bias=bias), [S],
        2.0 * M * C * LL * C)
    # the skip projection with ReLU and its bf16 copy (K = 256), the dss GEMM (plain, K = 256)
    p1, p1b = torch.empty(M, C, device=dev), torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    run_case("skip relu + bf16 copy (K = 256)", lambda: K.gemm(
        [K.Seg(zb, C, C, r3, T)], B, T, C, pb3, p1, C, relu=True, ybf=p1b, ybf_ld=C, bias=bias),
        [p1, p1b], 2.0 * M * C * C)
    run_case("dss plain (K = 256)", lambda: K.gemm(
        [K.Seg(zb, C, C, r3, T)], B, T, C, pb3, p1, C), [p1], 2.0 * M * C * C)
    # the output projection's input gradient through the skip projection's ReLU (RELU_MASK)
    mask = torch.randn(M, C, device=dev)
    run_case("relu-mask dgrad (K = 256)", lambda: K.gemm(
        [K.Seg(zb, C, C, r3, T)], B, T, C, pb3, p1, C, epi=L.EPI_RELU_MASK, aux1=mask, ld1=C),
        [p1], 2.0 * M * C * C)
    # the conditioner input gradient: K = L 2C over every block's d(pre)
    pb4, (r5,) = pack([torch.randn(C, LL * 2 * C, 1, device=dev) * 0.01])
    run_case("cond dgrad (K = 10240, PLAIN)", lambda: K.gemm(
        [K.Seg(dpre, LL * 2 * C, LL * 2 * C, r5, T)], B, T, C, pb4, S, C), [S],
        2.0 * M * C * LL * 2 * C)


if __name__ == "__main__":
    main()
