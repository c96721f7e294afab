"""Dev probe: the DiffNet backward / res-skip GEMM launches of the mgc block (M = 30 720,
C = 256) with their product epilogues vs the same launch with no epilogue (EPI_NONE: K loop
only), HIP events.   python3 tools/dgrad_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L  # noqa: E402
from ensemble_svs_with_interactions_amd import kernels as K  # noqa: E402

EPI_NONE = 7
dev = "cuda"
B, T, C = 30, 1024, 256
M = B * T
torch.manual_seed(0)
bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)  # noqa: E731
pb = K.PackedBuffer(L.DT_BF16)
w_res = pb.add(torch.randn(C, C, 1, device=dev) * 0.05, C, C, 1, C, 1, 1)
w_skip = pb.add(torch.randn(C, C, 1, device=dev) * 0.05, C, C, 1, C, 1, 1)
w_dil = pb.add(torch.randn(C, 2 * C, 3, device=dev) * 0.05, C, 2 * C, 3, 6 * C, 3, 1)
w_rs = pb.add(torch.randn(2 * C, C, 1, device=dev) * 0.05, 2 * C, C, 1, C, 1, 1)
pb.finalize(dev)
pb.repack()
dx, dss, z = bf(M, C), bf(M, C), bf(M, C)
gf = bf(M, 2 * C)
dpre = bf(M, 2 * C)
Y = torch.empty(M, 2 * C, device=dev)
Yb = torch.empty(M, 2 * C, device=dev, dtype=torch.bfloat16)
cs = torch.empty(M // 128, 2 * C, device=dev)
xres = torch.randn(M, C, device=dev)
skip = torch.randn(M, C, device=dev)
xn = torch.empty(M, C, device=dev)
bias = torch.randn(2 * C, device=dev)


def timed(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


segs_gb = [K.Seg(dx, C, C, w_res, T), K.Seg(dss, C, C, w_skip, T)]
segs_dil = [K.Seg(dpre, 2 * C, 2 * C, w_dil, T, taps=3, dil=4, shift0=-4)]
segs_rs = [K.Seg(z, C, C, w_rs, T)]
cases = {
    "gate_bwd GATE_BWD": lambda: K.gemm(segs_gb, B, T, C, pb, Y, 2 * C, epi=L.EPI_GATE_BWD,
                                        aux1=gf, ld1=2 * C, C=C, ybf=Yb, ybf_ld=2 * C, csum=cs,
                                        csum_ld=2 * C, keep_y=False),
    "gate_bwd NONE": lambda: K.gemm(segs_gb, B, T, C, pb, Y, 2 * C, epi=EPI_NONE),
    "dil_dgrad ADDSCALE": lambda: K.gemm(segs_dil, B, T, C, pb, Y, C, epi=L.EPI_ADDSCALE,
                                         aux1=xres, ld1=C, alpha=0.7071, ybf=Yb, ybf_ld=C,
                                         csum=cs, csum_ld=2 * C),
    "dil_dgrad NONE": lambda: K.gemm(segs_dil, B, T, C, pb, Y, C, epi=EPI_NONE),
    "res_skip RESSKIP": lambda: K.gemm(segs_rs, B, T, 2 * C, pb, xn, C, bias=bias,
                                       epi=L.EPI_RESSKIP, aux0=skip, ld0=C, aux1=xres, ld1=C,
                                       accum=True, alpha=0.2236, C=C, ybf=Yb, ybf_ld=C),
    "res_skip NONE": lambda: K.gemm(segs_rs, B, T, 2 * C, pb, Y, 2 * C, epi=EPI_NONE),
}
# FFConvLSTM encoder launches: the LSTM input projection (K = 128 conv channels -> 8H = 512
# gates, bias, fp32 out) and the ReLU-mask conv dgrad (K = N = 256, fp32 mask, bf16 copy)
xk = bf(M, 128)
w_ih = pb2 = K.PackedBuffer(L.DT_BF16)
r_ih = pb2.add(torch.randn(512, 128, 1, device=dev) * 0.05, 512, 128, 1, 128, 1, 1)
r_rm = pb2.add(torch.randn(256, 256, 1, device=dev) * 0.05, 256, 256, 1, 256, 1, 1)
pb2.finalize(dev)
pb2.repack()
gates = torch.empty(M, 512, device=dev)
b512 = torch.randn(512, device=dev)
mask_src = torch.randn(M, 256, device=dev)
nd = torch.empty(M, 256, device=dev)
ndb = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
cases.update({
    "w_ih PLAIN": lambda: K.gemm([K.Seg(xk, 128, 128, r_ih, T)], B, T, 512, pb2, gates, 512,
                                 bias=b512),
    "w_ih NONE": lambda: K.gemm([K.Seg(xk, 128, 128, r_ih, T)], B, T, 512, pb2, gates, 512,
                                epi=EPI_NONE),
    "relu_mask RELU_MASK": lambda: K.gemm([K.Seg(z, C, C, r_rm, T)], B, T, 256, pb2, nd, 256,
                                          epi=L.EPI_RELU_MASK, aux1=mask_src, ld1=256, ybf=ndb,
                                          ybf_ld=256),
    "relu_mask NONE": lambda: K.gemm([K.Seg(z, C, C, r_rm, T)], B, T, 256, pb2, nd, 256,
                                     epi=EPI_NONE),
})
cases["dil_dgrad ADDSCALE nocsum"] = lambda: K.gemm(segs_dil, B, T, C, pb, Y, C,
                                                   epi=L.EPI_ADDSCALE, aux1=xres, ld1=C,
                                                   alpha=0.7071)
if os.environ.get("BIG"):  # 256 x 256 tiles for every epilogue that allows them
    L.call("ensvs_set_big_tile", 3, 0)
only = sys.argv[1:] or list(cases)
for name in cases:
    if any(o in name for o in only):
        print(f"{name:24s} {timed(cases[name]):7.1f} us", flush=True)
