"""Dev probe of the DiffNet gate GEMM (M = 30 720 frames, N = 512, K = 3 x 256 + 256) as the
training step issues it (bf16 operands, GATE epilogue, bf16 z shadow, gate/filter save):
per-launch times of kernel variants with HIP events, and hipBLASLt's plain bf16 matmul of
the same M, N, K for an anchor.   python3 tools/gate_probe.py [iters] [variant]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L  # noqa: E402
from ensemble_svs_with_interactions_amd import kernels as K  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ONLY = sys.argv[2] if len(sys.argv) > 2 else None
dev = "cuda"
B, T, C, E = 30, 1024, 256, 256
M, N = B * T, 2 * C
torch.manual_seed(0)
x = torch.randn(M, C, device=dev).to(torch.bfloat16)
cond = torch.randn(M, E, device=dev).to(torch.bfloat16)
pb = K.PackedBuffer(L.DT_BF16)
rd = pb.add(torch.randn(N, C, 3, device=dev) * 0.05, N, C, 3, 3 * C, 3, 1)
rc = pb.add(torch.randn(N, E, 1, device=dev) * 0.05, N, E, 1, E, 1, 1)
pb.finalize(dev)
pb.repack()
segs = [K.Seg(x, C, C, rd, T, taps=3, dil=4, shift0=-4), K.Seg(cond, E, E, rc, T)]
bias = torch.randn(N, device=dev)
z = torch.empty(M, C, device=dev)
zb = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
gf32 = torch.empty(M, N, device=dev)
gf16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
y = torch.empty(M, N, device=dev)


def timed(fn):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(ITERS):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / ITERS * 1e3


def gate(gf):
    return lambda: K.gemm(segs, B, T, N, pb, z, C, epi=L.EPI_GATE, aux0=gf, ld0=N, C=C,
                          ybf=zb, ybf_ld=C, keep_y=False, bias=bias)


xk = torch.randn(M, 1024, device=dev).to(torch.bfloat16)
pk = K.PackedBuffer(L.DT_BF16)
rk = pk.add(torch.randn(N, 1024, 1, device=dev) * 0.03, N, 1024, 1, 1024, 1, 1)
pk.finalize(dev)
pk.repack()
seg1 = [K.Seg(xk, 1024, 1024, rk, T)]
variants = {
    "gate_gf16": gate(gf16),
    "gate_none": lambda: K.gemm(segs, B, T, N, pb, y, N, epi=L.EPI_NONE),
    "plain_f32": lambda: K.gemm(segs, B, T, N, pb, y, N),
    "k1024_plain_f32": lambda: K.gemm(seg1, B, T, N, pk, y, N),
    "k1024_none": lambda: K.gemm(seg1, B, T, N, pk, y, N, epi=L.EPI_NONE),
}
A = torch.randn(M, 1024, device=dev).to(torch.bfloat16)
W = torch.randn(1024, N, device=dev).to(torch.bfloat16)
for mode, stages, label in ((1, 5, "ring5"), (1, 4, "ring4"), (1, 3, "ring3"),
                            (2, 0, "big64x2"), (0, 0, "128")):
    K.set_big_tile(mode, stages)
    for name, fn in variants.items():
        if ONLY and name != ONLY:
            continue
        print(f"{label} {name}: {timed(fn):.1f} us", flush=True)
K.set_big_tile(2, 5)
if not ONLY:
    print(f"hipBLASLt bf16 matmul {M}x1024x{N} (bf16 out): "
          f"{timed(lambda: torch.matmul(A, W)):.1f} us", flush=True)
