"""Small-M GEMM probe (dev tool): the reverse-diffusion gate GEMM shape (M = 2 004 frames,
N = 512) with K = 1 024 / 512 / 256 (3 taps + cond, 1 tap + cond, cond), one-group vs
two-K-group kernel; average of back-to-back launches.   python tools/small_gemm_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L  # noqa: E402
from ensemble_svs_with_interactions_amd import kernels as K  # noqa: E402

dev = "cuda"
B, T, C, E = 1, 2004, 256, 256
M, N = B * T, 2 * C
torch.manual_seed(0)
x = torch.randn(M, C, device=dev).to(torch.bfloat16)
cond = torch.randn(M, E, device=dev).to(torch.bfloat16)
pb = K.PackedBuffer(L.DT_BF16)
rd = pb.add(torch.randn(N, C, 3, device=dev) * 0.05, N, C, 3, 3 * C, 3, 1)
r1 = pb.add(torch.randn(N, C, 1, device=dev) * 0.05, N, C, 1, C, 1, 1)
rc = pb.add(torch.randn(N, E, 1, device=dev) * 0.05, N, E, 1, E, 1, 1)
pb.finalize(dev)
pb.repack()
z = torch.empty(M, C, device=dev)
gf = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
zb = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
bias = torch.randn(N, device=dev)
y = torch.empty(M, N, device=dev)
shapes = {
    "K1024 gate": ([K.Seg(x, C, C, rd, T, taps=3, dil=4, shift0=-4), K.Seg(cond, E, E, rc, T)],
                   dict(epi=L.EPI_GATE, aux0=gf, ld0=N, C=C, ybf=zb, ybf_ld=C, keep_y=False)),
    "K512 plain": ([K.Seg(x, C, C, r1, T), K.Seg(cond, E, E, rc, T)], {}),
    "K256 plain": ([K.Seg(cond, E, E, rc, T)], {}),
    "K256 none": ([K.Seg(cond, E, E, rc, T)], dict(epi=L.EPI_NONE)),
    "K64 none": ([K.Seg(cond, 64, 64, rc, T)], dict(epi=L.EPI_NONE)),
}


def timed(fn, n=50):
    """Average per launch of n back-to-back launches replayed from a HIP graph (no host
    gaps between them)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side), torch.cuda.graph(g, stream=side):
        for _ in range(n):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (5 * n) * 1e3


for dual in (0, 1):
    K.set_dual_small(dual)
    for name, (segs, kw) in shapes.items():
        gate = kw.get("epi") == L.EPI_GATE
        out = z if gate else y
        ld = C if gate else N
        us = timed(lambda: K.gemm(segs, B, T, N, pb, out, ld, bias=bias, **kw))
        print(f"dual={dual} {name}: {us:.1f} us", flush=True)
K.set_dual_small(1)
K.BF16_ACT["on"] = False
xf = torch.randn(M, E, device=dev)
print(f"register-staged K256 plain: "
      f"{timed(lambda: K.gemm([K.Seg(xf, E, E, rc, T)], B, T, N, pb, y, N, bias=bias)):.1f} us")
K.BF16_ACT["on"] = True
# empty-kernel floor: a tiny launch back to back
tiny = torch.zeros(1, device=dev)
print(f"launch floor (axpy n=1): {timed(lambda: L.call('ensvs_axpy', tiny.data_ptr(), tiny.data_ptr(), 1.0, 1, K.stream())):.1f} us")
