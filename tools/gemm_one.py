"""Run one GEMM shape through both forward kernels (register-staged and glds) for
rocprofv3 --pmc passes.  Dev tool: python3 tools/gemm_one.py [M N K taps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib, kernels as K  # noqa: E402

M, N, Kc, taps = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (30720, 1024, 1024, 1)))
T = 1024
B = M // T
dev = "cuda"
pb = K.PackedBuffer(_lib.DT_BF16)
w = torch.randn(N, Kc, taps, device=dev) * 0.02
ref = pb.add(w, N, Kc, taps, Kc * taps, taps, 1)
pb.finalize(dev)
pb.repack()
x = torch.randn(M, Kc, device=dev)
y = torch.empty(M, N, device=dev)
seg = [K.Seg(x, Kc, Kc, ref, T, taps=taps, dil=1, shift0=-(taps // 2))]
for on in (False, True):
    K.BF16_ACT.update(on=on, stages=2, min_reuse=1)
    for _ in range(10):
        K.gemm(seg, B, T, N, pb, y, N)
torch.cuda.synchronize()
print("ok", flush=True)
