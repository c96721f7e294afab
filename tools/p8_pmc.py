"""One GEMM shape on the four-phase kernel (or the 128 x 128 one), repeated, for rocprofv3
--pmc passes (dev tool):
   rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... -- python3 tools/p8_pmc.py [shape] [mode]
shape: dgrad (M 30 720, N 1 024, K 2 x 2 048) | proj (N 4 096, K 512) | gate; mode: ensvs_set_p8."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib as L, kernels as K  # noqa: E402

SHAPES = {"dgrad": (1024, [(2048, 1, 1), (2048, 1, 1)], False),
          "proj": (4096, [(512, 1, 1)], True),
          "gate": (512, [(256, 3, 4), (256, 1, 1)], True)}

if __name__ == "__main__":
    L.load()
    shape = sys.argv[1] if len(sys.argv) > 1 else "dgrad"
    mode = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    N, spec, bias = SHAPES[shape]
    dev, T, M = torch.device("cuda"), 1024, 30 * 1024
    L.call("ensvs_set_p8", mode)
    pb = K.PackedBuffer(L.DT_BF16)
    segs = []
    for (Kc, taps, dil) in spec:
        ref = pb.add(torch.randn(N, Kc, taps, device=dev) * 0.03, N, Kc, taps, Kc * taps, taps, 1)
        segs.append(K.Seg(torch.randn(M, Kc, device=dev).to(torch.bfloat16), Kc, Kc, ref, T,
                          taps=taps, dil=dil, shift0=-(taps // 2) * dil))
    pb.finalize(dev)
    pb.repack()
    bv = torch.randn(N, device=dev) if bias else None
    if shape == "gate":
        C = N // 2
        z = torch.empty(M, C, device=dev)
        gf = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        zb = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        fn = lambda: K.gemm(segs, M // T, T, N, pb, z, C, epi=L.EPI_GATE, aux0=gf, ld0=N,  # noqa
                            C=C, ybf=zb, ybf_ld=C, keep_y=False, bias=bv)
    else:
        Y = torch.empty(M, N, device=dev)
        fn = lambda: K.gemm(segs, M // T, T, N, pb, Y, N, bias=bv)  # noqa: E731
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    print("done", shape, mode, flush=True)
