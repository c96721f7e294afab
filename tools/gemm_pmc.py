"""Launch one GEMM shape of the training step 20 times, for rocprofv3 --pmc passes (dev tool).

  rocprofv3 --pmc <counters> --output-format csv -d OUT -o p -- python3 tools/gemm_pmc.py CASE
CASE: gate_fwd (mgc gate GEMM, 256 x 256 kernel), gate_bwd (mgc gate-backward dgrad,
M 30720, N 512, K 512, EPI_GATE_BWD + tile column sums), dil_dgrad (mgc dilated-conv
dgrad, N 256, K 3 x 512), wgrad_cond (conditioner weight gradient, N 10240, K 256),
wgrad_dil (dilated-conv weight gradient, N 512, K 256 x 3); the 128 x 256 kernel's launches:
skip_sum (N 256, K 5 120, lean plain), cond_dgrad (N 256, K 10 240, lean plain), res_fwd
(N 256, K 256, ADDSCALE with the bf16 copy and its per-sequence add).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ensemble_svs_with_interactions_amd import _lib, kernels as K  # noqa: E402


def main(case, iters=20):
    dev = torch.device("cuda")
    B, T = 30, 1024
    M = B * T
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    if case.startswith("wgrad"):
        N, Kc, taps, dil = (10240, 256, 1, 1) if case == "wgrad_cond" else (512, 256, 3, 4)
        dy, x = rnd(M, N).bfloat16(), rnd(M, Kc).bfloat16()
        dst = torch.zeros(N, Kc, taps, device=dev)
        fn = lambda: K.wgrad(dy, N, x, Kc, B, T, T, N, Kc, taps, dil,  # noqa: E731
                             -dil if taps > 1 else 0, _lib.PAD_ZERO, dst, Kc * taps, taps, 1,
                             accum=True)
    elif case in ("skip_sum", "cond_dgrad", "res_fwd"):
        N = 256
        Kc = {"skip_sum": 20 * N, "cond_dgrad": 40 * N, "res_fwd": N}[case]
        pb = K.PackedBuffer(_lib.DT_BF16)
        ref = pb.add(rnd(N, Kc, 1) * 0.01, N, Kc, 1, Kc, 1, 1)
        pb.finalize(dev)
        pb.repack()
        x = rnd(M, Kc).bfloat16()
        y = torch.empty(M, N, device=dev)
        segs = [K.Seg(x, Kc, Kc, ref, T)]
        if case == "res_fwd":
            xr = rnd(M, N)
            yb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ds, bias = rnd(B, 20 * N), rnd(N)
            fn = lambda: K.gemm(segs, B, T, N, pb, y, N, epi=_lib.EPI_ADDSCALE, aux1=xr,  # noqa
                                ld1=N, alpha=0.7071, ybf=yb, ybf_ld=N, ybf_radd=ds[:, N:],
                                ybf_radd_ld=20 * N, bias=bias)
        else:
            fn = lambda: K.gemm(segs, B, T, N, pb, y, N)  # noqa: E731
    else:
        pb = K.PackedBuffer(_lib.DT_BF16)
        if case == "gate_fwd":
            N, segs_spec = 512, [(256, 3, 4), (256, 1, 1)]
        elif case == "gate_bwd":  # dz (N = C channels) from [dx, dss], expanded to 2C
            N, segs_spec = 256, [(256, 1, 1), (256, 1, 1)]
        else:
            N, segs_spec = 256, [(512, 3, 4)]
        refs, xs = [], []
        for (Kc, taps, dil) in segs_spec:
            w = rnd(N, Kc, taps) * 0.02
            refs.append((pb.add(w, N, Kc, taps, Kc * taps, taps, 1), Kc, taps, dil))
            xs.append(rnd(M, Kc).bfloat16())
        pb.finalize(dev)
        pb.repack()
        segs = [K.Seg(x, Kc, Kc, ref, T, taps=taps, dil=dil, shift0=-dil if taps > 1 else 0)
                for x, (ref, Kc, taps, dil) in zip(xs, refs)]
        C = N // 2 if case == "gate_fwd" else N
        if case == "gate_fwd":
            z = torch.empty(M, C, device=dev)
            gf = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            zb = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
            fn = lambda: K.gemm(segs, B, T, N, pb, z, C, epi=_lib.EPI_GATE, aux0=gf, ld0=N,  # noqa
                                C=C, ybf=zb, ybf_ld=C, keep_y=False)
        elif case == "gate_bwd":
            y = torch.empty(M, 2 * C, device=dev)
            gf = rnd(M, 2 * C).bfloat16()
            yb = torch.empty(M, 2 * C, device=dev, dtype=torch.bfloat16)
            cs = torch.empty(M // 128, 2 * C, device=dev)
            fn = lambda: K.gemm(segs, B, T, N, pb, y, 2 * C, epi=_lib.EPI_GATE_BWD, aux1=gf,  # noqa
                                ld1=2 * C, C=C, ybf=yb, ybf_ld=2 * C, csum=cs, csum_ld=2 * C,
                                keep_y=False)
        else:
            y = torch.empty(M, N, device=dev)
            yb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            dx = rnd(M, N)
            cs = torch.empty(M // 128, N, device=dev)
            fn = lambda: K.gemm(segs, B, T, N, pb, y, N, epi=_lib.EPI_ADDSCALE, aux1=dx,  # noqa
                                ld1=N, alpha=0.7071, ybf=yb, ybf_ld=N, csum=cs, csum_ld=N)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{case}: {s.elapsed_time(e) / iters * 1e3:.1f} us/call", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gate_bwd")
