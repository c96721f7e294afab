"""128 x 256-tile bf16-operand GEMM (conv_gemm_b16_p8h_kernel, ensvs_set_p8h) against the
128 x 128 kernel: identical bits for every epilogue it takes -- lean plain, plain with
accumulate / ReLU / bf16 copy, ADDSCALE, RELU_MASK, GATE_BWD (fp32 and bf16 gate/filter save)
-- and for the 128-row-tile column sums, multi-segment / multi-tap K with padding, a ragged M
tail, N = 256 (the DiffNet's C; wider launches with >= 128 tiles of 256 x 256 go to the
four-phase kernel first), K-loops of 1 to 80 K-steps (three-buffer ring wrap, the prologue's
short cases)."""
import pytest
import torch

from ensemble_svs_with_interactions_amd import _lib as L
from ensemble_svs_with_interactions_amd import kernels as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pack(ws):
    pb = K.PackedBuffer(L.DT_BF16)
    refs = [pb.add(w, w.shape[0], w.shape[1], w.shape[2], w.shape[1] * w.shape[2], w.shape[2], 1)
            for w in ws]
    pb.finalize(DEV)
    pb.repack()
    return pb, refs


def _both(run):
    """run() on the 128 x 128 kernel (p8h off), then on the 128 x 256 kernel (mode 2: every
    launch it can take)."""
    outs = []
    try:
        for on in (0, 2):
            L.call("ensvs_set_p8h", on)
            outs.append(run())
            torch.cuda.synchronize()
    finally:
        L.call("ensvs_set_p8h", 1)
    return outs


def _bf(t):
    return t.to(torch.bfloat16).contiguous()


def _assert_same(a, b):
    for u, v in zip(a, b):
        if u is not None:
            assert torch.equal(u, v), (u.float() - v.float()).abs().max().item()


@pytest.mark.parametrize("epi", ["plain_lean", "plain_full", "plain_csum", L.EPI_ADDSCALE,
                                 "addscale_csum", L.EPI_RELU_MASK, L.EPI_GATE_BWD,
                                 "gate_bwd_bf16", "gate_bwd_no_y"])
@pytest.mark.parametrize("B,T", [(30, 1024), (30, 1000)])
def test_p8h_epilogues_bitwise(epi, B, T):
    csum = epi in ("plain_csum", "addscale_csum", L.EPI_GATE_BWD, "gate_bwd_bf16",
                   "gate_bwd_no_y")
    if csum and T % 128:
        pytest.skip("column sums take whole 128-row tiles")
    torch.manual_seed(13)
    C = 256
    M = B * T
    N = C
    # the dilated-conv input gradient's shape: 3 taps over 2C channels, plus a plain segment
    dp = _bf(torch.randn(M, 2 * C, device=DEV))
    x2 = _bf(torch.randn(M, C, device=DEV))
    wd = torch.randn(N, 2 * C, 3, device=DEV) / (6 * C) ** 0.5
    w2 = torch.randn(N, C, 1, device=DEV) / C ** 0.5
    pb, (rd, r2) = _pack([wd, w2])
    segs = [K.Seg(dp, 2 * C, 2 * C, rd, T, taps=3, dil=8, shift0=-8), K.Seg(x2, C, C, r2, T)]
    bias = torch.randn(N, device=DEV)
    aux1 = torch.randn(M, 2 * N, device=DEV)
    radd = torch.randn(B, N, device=DEV)

    def run():
        g = torch.Generator(DEV).manual_seed(5)
        y = torch.randn(M, 2 * N, device=DEV, generator=g)
        ybf = torch.zeros(M, 2 * N, device=DEV, dtype=torch.bfloat16)
        cs = torch.zeros(M // 128, 2 * N, device=DEV) if csum else None
        kw = dict(bias=bias)
        if epi == "plain_lean":
            pass
        elif epi == "plain_full":
            kw.update(relu=True, accum=True, ybf=ybf, ybf_ld=2 * N, ybf_radd=radd,
                      ybf_radd_ld=N)
        elif epi == "plain_csum":
            kw = dict(ybf=ybf, ybf_ld=2 * N, csum=cs, csum_ld=2 * N)
        elif epi == L.EPI_ADDSCALE:
            kw.update(epi=epi, aux1=aux1, ld1=2 * N, alpha=0.7071, ybf=ybf, ybf_ld=2 * N)
        elif epi == "addscale_csum":
            kw = dict(epi=L.EPI_ADDSCALE, aux1=aux1, ld1=2 * N, alpha=0.7071, ybf=ybf,
                      ybf_ld=2 * N, csum=cs, csum_ld=2 * N)
        elif epi == L.EPI_RELU_MASK:
            kw = dict(epi=epi, aux1=aux1, ld1=2 * N, accum=True)
        else:
            a1 = aux1 if epi == L.EPI_GATE_BWD else _bf(aux1)
            kw = dict(epi=L.EPI_GATE_BWD, aux1=a1, ld1=2 * N, C=C, ybf=ybf, ybf_ld=2 * N,
                      csum=cs, csum_ld=2 * N, keep_y=epi != "gate_bwd_no_y")
        K.gemm(segs, B, T, N, pb, y, 2 * N, **kw)
        return y, ybf, cs
    a, b = _both(run)
    _assert_same(a, b)


@pytest.mark.parametrize("N,specs", [
    (256, [(128, 7, 1, L.PAD_REFLECT), (40, 1, 1, L.PAD_ZERO), (72, 3, 2, L.PAD_REPLICATE)]),
    (256, [(64, 1, 1, L.PAD_ZERO)]),                  # one K-step
    (256, [(128, 1, 1, L.PAD_ZERO)]),                 # two (prologue only)
    (256, [(192, 1, 1, L.PAD_ZERO)]),                 # three: the ring's first wrap
    (256, [(5120, 1, 1, L.PAD_ZERO)]),                # the DiffNet skip sum, K = L C
    (256, [(256, 3, 4, L.PAD_ZERO), (256, 1, 1, L.PAD_ZERO)]),
])
@pytest.mark.parametrize("B,T", [(30, 1024), (17, 999)])
def test_p8h_segments_bitwise(N, specs, B, T):
    torch.manual_seed(7)
    M = B * T
    if (M + 127) // 128 * (N // 256) < 128:
        pytest.skip("fewer than 128 tiles: the 128 x 128 kernel's launch")
    xs, ws = [], []
    for (Kc, taps, dil, pad) in specs:
        xs.append(_bf(torch.randn(M, Kc, device=DEV)))
        ws.append(torch.randn(N, Kc, taps, device=DEV) / (Kc * taps) ** 0.5)
    pb, refs = _pack(ws)
    segs = [K.Seg(x, Kc, Kc, r, T, taps=taps, dil=dil, shift0=-(taps // 2) * dil, pad=pad)
            for x, r, (Kc, taps, dil, pad) in zip(xs, refs, specs)]
    bias = torch.randn(N, device=DEV)

    def run():
        y = torch.empty(M, N, device=DEV)
        K.gemm(segs, B, T, N, pb, y, N, bias=bias)
        return (y,)
    a, b = _both(run)
    _assert_same(a, b)
    ref = sum(torch.nn.functional.conv1d(
        torch.nn.functional.pad(x.float().view(B, T, -1).transpose(1, 2),
                                ((taps // 2) * dil, (taps // 2) * dil),
                                mode={L.PAD_ZERO: "constant", L.PAD_REFLECT: "reflect",
                                      L.PAD_REPLICATE: "replicate"}[pad]),
        w.to(torch.bfloat16).float(), dilation=dil)
        for x, w, (Kc, taps, dil, pad) in zip(xs, ws, specs))
    ref = ref.transpose(1, 2).reshape(M, N) + bias
    err = (b[0] - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("N,specs,epi", [
    (4096, [(512, 1, 1, L.PAD_ZERO)], "plain"),                      # 8 K-steps
    (1024, [(2048, 1, 1, L.PAD_ZERO), (2048, 1, 1, L.PAD_ZERO)], "plain"),
    (512, [(64, 1, 1, L.PAD_ZERO)], "plain"),                        # 1 K-step
    (512, [(128, 1, 1, L.PAD_ZERO)], "plain"),                       # 2
    (512, [(192, 1, 1, L.PAD_ZERO)], "plain"),                       # 3: short of the lead
    (512, [(320, 1, 1, L.PAD_ZERO)], "relu_bf16"),                   # 5: the generic epilogue
    (512, [(256, 3, 4, L.PAD_ZERO), (256, 1, 1, L.PAD_ZERO)], "gate"),
    (768, [(128, 7, 1, L.PAD_REFLECT), (40, 1, 1, L.PAD_ZERO), (72, 3, 2, L.PAD_REPLICATE)],
     "plain"),
])
@pytest.mark.parametrize("B,T", [(30, 1024), (31, 999)])
def test_p8_barrier_forms_bitwise(N, specs, epi, B, T):
    """The four-phase 256 x 256 kernel, one barrier per phase and two with the wave rows
    staggered, against the 128 x 128 kernel (ensvs_set_p8 0 / 2 / 6): the same bits, K-loops
    of 1 to 64 K-steps, multi-segment / multi-tap K, the plain, generic and gate epilogues."""
    torch.manual_seed(9)
    M = B * T
    xs, ws = [], []
    for (Kc, taps, dil, pad) in specs:
        xs.append(_bf(torch.randn(M, Kc, device=DEV)))
        ws.append(torch.randn(N, Kc, taps, device=DEV) / (Kc * taps) ** 0.5)
    pb, refs = _pack(ws)
    segs = [K.Seg(x, Kc, Kc, r, T, taps=taps, dil=dil, shift0=-(taps // 2) * dil, pad=pad)
            for x, r, (Kc, taps, dil, pad) in zip(xs, refs, specs)]
    bias = torch.randn(N, device=DEV)
    C = N // 2

    def run():
        if epi == "gate":
            z = torch.zeros(M, C, device=DEV)
            gf = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
            zb = torch.zeros(M, C, device=DEV, dtype=torch.bfloat16)
            K.gemm(segs, B, T, N, pb, z, C, epi=L.EPI_GATE, aux0=gf, ld0=N, C=C, ybf=zb,
                   ybf_ld=C, keep_y=True, bias=bias)
            return z, gf, zb
        y = torch.empty(M, N, device=DEV)
        if epi == "relu_bf16":
            yb = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
            K.gemm(segs, B, T, N, pb, y, N, bias=bias, relu=True, ybf=yb, ybf_ld=N)
            return y, yb
        K.gemm(segs, B, T, N, pb, y, N, bias=bias)
        return (y,)
    outs = []
    try:
        for mode in (0, 2, 6):
            L.call("ensvs_set_p8", mode)
            outs.append(run())
            torch.cuda.synchronize()
    finally:
        L.call("ensvs_set_p8", 6)
    _assert_same(outs[0], outs[1])
    _assert_same(outs[0], outs[2])


@pytest.mark.parametrize("case", ["conv_k7", "addscale"])
@pytest.mark.parametrize("B,T", [(30, 1024), (7, 1000)])
def test_small_n128_bitwise(case, B, T):
    """ensvs_set_small(2) (A/B): the N = 128 launches of < 256 tiles of 128 x 128 on the 64 x 64
    kernel give the 128 x 128 kernel's bits (tools/n128_bench.py, profiles/r6_n128_bench.txt)."""
    torch.manual_seed(17)
    C = 128
    if case == "conv_k7":
        x = _bf(torch.randn(B * T, C, device=DEV))
        pb, (r,) = _pack([torch.randn(C, C, 7, device=DEV) * 0.03])
        bias = torch.randn(C, device=DEV)
        segs = [K.Seg(x, C, C, r, T, taps=7, shift0=-3)]
        kw = dict(bias=bias)
    else:
        x = _bf(torch.randn(B * T, 2 * C, device=DEV))
        pb, (r,) = _pack([torch.randn(C, 2 * C, 3, device=DEV) * 0.03])
        segs = [K.Seg(x, 2 * C, 2 * C, r, T, taps=3, dil=2, shift0=-2)]
        kw = dict(epi=L.EPI_ADDSCALE, aux1=torch.randn(B * T, C, device=DEV), ld1=C, alpha=0.7071)
    outs = []
    try:
        for mode in (1, 2):
            L.call("ensvs_set_small", mode)
            y = torch.full((B * T, C), float("nan"), device=DEV)
            K.gemm(segs, B, T, C, pb, y, C, **kw)
            torch.cuda.synchronize()
            outs.append(y)
    finally:
        L.call("ensvs_set_small", 1)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max().item()
