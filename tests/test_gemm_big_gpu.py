"""256 x 256-tile bf16-operand GEMM (conv_gemm_b16_big_kernel) against the 128 x 128 kernel:
identical bits for every epilogue it takes (incl. the bf16 gate/filter save and its backward
read), multi-segment / multi-tap K, padding modes and a ragged M tail, at the row counts
where the step routes to it (>= 192 tiles)."""
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


def _both(run, mode=2, stages=0):
    """run() on the 128 x 128 kernel, then on the 256 x 256 kernel `mode` / `stages`."""
    outs = []
    try:
        for m, st in ((0, 0), (mode, stages)):
            K.set_big_tile(m, st)
            outs.append(run())
            torch.cuda.synchronize()
    finally:
        K.set_big_tile(2, 5)
    return outs


def _bf(t):
    return t.to(torch.bfloat16).contiguous()


@pytest.mark.parametrize("epi", [L.EPI_PLAIN, L.EPI_GATE, "gate_bf16", L.EPI_RESSKIP,
                                 L.EPI_GATE_BWD, "gate_bwd_bf16", L.EPI_ADDSCALE,
                                 L.EPI_RELU_MASK])
@pytest.mark.parametrize("B,T", [(30, 1024), (30, 1000)])
def test_big_tile_epilogues_bitwise(epi, B, T):
    _epilogue_case(epi, B, T, 3, 0)  # mode 3: every epilogue on the 256 x 256 kernel


@pytest.mark.parametrize("mode,stages", [(1, 3), (1, 4), (1, 5)])
def test_big_tile_variants_bitwise(mode, stages):
    _epilogue_case("gate_bf16", 30, 1000, mode, stages)  # (modes 1-2 take the gate GEMMs)


def _epilogue_case(epi, B, T, mode, stages):
    torch.manual_seed(11)
    C, E = 256, 256
    M = B * T
    x = _bf(torch.randn(M, C, device=DEV))
    cond = _bf(torch.randn(M, E, device=DEV))
    N = 2 * C
    wd = torch.randn(N, C, 3, device=DEV) / (3 * C) ** 0.5
    wc = torch.randn(N, E, 1, device=DEV) / E ** 0.5
    pb, (rd, rc) = _pack([wd, wc])
    segs = [K.Seg(x, C, C, rd, T, taps=3, dil=4, shift0=-4), K.Seg(cond, E, E, rc, T)]
    bias = torch.randn(N, device=DEV)
    aux1 = torch.randn(M, N, device=DEV)
    radd = torch.randn(B, C, device=DEV)

    def run():
        g = torch.Generator(DEV).manual_seed(3)
        y = torch.randn(M, N, device=DEV, generator=g)
        aux0 = torch.randn(M, N, device=DEV, generator=g)
        ybf = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        kw = dict(bias=bias)
        Nn = N
        if epi == L.EPI_PLAIN:
            kw.update(relu=True, accum=True, ybf=ybf, ybf_ld=N)
        elif epi in (L.EPI_GATE, "gate_bf16"):
            if epi == "gate_bf16":
                aux0 = _bf(aux0)
            kw.update(epi=L.EPI_GATE, aux0=aux0, ld0=N, C=C, ybf=ybf, ybf_ld=C, keep_y=False)
        elif epi == L.EPI_RESSKIP:
            kw.update(epi=epi, aux0=aux0, ld0=C, aux1=aux1, ld1=C, C=C, alpha=0.5, accum=True,
                      ybf=ybf, ybf_ld=C, ybf_radd=radd, ybf_radd_ld=C)
        elif epi in (L.EPI_GATE_BWD, "gate_bwd_bf16"):
            a1 = _bf(aux1) if epi == "gate_bwd_bf16" else aux1
            kw = dict(epi=L.EPI_GATE_BWD, aux1=a1, ld1=N, C=C, ybf=ybf, ybf_ld=N)
            Nn = C
        elif epi == L.EPI_ADDSCALE:
            kw = dict(epi=epi, aux1=aux1, ld1=N, alpha=0.25, relu=True)
        else:
            kw = dict(epi=epi, aux1=aux1, ld1=N, accum=True)
        K.gemm(segs, B, T, Nn, pb, y, N, **kw)
        return y, aux0, ybf
    (y0, a0, b0), (y1, a1_, b1) = _both(run, mode, stages)
    assert torch.equal(y0, y1)
    assert torch.equal(a0, a1_)
    assert torch.equal(b0, b1)


def test_big_tile_three_segments_reflect():
    """3 K-segments (7-tap reflect conv + 2 plain), N = 768 (3 N tiles)."""
    torch.manual_seed(5)
    B, T = 40, 1024
    M = B * T
    specs = [(128, 7, 1, L.PAD_REFLECT), (40, 1, 1, L.PAD_ZERO), (72, 3, 2, L.PAD_REPLICATE)]
    xs, ws = [], []
    N = 768
    for (Kc, taps, dil, pad) in specs:
        xs.append(_bf(torch.randn(M, Kc, device=DEV)))
        ws.append(torch.randn(N, Kc, taps, device=DEV) / (Kc * taps) ** 0.5)
    pb, refs = _pack(ws)
    segs = [K.Seg(x, Kc, Kc, r, T, taps=taps, dil=dil, shift0=-(taps // 2) * dil, pad=pad)
            for x, r, (Kc, taps, dil, pad) in zip(xs, refs, specs)]

    def run():
        y = torch.empty(M, N, device=DEV)
        K.gemm(segs, B, T, N, pb, y, N)
        return y
    a, b = _both(run, 3)
    assert torch.equal(a, b)
