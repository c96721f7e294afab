"""bf16-activation GEMM path (ensvs_cast_bf16 + ensvs_conv_gemm_bf16a: global_load_lds
staging, swizzled LDS, counted vmcnt) against the register-staged bf16 kernel: identical
bits for every epilogue, padding mode, tap/dilation, multi-segment K and ragged M/N/K."""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import kernels as K
from ensemble_svs_with_interactions_amd import _lib as L

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
    """run() with the bf16-activation path forced off, then forced on (split-K off: these
    compare the staging paths of one accumulation order; test_splitk_* cover split-K)."""
    saved = dict(K.BF16_ACT)
    split = K.SPLITK["on"]
    outs = []
    try:
        K.SPLITK["on"] = False
        K.set_dual_small(False)
        for on in (False, True):
            K.BF16_ACT.update(on=on, min_reuse=1, min_rows=0)
            outs.append(run())
            torch.cuda.synchronize()
    finally:
        K.BF16_ACT.clear()
        K.BF16_ACT.update(saved)
        K.SPLITK["on"] = split
        K.set_dual_small(False)
    return outs


@pytest.mark.parametrize("stages", [2, 3])
@pytest.mark.parametrize("B,T,specs,N", [
    (3, 100, [(64, 3, 2, L.PAD_ZERO, True), (32, 1, 1, L.PAD_ZERO, False)], 256),
    (2, 77, [(40, 5, 1, L.PAD_REFLECT, False)], 200),
    (4, 33, [(24, 3, 4, L.PAD_REPLICATE, True), (16, 1, 1, L.PAD_ZERO, False),
             (8, 2, 1, L.PAD_ZERO, False)], 130),
    (30, 1024, [(256, 3, 8, L.PAD_ZERO, True), (256, 1, 1, L.PAD_ZERO, False)], 512),
])
def test_bf16a_plain_bitwise(stages, B, T, specs, N):
    torch.manual_seed(stages + B)
    segs_in = []
    for (Kc, taps, dil, pad, radd) in specs:
        x = torch.randn(B * T, Kc + 8, device=DEV)  # ld > K
        w = torch.randn(N, Kc, taps, device=DEV) / (Kc * taps) ** 0.5
        r = torch.randn(B, Kc, device=DEV) if radd else None
        segs_in.append((x, w, Kc, taps, dil, pad, r))
    pb, refs = _pack([s[1] for s in segs_in])
    segs = [K.Seg(x, Kc + 8, Kc, ref, T, taps=taps, dil=dil, shift0=-(taps // 2) * dil, pad=pad,
                  radd=r, radd_ld=0 if r is None else Kc)
            for (x, w, Kc, taps, dil, pad, r), ref in zip(segs_in, refs)]
    bias = torch.randn(N, device=DEV)

    def run():
        y = torch.randn(B * T, N, device=DEV, generator=torch.Generator(DEV).manual_seed(5))
        K.BF16_ACT["stages"] = stages
        K.gemm(segs, B, T, N, pb, y, N, bias=bias, relu=True, accum=True)
        return y
    a, b = _both(run)
    assert torch.equal(a, b)


@pytest.mark.parametrize("epi", [L.EPI_GATE, L.EPI_RESSKIP, L.EPI_GATE_BWD, L.EPI_ADDSCALE,
                                 L.EPI_RELU_MASK, L.EPI_GATE_TS, "sigmoid"])
def test_bf16a_epilogues_bitwise(epi):
    torch.manual_seed(7)
    B, T, C, E = 2, 150, 64, 48
    x = torch.randn(B * T, C, device=DEV)
    cond = torch.randn(B * T, E, device=DEV)
    d = torch.randn(B, C, device=DEV)
    N = 2 * C
    wd = torch.randn(N, C, 3, device=DEV) / (3 * C) ** 0.5
    wc = torch.randn(N, E, 1, device=DEV) / E ** 0.5
    pb, (rd, rc) = _pack([wd, wc])
    segs = [K.Seg(x, C, C, rd, T, taps=3, dil=2, shift0=-2, radd=d, radd_ld=C),
            K.Seg(cond, E, E, rc, T)]
    bias = torch.randn(N, device=DEV)
    aux1 = torch.randn(B * T, N, device=DEV)

    def run():
        g = torch.Generator(DEV).manual_seed(3)
        y = torch.randn(B * T, N, device=DEV, generator=g)
        aux0 = torch.randn(B * T, N, device=DEV, generator=g)
        kw = dict(bias=bias)
        if epi == "sigmoid":
            kw.update(relu=2)
        elif epi in (L.EPI_GATE, L.EPI_RESSKIP, L.EPI_GATE_TS):
            kw.update(epi=epi, aux0=aux0, ld0=N, aux1=aux1, ld1=N, C=C, alpha=0.5, accum=True)
        elif epi == L.EPI_GATE_BWD:
            kw.update(epi=epi, aux1=aux1, ld1=N, C=C)
        else:
            kw.update(epi=epi, aux1=aux1, ld1=N, alpha=0.25, accum=True)
        Nn = C if epi == L.EPI_GATE_BWD else N
        K.gemm(segs, B, T, Nn, pb, y, N, **kw)
        return y, aux0
    (y0, a0), (y1, a1) = _both(run)
    assert torch.equal(y0, y1) and torch.equal(a0, a1)


@pytest.mark.parametrize("which", ["mgc", "bap", "mgc_t256"])
def test_diffnet_bf16_operands_bitwise(which):
    """DiffNet forward + backward on the bf16-operand path (cond, dss and dpre rounded once,
    dx rounded by its axpby or the dgrad epilogue, the rest by per-GEMM casts) equals the
    register-staged path bit for bit.  mgc_t256: whole 128-frame tiles per sequence, so the
    dgrad GEMM's epilogue also produces dx_l and the tile column sums of dy (fallback:
    ensvs_tile_colsum + axpby)."""
    from ensemble_svs_with_interactions_amd import configs, engine
    from golden_util import full_shapes, load_case
    from gpu_util import build
    engine.set_gemm_precision("bf16")
    t256 = which == "mgc_t256"
    which = which.split("_")[0]
    a, meta = load_case(f"diffnet_{which}")
    if t256:  # same weights, synthetic inputs of 2 x 256 frames
        rng = np.random.default_rng(11)
        Mc, E = a["spec"].shape[2], a["cond"].shape[1]
        a = dict(spec=rng.standard_normal((2, 1, Mc, 256), dtype=np.float32),
                 cond=rng.standard_normal((2, E, 256), dtype=np.float32),
                 t=np.array([3, 77], dtype=np.int64),
                 R=rng.standard_normal((2, 1, Mc, 256), dtype=np.float32))
    cfg = configs.multitrack_diffusion(num_speakers=4)[f"{which}_model"]["denoise_fn"]
    B, _, Mc, T = a["spec"].shape
    E = a["cond"].shape[1]
    xin = torch.from_numpy(a["spec"])[:, 0].transpose(1, 2).contiguous().view(B * T, Mc).cuda()
    cnd = torch.from_numpy(a["cond"]).transpose(1, 2).contiguous().view(B * T, E).cuda()
    t = torch.from_numpy(a["t"]).cuda()
    R = torch.from_numpy(a["R"])[:, 0].transpose(1, 2).contiguous().view(B * T, Mc).cuda()

    def run():
        mod = build(cfg, full_shapes(), meta["prefix"])
        out, st = mod._fwd(xin, Mc, t, cnd, E, B, T)
        dcond = mod._bwd(st, R)
        torch.cuda.synchronize()
        return out.clone(), dcond.clone(), {k: p.grad.clone() for k, p in mod.named_parameters()}
    (o0, d0, g0), (o1, d1, g1) = _both(run)
    assert torch.equal(o0, o1) and torch.equal(d0, d1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("epi", [L.EPI_PLAIN, L.EPI_ADDSCALE])
def test_bf16a_tile_colsum_bitwise(epi):
    """Per-128-row-tile column sums of the accumulator (and the ADDSCALE output with its bf16
    copy) from the LDS epilogue equal the fallback (plain GEMM + ensvs_tile_colsum + axpby) bit
    for bit, and the sums match an fp64 column sum of the plain GEMM output."""
    torch.manual_seed(9)
    B, T, C, N = 2, 256, 96, 64
    x = torch.randn(B * T, C, device=DEV)
    w = torch.randn(N, C, 3, device=DEV) / (3 * C) ** 0.5
    pb, (r,) = _pack([w])
    segs = [K.Seg(x, C, C, r, T, taps=3, dil=2, shift0=-2)]
    aux1 = torch.randn(B * T, N, device=DEV)
    ld = 3 * N

    def run():
        y = torch.empty(B * T, N, device=DEV)
        yb = torch.empty(B * T, N, device=DEV, dtype=torch.bfloat16)
        cs = torch.full((B * T // 128, ld), 7.0, device=DEV)
        kw = {} if epi == L.EPI_PLAIN else dict(epi=epi, aux1=aux1, ld1=N, alpha=0.7071)
        K.gemm(segs, B, T, N, pb, y, N, ybf=yb, ybf_ld=N, csum=cs, csum_ld=ld, csum_off=N, **kw)
        torch.cuda.synchronize()
        return y, yb, cs
    (y0, b0, c0), (y1, b1, c1) = _both(run)
    assert torch.equal(y0, y1) and torch.equal(b0, b1) and torch.equal(c0, c1)
    assert torch.equal(b0, y0.to(torch.bfloat16))
    assert (c0[:, :N] == 7.0).all() and (c0[:, 2 * N:] == 7.0).all()
    acc = y0 if epi == L.EPI_PLAIN else y0 - 0.7071 * aux1
    ref = acc.double().view(B * T // 128, 128, N).sum(1)
    torch.testing.assert_close(c0[:, N:2 * N].double(), ref, rtol=1e-4, atol=1e-3)


def _close(a, b, rtol):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item() < rtol


@pytest.mark.parametrize("C", [256, 128])
@pytest.mark.parametrize("epi", [L.EPI_PLAIN, L.EPI_GATE, "gate_bf16", L.EPI_RESSKIP,
                                 L.EPI_GATE_BWD, L.EPI_ADDSCALE, L.EPI_RELU_MASK])
def test_splitk_and_dual_match_unsplit(epi, C):
    """Small-M launches (2 x 1002 frames: 64 tiles, 16 K-steps): the 64 x 64-tile kernel (the
    default) bit-identical to the one-group kernel; the two-K-group kernel and split-K (4 K
    splits): the same results as the one-group kernel up
    to fp32 summation order (rel 1e-5; bf16 copies within one bf16 rounding), every epilogue
    and bf16 output copy, and bit-identical from run to run."""
    torch.manual_seed(21)
    B, T, E = 2, 1002 if C == 256 else 252, C
    M, N = B * T, 2 * C
    x = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    cond = torch.randn(M, E, device=DEV).to(torch.bfloat16)
    wd = torch.randn(N, C, 3, device=DEV) / (3 * C) ** 0.5
    wc = torch.randn(N, E, 1, device=DEV) / E ** 0.5
    pb, (rd, rc) = _pack([wd, wc])
    segs = [K.Seg(x, C, C, rd, T, taps=3, dil=4, shift0=-4), K.Seg(cond, E, E, rc, T)]
    bias = torch.randn(N, device=DEV)
    aux1 = torch.randn(M, N, device=DEV)
    radd = torch.randn(B, C, device=DEV)

    def run():
        g = torch.Generator(DEV).manual_seed(4)
        y = torch.randn(M, N, device=DEV, generator=g)
        aux0 = torch.randn(M, N, device=DEV, generator=g)
        ybf = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        Nn, kw = N, dict(bias=bias)
        if epi == L.EPI_PLAIN:
            kw.update(relu=True, accum=True, ybf=ybf, ybf_ld=N)
        elif epi in (L.EPI_GATE, "gate_bf16"):
            if epi == "gate_bf16":
                aux0 = aux0.to(torch.bfloat16)
            kw.update(epi=L.EPI_GATE, aux0=aux0, ld0=N, C=C, ybf=ybf, ybf_ld=C)
        elif epi == L.EPI_RESSKIP:
            kw.update(epi=epi, aux0=aux0, ld0=C, aux1=aux1, ld1=C, C=C, alpha=0.5, accum=True,
                      ybf=ybf, ybf_ld=C, ybf_radd=radd, ybf_radd_ld=C)
        elif epi == L.EPI_GATE_BWD:
            kw = dict(epi=epi, aux1=aux1, ld1=N, C=C, ybf=ybf, ybf_ld=N)
            Nn = C
        elif epi == L.EPI_ADDSCALE:
            kw = dict(epi=epi, aux1=aux1, ld1=N, alpha=0.25)
        else:
            kw = dict(epi=epi, aux1=aux1, ld1=N, accum=True)
        K.gemm(segs, B, T, Nn, pb, y, N, **kw)
        torch.cuda.synchronize()
        return y, aux0, ybf
    split = K.SPLITK["on"]
    try:
        K.SPLITK["on"] = False
        K.set_small(False)
        K.set_dual_small(False)
        ref = run()
        K.set_small(True)
        small = run()
        K.set_small(False)
        K.set_dual_small(True)
        dual = [run(), run()]
        K.SPLITK["on"] = True
        spl = [run(), run()]
    finally:
        K.SPLITK["on"] = split
        K.set_dual_small(False)
        K.set_small(True)
    # the 64 x 64-tile kernel: the one-group kernel's accumulation order, identical bits
    for t0, t1 in zip(ref, small):
        assert torch.equal(t0, t1)
    for (y1, a1, b1), (y2, a2, b2) in (dual, spl):
        assert torch.equal(y1, y2) and torch.equal(a1, a2) and torch.equal(b1, b2)
        y0, a0, b0 = ref
        assert _close(y1, y0, 1e-5)
        assert _close(a1, a0, 1e-2 if a0.dtype == torch.bfloat16 else 1e-5)
        assert _close(b1.float(), b0.float(), 1e-2)


@pytest.mark.parametrize("N", [5, 60, 128, 256])
@pytest.mark.parametrize("relu", [False, True])
def test_small_kernel_ragged_n_bitwise(N, relu):
    """The 64 x 64 kernel (small M, and N <= 64 at any M) against the one-group 128 x 128
    kernel: identical bits for ragged N (N = 5: a scalar epilogue column) with a bf16 copy
    of the output, 2 x 252 rows (tiles across the sequence boundary)."""
    torch.manual_seed(N)
    B, T, Kc = 2, 252, 128
    M = B * T
    x = torch.randn(M, Kc, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, Kc, 1, device=DEV) / Kc ** 0.5
    pb, (r,) = _pack([w])
    bias = torch.randn(N, device=DEV)

    def run():
        y = torch.full((M, N), 7.0, device=DEV)
        yb = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        kw = dict(ybf=yb, ybf_ld=N) if N % 4 == 0 else {}
        K.gemm([K.Seg(x, Kc, Kc, r, T)], B, T, N, pb, y, N, bias=bias, relu=relu, **kw)
        torch.cuda.synchronize()
        return y, yb
    try:
        K.set_small(False)
        K.set_dual_small(False)
        ref = run()
        K.set_small(True)
        got = run()
    finally:
        K.set_small(True)
        K.set_dual_small(False)
    assert torch.equal(ref[0], got[0])
    assert torch.equal(ref[1], got[1])


@pytest.mark.parametrize("C,B,T,ldm", [(256, 3, 256, 1), (128, 2, 384, 3), (256, 30, 1024, 1)])
def test_gate_bwd_dma_epilogue_bitwise(C, B, T, ldm):
    """The DiffNet gate-backward dgrad in its production form (bf16 dx / dss segments, bf16
    gate/filter save in, bf16 d(pre) out into a wider [M][ldm * 2C] buffer, per-tile column
    sums, no fp32 Y): the LDS-DMA epilogue equals the register-batched one bit for bit."""
    torch.manual_seed(C + T)
    M = B * T
    dx = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    dss = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    w0 = (torch.randn(C, C, 1, device=DEV) / C ** 0.5).to(torch.bfloat16).float()
    w1 = (torch.randn(C, C, 1, device=DEV) / C ** 0.5).to(torch.bfloat16).float()
    pb, (r0, r1) = _pack([w0, w1])
    segs = [K.Seg(dx, C, C, r0, T), K.Seg(dss, C, C, r1, T)]
    gf = (torch.randn(M, 2 * C, device=DEV) * 2).to(torch.bfloat16)
    Y = torch.empty(M, 2 * C, device=DEV)

    def run(on):
        L.call("ensvs_set_gbw_dma", int(on))
        yb = torch.full((M, ldm * 2 * C), 3.0, device=DEV).to(torch.bfloat16)
        cs = torch.full((M // 128, ldm * 2 * C), 7.0, device=DEV)
        K.gemm(segs, B, T, C, pb, Y, 2 * C, epi=L.EPI_GATE_BWD, aux1=gf, ld1=2 * C, C=C,
               ybf=yb, ybf_ld=ldm * 2 * C, csum=cs, csum_ld=ldm * 2 * C, keep_y=False)
        torch.cuda.synchronize()
        return yb, cs
    try:
        y0, c0 = run(False)
        y1, c1 = run(True)
    finally:
        L.call("ensvs_set_gbw_dma", 1)
    assert torch.equal(y0, y1) and torch.equal(c0, c1)
    assert (y1[:, 2 * C:] == 3.0).all() and (c1[:, 2 * C:] == 7.0).all()
    # and the values: d(gate), d(filter) of z = sigmoid(g) tanh(f) against float64
    g, f = gf.double()[:, :C], gf.double()[:, C:]
    dz = dx.double() @ w0.double()[:, :, 0].t() + dss.double() @ w1.double()[:, :, 0].t()
    sg, th = torch.sigmoid(g), torch.tanh(f)
    ref = torch.cat([dz * th * sg * (1 - sg), dz * sg * (1 - th * th)], 1)
    got = y1[:, :2 * C].double()
    assert ((got - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("C,B,T,bias", [(256, 3, 256, False), (128, 2, 384, True),
                                        (256, 30, 1024, False)])
def test_addscale_dma_epilogue_bitwise(C, B, T, bias):
    """The DiffNet dilated-conv dgrad (3-tap bf16 d(pre) segment, ADDSCALE: dx_l = dx_l+1 /
    sqrt 2 + dy, fp32 out + bf16 copy, per-tile column sums): the LDS-DMA epilogue equals the
    register one bit for bit."""
    torch.manual_seed(C + T + 1)
    M = B * T
    dpre = torch.randn(M, 2 * C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C, 2 * C, 3, device=DEV) / (6 * C) ** 0.5).to(torch.bfloat16).float()
    pb, (r,) = _pack([w])
    segs = [K.Seg(dpre, 2 * C, 2 * C, r, T, taps=3, dil=2, shift0=-2)]
    dx = torch.randn(M, C, device=DEV)
    b = torch.randn(C, device=DEV) if bias else None

    def run(on):
        L.call("ensvs_set_gbw_dma", int(on))
        y = torch.full((M, C), 5.0, device=DEV)
        yb = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
        kw = dict(epi=L.EPI_ADDSCALE, aux1=dx, ld1=C, alpha=0.7071, ybf=yb, ybf_ld=C)
        if b is None:
            cs = torch.full((M // 128, 3 * C), 7.0, device=DEV)
            kw.update(csum=cs, csum_ld=3 * C, csum_off=C)
        else:
            cs = None
            kw.update(bias=b)
        K.gemm(segs, B, T, C, pb, y, C, **kw)
        torch.cuda.synchronize()
        return y, yb, cs
    try:
        y0, b0, c0 = run(False)
        y1, b1, c1 = run(True)
    finally:
        L.call("ensvs_set_gbw_dma", 1)
    assert torch.equal(y0, y1) and torch.equal(b0, b1)
    if c0 is not None:
        assert torch.equal(c0, c1)
    assert torch.equal(b1, y1.to(torch.bfloat16))
