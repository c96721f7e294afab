"""Numerics of the MFMA implicit-GEMM engine against plain PyTorch fp32 ops."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from ensemble_svs_with_interactions_amd import kernels as K
from ensemble_svs_with_interactions_amd import _lib as L

DEV = "cuda"


def rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def pack(dtype, w, transpose=False, flip=False, perm_c=0, scale=1.0, src2=None):
    """w: Conv1d weight (N, K, taps)."""
    pb = K.PackedBuffer(dtype)
    N, Kc, taps = w.shape
    ref = pb.add(w, N, Kc, taps, Kc * taps, taps, 1, perm_c=perm_c, flip=flip,
                 transpose=transpose, scale=scale, src2=src2)
    pb.finalize(w.device)
    pb.repack()
    return pb, ref


@pytest.mark.parametrize("dt,tol", [(L.DT_F32, 2e-5), (L.DT_BF16, 2e-2)])
@pytest.mark.parametrize("taps,dil,pad", [(1, 1, L.PAD_ZERO), (7, 1, L.PAD_REFLECT),
                                          (3, 2, L.PAD_ZERO), (3, 4, L.PAD_REPLICATE)])
def test_conv_fwd(dt, tol, taps, dil, pad):
    torch.manual_seed(0)
    B, T, Cin, Cout = 3, 57, 70, 133
    x = torch.randn(B, T, Cin, device=DEV)
    w = torch.randn(Cout, Cin, taps, device=DEV) / (Cin * taps) ** 0.5
    b = torch.randn(Cout, device=DEV)
    half = (taps - 1) // 2 * dil
    mode = {L.PAD_ZERO: "constant", L.PAD_REFLECT: "reflect", L.PAD_REPLICATE: "replicate"}[pad]
    xp = F.pad(x.transpose(1, 2), (half, half), mode=mode)
    ref = F.conv1d(xp, w, b, dilation=dil).transpose(1, 2)
    pb, r = pack(dt, w)
    y = torch.empty(B, T, Cout, device=DEV)
    K.gemm([K.Seg(x, Cin, Cin, r, T, taps=taps, dil=dil, shift0=-half, pad=pad)], B, T, Cout,
           pb, y, Cout, bias=b)
    torch.cuda.synchronize()
    assert rel(y, ref) < tol


@pytest.mark.parametrize("dt,tol", [(L.DT_F32, 2e-5), (L.DT_BF16, 2e-2)])
def test_diffnet_gate_and_resskip(dt, tol):
    torch.manual_seed(1)
    B, T, C, E, dil = 2, 45, 64, 48, 2
    x = torch.randn(B, T, C, device=DEV)
    cond = torch.randn(B, T, E, device=DEV)
    d = torch.randn(B, C, device=DEV)
    wd = torch.randn(2 * C, C, 3, device=DEV) / (3 * C) ** 0.5
    bd = torch.randn(2 * C, device=DEV)
    wc = torch.randn(2 * C, E, 1, device=DEV) / E ** 0.5
    bc = torch.randn(2 * C, device=DEV)
    wo = torch.randn(2 * C, C, 1, device=DEV) / C ** 0.5
    bo = torch.randn(2 * C, device=DEV)
    # reference (denoiser.py ResidualBlock with pre-projected diffusion step d)
    y = x.transpose(1, 2) + d[:, :, None]
    yy = F.conv1d(y, wd, bd, padding=dil, dilation=dil) + F.conv1d(cond.transpose(1, 2), wc, bc)
    gate, filt = yy.chunk(2, dim=1)
    z = torch.sigmoid(gate) * torch.tanh(filt)
    o = F.conv1d(z, wo, bo)
    res, skip = o.chunk(2, dim=1)
    xn_ref = ((x.transpose(1, 2) + res) / 2 ** 0.5).transpose(1, 2)

    pb = K.PackedBuffer(dt)
    rd = pb.add(wd, 2 * C, C, 3, 3 * C, 3, 1, perm_c=C)
    rc = pb.add(wc, 2 * C, E, 1, E, 1, 1, perm_c=C)
    ro = pb.add(wo, 2 * C, C, 1, C, 1, 1, perm_c=C)
    pb.finalize(DEV)
    pb.repack()
    bb = K.PackedBuffer(L.DT_F32)
    rbg = bb.add(bd.view(-1, 1, 1), 2 * C, 1, 1, 1, 1, 1, perm_c=C, src2=bc.view(-1, 1, 1), kpad_to=1)
    rbo = bb.add(bo.view(-1, 1, 1), 2 * C, 1, 1, 1, 1, 1, perm_c=C, kpad_to=1)
    bb.finalize(DEV)
    bb.repack()

    Z = torch.empty(B, T, C, device=DEV)
    GF = torch.empty(B, T, 2 * C, device=DEV)
    K.gemm([K.Seg(x, C, C, rd, T, taps=3, dil=dil, shift0=-dil, radd=d, radd_ld=C),
            K.Seg(cond, E, E, rc, T)], B, T, 2 * C, pb, Z, C, bias=bb.buf, bias_off=rbg.offset,
           epi=L.EPI_GATE, aux0=GF, ld0=2 * C, C=C)
    skip_acc = torch.full((B, T, C), 0.5, device=DEV)
    xn = torch.empty(B, T, C, device=DEV)
    K.gemm([K.Seg(Z, C, C, ro, T)], B, T, 2 * C, pb, xn, C, bias=bb.buf, bias_off=rbo.offset,
           epi=L.EPI_RESSKIP, aux0=skip_acc, ld0=C, aux1=x, ld1=C, accum=True, C=C, alpha=1.0)
    torch.cuda.synchronize()
    assert rel(Z, z.transpose(1, 2)) < tol
    assert rel(GF[..., :C], gate.transpose(1, 2)) < tol
    assert rel(GF[..., C:], filt.transpose(1, 2)) < tol
    assert rel(xn, xn_ref) < tol
    assert rel(skip_acc, skip.transpose(1, 2) + 0.5) < tol


@pytest.mark.parametrize("dt,tol", [(L.DT_F32, 2e-5), (L.DT_BF16, 2e-2)])
def test_conv_dgrad_wgrad(dt, tol):
    torch.manual_seed(2)
    B, T, Cin, Cout, taps, dil = 2, 70, 36, 150, 3, 2
    x = torch.randn(B, T, Cin, device=DEV, requires_grad=True)
    w = (torch.randn(Cout, Cin, taps, device=DEV) / (Cin * taps) ** 0.5).requires_grad_()
    y = F.conv1d(x.transpose(1, 2), w, padding=dil, dilation=dil).transpose(1, 2)
    g = torch.randn(y.shape, device=DEV)
    y.backward(g)
    # dgrad: conv over g with flipped, transposed weights
    pb, r = pack(dt, w.detach(), transpose=True, flip=True)
    dx = torch.empty(B, T, Cin, device=DEV)
    K.gemm([K.Seg(g, Cout, Cout, r, T, taps=taps, dil=dil, shift0=-dil)], B, T, Cin, pb, dx, Cin)
    dw = torch.empty(Cout, Cin, taps, device=DEV)
    K.wgrad(g, Cout, x.detach(), Cin, B, T, T, Cout, Cin, taps, dil, -dil, L.PAD_ZERO, dw,
            Cin * taps, taps, 1, dtype=dt)
    torch.cuda.synchronize()
    assert rel(dx, x.grad) < tol
    assert rel(dw, w.grad) < tol


@pytest.mark.parametrize("dt,tol", [(L.DT_F32, 2e-5), (L.DT_BF16, 2e-2)])
def test_reflect_wgrad_and_full_dgrad(dt, tol):
    torch.manual_seed(3)
    B, T, Cin, Cout = 2, 40, 20, 24
    x = torch.randn(B, T, Cin, device=DEV, requires_grad=True)
    w = (torch.randn(Cout, Cin, 7, device=DEV) / (Cin * 7) ** 0.5).requires_grad_()
    y = F.conv1d(F.pad(x.transpose(1, 2), (3, 3), mode="reflect"), w).transpose(1, 2)
    g = torch.randn(y.shape, device=DEV)
    y.backward(g)
    dw = torch.empty(Cout, Cin, 7, device=DEV)
    K.wgrad(g, Cout, x.detach(), Cin, B, T, T, Cout, Cin, 7, 1, -3, L.PAD_REFLECT, dw,
            Cin * 7, 7, 1, dtype=dt)
    # full conv -> gradient of the padded input, then fold the reflection
    pb, r = pack(dt, w.detach(), transpose=True, flip=True)
    dxp = torch.empty(B, T + 6, Cin, device=DEV)
    K.gemm([K.Seg(g, Cout, Cout, r, T, taps=7, dil=1, shift0=-6)], B, T + 6, Cin, pb, dxp, Cin)
    torch.cuda.synchronize()
    ref_p = torch.zeros(B, T + 6, Cin, device=DEV)
    xp = F.pad(x.detach().transpose(1, 2), (3, 3), mode="reflect").requires_grad_()
    F.conv1d(xp, w.detach()).transpose(1, 2).backward(g)
    assert rel(dxp, xp.grad.transpose(1, 2)) < tol
    assert rel(dw, w.grad) < tol


def test_colsum_grouped():
    torch.manual_seed(4)
    y = torch.randn(3, 333, 70, device=DEV)
    out = torch.empty(3, 70, device=DEV)
    K.colsum(y, 70, 333, 70, out, groups=3)
    mean = y.reshape(-1, 70).mean(0)
    var = torch.empty(70, device=DEV)
    K.colsum(y, 70, 999, 70, var, mean=mean, scale=1.0 / 999)
    torch.cuda.synchronize()
    assert rel(out, y.sum(1)) < 1e-5
    assert rel(var, y.reshape(-1, 70).var(0, unbiased=False)) < 1e-5


@pytest.mark.parametrize("dt,tol", [(L.DT_F32, 2e-5), (L.DT_BF16, 2e-2)])
@pytest.mark.parametrize("splits", [1, 7])
def test_wgrad_radd_tiles_splits(dt, tol, splits):
    """Multi-tile wgrad (N, K not multiples of 128) of x + radd[b] with accumulate and
    scale, direct (splits=1) and split-reduced."""
    torch.manual_seed(5)
    B, T, Cin, Cout, taps, dil = 3, 96, 260, 300, 3, 4
    x = torch.randn(B, T, Cin, device=DEV)
    radd = torch.randn(B, Cin, device=DEV)
    xe = (x + radd[:, None, :]).requires_grad_()
    w = (torch.randn(Cout, Cin, taps, device=DEV) / (Cin * taps) ** 0.5).requires_grad_()
    y = F.conv1d(xe.transpose(1, 2), w, padding=dil, dilation=dil).transpose(1, 2)
    g = torch.randn(y.shape, device=DEV)
    y.backward(g)
    dw0 = torch.randn(Cout, Cin, taps, device=DEV)
    dw = dw0.clone()
    K.wgrad(g, Cout, x, Cin, B, T, T, Cout, Cin, taps, dil, -dil, L.PAD_ZERO, dw,
            Cin * taps, taps, 1, dtype=dt, radd=radd, radd_ld=Cin, accum=True, scale=0.5,
            splits=splits)
    torch.cuda.synchronize()
    assert rel(dw - dw0, 0.5 * w.grad) < tol


@pytest.mark.parametrize("shape", [(30, 1024, 64, 256, 1, 1, L.PAD_ZERO),
                                   (4, 333, 256, 512, 1, 1, L.PAD_ZERO),
                                   (3, 517, 128, 128, 7, 1, L.PAD_REFLECT),
                                   (5, 200, 256, 256, 3, 4, L.PAD_ZERO)])
@pytest.mark.parametrize("splits", [1, 5, None])
def test_wgrad_fp32_source_bitwise_equals_bf16_operands(shape, splits):
    """The fp32-operand weight gradient in production precision (rows rounded to bf16 while
    staged; the deep-prefetch ring kernel) gives the same bits as the bf16-operand kernel on
    pre-rounded copies (ensvs_cast_bf16), incl. ragged M, taps/padding and split reduction."""
    torch.manual_seed(11)
    B, T, Cin, Cout, taps, dil, pad = shape
    M = B * T
    x = torch.randn(M, Cin, device=DEV)
    g = torch.randn(M, Cout, device=DEV)
    outs = []
    for b16 in (False, True):
        dw = torch.full((Cout, Cin, taps), 0.25, device=DEV)
        xs, gs = (K.cast_bf16(x, Cin, Cin, M), K.cast_bf16(g, Cout, Cout, M)) if b16 else (x, g)
        K.wgrad(gs, Cout, xs, Cin, B, T, T, Cout, Cin, taps, dil, -dil * (taps // 2), pad, dw,
                Cin * taps, taps, 1, dtype=L.DT_BF16, accum=True, scale=0.5, splits=splits)
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = torch.einsum("mn,mk->nk", g.double(), x.double()).float() if taps == 1 else None
    if ref is not None:
        assert rel(outs[0][:, :, 0] - 0.25, 0.5 * ref) < 2e-2


@pytest.mark.parametrize("shape", [(30, 1024, 39, 256, 1, 1, L.PAD_ZERO),
                                   (30, 1024, 1, 128, 7, 1, L.PAD_ZERO),
                                   (30, 1024, 5, 128, 1, 1, L.PAD_ZERO),
                                   (7, 1097, 130, 1024, 1, 1, L.PAD_ZERO),
                                   (3, 517, 3, 64, 3, 2, L.PAD_REFLECT),
                                   (30, 1024, 128, 5, 1, 1, L.PAD_ZERO),
                                   (30, 1024, 128, 1, 1, 1, L.PAD_ZERO),
                                   (7, 1097, 130, 4, 1, 1, L.PAD_ZERO),
                                   (5, 700, 256, 60, 1, 1, L.PAD_ZERO)])
def test_wgrad_odd_channels_cast_route(shape):
    """fp32-operand weight gradients with K % 4 != 0 or N % 4 != 0 (kernels.WGRAD_CAST: bf16
    copies zero-padded to 8 channels, through the LDS-DMA kernel) against the register kernel
    they replace and a float64 reference, incl. taps with reflect padding and ragged M (N = 60:
    the vector kernel, unchanged)."""
    torch.manual_seed(12)
    B, T, Cin, Cout, taps, dil, pad = shape
    M = B * T
    x = torch.randn(M, Cin, device=DEV)
    g = torch.randn(M, Cout, device=DEV)
    outs = []
    try:
        for on in (False, True):
            K.WGRAD_CAST["on"] = on
            dw = torch.full((Cout, Cin, taps), 0.25, device=DEV)
            K.wgrad(g, Cout, x, Cin, B, T, T, Cout, Cin, taps, dil, -dil * (taps // 2), pad, dw,
                    Cin * taps, taps, 1, dtype=L.DT_BF16, accum=True, scale=0.5)
            outs.append(dw)
    finally:
        K.WGRAD_CAST["on"] = True
    torch.cuda.synchronize()
    assert rel(outs[1] - 0.25, outs[0] - 0.25) < 1e-5
    if taps == 1:
        ref = torch.einsum("mn,mk->nk", g.double(), x.double()).float()
        assert rel(outs[1][:, :, 0] - 0.25, 0.5 * ref) < 2e-2


def test_colsum_vectorized_tail():
    torch.manual_seed(6)
    y = torch.randn(5000, 128, device=DEV)
    out = torch.full((102,), 1.0, device=DEV)
    K.colsum(y, 128, 5000, 102, out, accum=True, scale=2.0)
    mean = y[:, :102].mean(0)
    var = torch.empty(102, device=DEV)
    K.colsum(y, 128, 5000, 102, var, mean=mean, scale=1.0 / 5000)
    grp = torch.empty(4, 102, device=DEV)
    K.colsum(y, 128, 1250, 102, grp, groups=4)
    torch.cuda.synchronize()
    assert rel(out, 1.0 + 2.0 * y[:, :102].sum(0)) < 1e-5
    assert rel(var, y[:, :102].var(0, unbiased=False)) < 1e-5
    assert rel(grp, y[:, :102].reshape(4, 1250, 102).sum(1)) < 1e-5


@pytest.mark.parametrize("M,ld,ph0,nv", [(3000, 96, 5, 60), (30720, 87, 0, 47), (100, 300, 10, 129),
                                         (65, 8, 1, 1)])
def test_phoneme_ids_argmax(M, ld, ph0, nv):
    """ensvs_phoneme_ids = torch.argmax over the phoneme columns (first maximum; ties and
    all-zero rows -> the first column): the LDS-tiled kernel (nv <= 128) and the per-row one."""
    from ensemble_svs_with_interactions_amd._lib import call
    torch.manual_seed(M + nv)
    x = torch.randn(M, ld, device=DEV)
    oh = torch.zeros(M, nv, device=DEV)
    oh[torch.arange(M, device=DEV), torch.randint(0, nv, (M,), device=DEV)] = 1.0
    oh[::7] = 0.0  # all-zero rows
    oh[3::11, : min(2, nv)] = 1.0  # ties
    x[:, ph0:ph0 + nv] = oh
    ids = torch.full((M,), -1, dtype=torch.int32, device=DEV)
    call("ensvs_phoneme_ids", x.data_ptr(), ld, M, ph0, nv, ids.data_ptr(), K.stream())
    torch.cuda.synchronize()
    assert torch.equal(ids.long(), torch.argmax(x[:, ph0:ph0 + nv], dim=1))


@pytest.mark.parametrize("M,C,T,ldy,off,two", [(30720, 256, 1024, 256, 0, True),
                                               (3000, 200, 300, 520, 3, False),
                                               (2048, 64, 512, 128, 64, True)])
def test_embed_add_rows(M, C, T, ldy, off, two):
    """ensvs_embed_add: Y[m] += emb[ids0[m]] (+ emb[ids1[m]]) + spk0[m / T] (+ spk1[m / T]),
    float4 lanes where aligned (off = 3: the scalar form), bitwise against torch in the same
    addition order."""
    from ensemble_svs_with_interactions_amd._lib import call
    torch.manual_seed(M + C)
    V, B = 47, M // T
    y = torch.randn(M, ldy, device=DEV)
    emb = torch.randn(V, C, device=DEV)
    ids0 = torch.randint(0, V, (M,), device=DEV, dtype=torch.int32)
    ids1 = torch.randint(0, V, (M,), device=DEV, dtype=torch.int32)
    spk = torch.randn(2, B, C + 4, device=DEV)
    ref = y.clone()
    r = ref[:, off:off + C]
    bt = torch.arange(M, device=DEV) // T
    r += emb[ids0.long()]
    if two:
        r += emb[ids1.long()]
    r += spk[0, :, :C][bt]
    if two:
        r += spk[1, :, :C][bt]
    call("ensvs_embed_add", y.data_ptr() + 4 * off, ldy, M, C, T, emb.data_ptr(), ids0.data_ptr(),
         ids1.data_ptr() if two else None, spk[0].data_ptr(), spk[1].data_ptr() if two else None,
         C + 4, K.stream())
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("n,off", [(23_501_237, 0), (23_501_237, 1), (1000, 0), (7, 0), (4, 1)])
def test_l2norm(n, off):
    """ensvs_l2norm / ensvs_l2norm_chk (the clip-by-global-norm of the fused Adam): float4
    form on aligned buffers (off = 0, any n: the n % 4 tail), the scalar one otherwise."""
    from ensemble_svs_with_interactions_amd._lib import call
    torch.manual_seed(n % 1000 + off)
    buf = torch.randn(n + off, device=DEV) * 1e-2
    x = buf[off:]
    part, out = torch.empty(1024, device=DEV), torch.empty(1, device=DEV)
    ref = torch.linalg.vector_norm(x.double()).item()
    for name, extra in (("ensvs_l2norm", ()), ("ensvs_l2norm_chk", (None,))):
        out.fill_(-1.0)
        call(name, x.data_ptr(), n, part.data_ptr(), out.data_ptr(), *extra, K.stream())
        torch.cuda.synchronize()
        assert abs(out.item() - ref) <= 2e-6 * ref, (name, out.item(), ref)


@pytest.mark.parametrize("M", [3000, 30720])
def test_embedding_and_speaker_backward_deterministic(M):
    """3 000 frames: 12 chunk partials (the reduce's tail loop); 30 720: 120 (its 16-wide
    batches)."""
    from ensemble_svs_with_interactions_amd._lib import call, query
    torch.manual_seed(7)
    C, V, ld = 200, 47, 208
    dy = torch.randn(M, ld, device=DEV)
    ids = torch.randint(0, V, (M,), device=DEV, dtype=torch.int32)
    outs = []
    for _ in range(2):
        demb = torch.ones(V, C, device=DEV)
        part = torch.empty(query("ensvs_embed_bwd_workspace", M, C, V), device=DEV)
        call("ensvs_embed_bwd", dy.data_ptr(), ld, M, C, ids.data_ptr(), V, part.data_ptr(),
             demb.data_ptr(), K.stream())
        outs.append(demb)
    ref = torch.ones(V, C, device=DEV).index_add_(0, ids.long(), dy[:, :C])
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert rel(outs[0], ref) < 1e-5
    B, R = 37, 5
    dseq = torch.randn(B, C, device=DEV)
    spk = torch.randint(0, R, (B,), device=DEV)
    tab = torch.full((R, C), 0.5, device=DEV)
    call("ensvs_spk_scatter", dseq.data_ptr(), B, C, spk.data_ptr(), tab.data_ptr(), K.stream())
    ref = torch.full((R, C), 0.5, device=DEV).index_add_(0, spk, dseq)
    torch.cuda.synchronize()
    assert rel(tab, ref) < 1e-6


@pytest.mark.parametrize("shape", [(30, 1024, 256, 512, 3, 4, L.PAD_ZERO),
                                   (3, 517, 264, 296, 1, 1, L.PAD_ZERO),
                                   (2, 333, 512, 256, 7, 1, L.PAD_REFLECT),
                                   (4, 250, 256, 10240, 1, 1, L.PAD_ZERO),
                                   (2, 300, 1032, 1016, 1, 1, L.PAD_ZERO),
                                   (3, 200, 520, 2048, 3, 2, L.PAD_ZERO)])
@pytest.mark.parametrize("splits", [1, 5, 21])
def test_wgrad_big_tile_bitwise(shape, splits):
    """bf16 weight gradients on the 256 x 256-tile kernel (shapes with >= 16 of its tiles)
    equal the 128 x 128 kernel's bits for the same split count (ragged N / K / M, taps,
    padding, direct and split-reduced); other shapes run the 128 x 128 kernel either way."""
    torch.manual_seed(13)
    B, T, Cin, Cout, taps, dil, pad = shape
    M = B * T
    xs = K.cast_bf16(torch.randn(M, Cin, device=DEV), Cin, Cin, M)
    gs = K.cast_bf16(torch.randn(M, Cout, device=DEV), Cout, Cout, M)
    outs = []
    try:
        for big in (False, True):
            L.call("ensvs_set_wgrad_big", int(big))
            dw = torch.full((Cout, Cin, taps), 0.25, device=DEV)
            K.wgrad(gs, Cout, xs, Cin, B, T, T, Cout, Cin, taps, dil, -dil * (taps // 2), pad, dw,
                    Cin * taps, taps, 1, dtype=L.DT_BF16, accum=True, scale=0.5, splits=splits)
            outs.append(dw)
        torch.cuda.synchronize()
    finally:
        L.call("ensvs_set_wgrad_big", 1)
    assert torch.equal(outs[0], outs[1])
    if taps == 1:
        ref = torch.einsum("mn,mk->nk", gs.double(), xs.double())
        assert rel(outs[1][:, :, 0].double() - 0.25, 0.5 * ref) < 1e-5
