"""Relative-position attention kernels (attention.hip; nnsvs/transformer/attentions.py:86-214)
one at a time against float64 torch restatements, at the shapes the encoder meets: T below
and above 64-multiples (the register-row softmax kernels take ceil(T / 64) <= 32 columns per
lane), dk with and without float4 runs, several lengths per batch, with and without the
dropout keep-mask.  tests/test_transformer.py checks the whole encoder against the oracle and
the reference's goldens."""
import pytest
import torch

from ensemble_svs_with_interactions_amd._lib import call

pytestmark = pytest.mark.gpu
W = 4


def _band(T):
    i = torch.arange(T)[:, None]
    j = torch.arange(T)[None, :]
    r = j - i + W
    return r, (r >= 0) & (r <= 2 * W)


def _setup(B, H, T, dk, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    C = H * dk
    lens = torch.tensor([T - 7 * b for b in range(B)], device="cuda", dtype=torch.int64)
    qs = torch.randn(B * T, C, device="cuda", generator=g)
    ek = torch.randn(2 * W + 1, dk, device="cuda", generator=g)
    S = torch.randn(B, H, T, T, device="cuda", generator=g)
    keep = (torch.rand(B, H, T, T, device="cuda", generator=g) > 0.2).float() / 0.8
    return g, C, lens, qs, ek, S, keep


def _st():
    return torch.cuda.current_stream().cuda_stream


CASES = [(2, 2, 37, 12), (2, 2, 130, 96), (3, 2, 1000, 96), (1, 2, 1024, 128), (1, 1, 2100, 8)]


@pytest.mark.parametrize("B,H,T,dk", CASES)
@pytest.mark.parametrize("drop", [False, True])
def test_softmax_fwd_bwd(B, H, T, dk, drop):
    g, C, lens, qs, ek, S, keep = _setup(B, H, T, dk, T + dk)
    r, band = _band(T)
    q = qs.double().view(B, T, H, dk).transpose(1, 2)                     # (B, H, T, dk)
    logits = q @ ek.double().t()                                            # (B, H, T, 2W+1)
    rel = torch.where(band.cuda(), torch.gather(logits, 3, r.clamp(0, 2 * W).cuda().expand(B, H, T, T)),
                      torch.zeros((), dtype=torch.float64, device="cuda"))
    valid = torch.arange(T, device="cuda")[None, :] < lens[:, None]
    mask = valid[:, None, :, None] & valid[:, None, None, :]
    sc = (S.double() + rel).masked_fill(~mask, -1e4)
    P = torch.softmax(sc, -1)
    Sk = S.clone()
    Pd = torch.empty_like(S) if drop else None
    kp = keep if drop else None
    call("ensvs_attn_softmax", Sk.data_ptr(), qs.data_ptr(), C, ek.data_ptr(),
                lens.data_ptr(), B, H, T, dk, W, kp.data_ptr() if drop else 0,
                Pd.data_ptr() if drop else 0, _st())
    torch.cuda.synchronize()
    assert (Sk.double() - P).abs().max().item() < 5e-6
    if drop:
        assert (Pd.double() - P * keep.double()).abs().max().item() < 5e-6
    # backward: dS = P (g - sum_j P g), g = dPd * keep; no gradient where masked
    dPd = torch.randn(B, H, T, T, device="cuda", generator=g)
    gg = dPd.double() * (keep.double() if drop else 1.0)
    ref = (P * (gg - (P * gg).sum(-1, keepdim=True))).masked_fill(~mask, 0.0)
    dS = dPd.clone()
    call("ensvs_attn_softmax_bwd", dS.data_ptr(), Sk.data_ptr(),
                kp.data_ptr() if drop else 0, lens.data_ptr(), B, H, T, _st())
    torch.cuda.synchronize()
    assert (dS.double() - ref).abs().max().item() < 1e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("B,H,T,dk", CASES)
def test_band_dot_and_table_grad(B, H, T, dk):
    g, C, lens, qs, ek, S, keep = _setup(B, H, T, dk, 7 * T + dk)
    r, band = _band(T)
    rc, bd = r.clamp(0, 2 * W).cuda(), band.cuda()
    vec = qs.double().view(B, T, H, dk).transpose(1, 2)
    # band_dot: D[row][i + r - w] += vec_i . tab[r]
    dots = vec @ ek.double().t()
    ref = S.double() + torch.where(bd, torch.gather(dots, 3, rc.expand(B, H, T, T)),
                                   torch.zeros((), dtype=torch.float64, device="cuda"))
    D = S.clone()
    call("ensvs_attn_band_dot", D.data_ptr(), qs.data_ptr(), C, ek.data_ptr(), B, H, T,
                dk, W, _st())
    torch.cuda.synchronize()
    assert (D.double() - ref).abs().max().item() < 1e-5 * ref.abs().max().item()
    # table grad: out[r][d] = sum_{b, h, i} A[b, h, i, i + r - w] X[b, i, h, d]
    A = S.double()
    pw = torch.zeros(B, H, T, 2 * W + 1, dtype=torch.float64, device="cuda")
    pw = pw.scatter_add(3, rc.expand(B, H, T, T), torch.where(bd, A, torch.zeros((), dtype=A.dtype,
                                                                                     device="cuda")))
    tref = torch.einsum("bhir,bhid->rd", pw, vec)
    from ensemble_svs_with_interactions_amd import _lib
    part = torch.empty(_lib.query("ensvs_attn_table_grad_workspace", dk, W), device="cuda")
    out = torch.full((2 * W + 1, dk), 3.0, device="cuda")
    call("ensvs_attn_table_grad", S.data_ptr(), qs.data_ptr(), C, B, H, T, dk, W,
                part.data_ptr(), out.data_ptr(), 1, _st())
    torch.cuda.synchronize()
    assert (out.double() - 3.0 - tref).abs().max().item() < 1e-5 * tref.abs().max().item()
