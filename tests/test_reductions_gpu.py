"""Launch-count reductions of the training step's partial sums.

* ensvs_colsum_once -- the column sums (bias gradients, BatchNorm statistics, per-sequence sums)
  in one launch, the last block of each column block reducing the split partials -- returns the
  bits of the two-launch ensvs_colsum (partial + final kernels), for plain and centred sums,
  groups, accumulation and ragged column counts, and leaves its ticket counters at zero.
* kernels.deferred_wgrad -- split weight gradients whose reductions are queued and issued as
  one ensvs_wgrad_reduce_batch launch -- returns the bits of the immediate reductions,
  overlapping destinations included (the queue flushes before an overlapping one).
"""
import pytest
import torch

from ensemble_svs_with_interactions_amd import _lib as L
from ensemble_svs_with_interactions_amd import kernels as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,groups,centred,accum", [
    (30720, 256, 1, False, False), (30720, 256, 1, True, False), (1024, 128, 30, False, True),
    (1024, 128, 30, True, False), (3000, 61, 1, False, True), (512, 1000, 4, False, False),
    (200, 67, 1, False, False), (100, 5, 3, True, True)])
def test_colsum_once_bitwise(M, N, groups, centred, accum):
    torch.manual_seed(M + N)
    y = torch.randn(groups * M, N + 3, device=DEV)
    ld = N + 3
    mean = torch.randn(groups, N, device=DEV) * 0.1 if centred else None
    max_splits = max(1, min(256, M // 128, -(-2048 // (-(-N // 64) * groups))))
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for once in (False, True):
        out = torch.full((groups, N + 1), 0.5, device=DEV)
        part = torch.empty(groups * max_splits * N, device=DEV)
        if once:
            cnt = torch.zeros(-(-N // 64) * groups, dtype=torch.int32, device=DEV)
            for _ in range(2):  # the counters are left zero: a second launch works as well
                o2 = out.clone()
                L.call("ensvs_colsum_once", y.data_ptr(), ld, M, groups, N, L.ptr(mean), 0.75,
                       part.data_ptr(), max_splits, cnt.data_ptr(), o2.data_ptr(), N + 1,
                       int(accum), st)
            torch.cuda.synchronize()
            assert int(cnt.abs().max()) == 0
            outs.append(o2)
        else:
            L.call("ensvs_colsum", y.data_ptr(), ld, M, groups, N, L.ptr(mean), 0.75,
                   part.data_ptr(), max_splits, out.data_ptr(), N + 1, int(accum), st)
            outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    yy = y.view(groups, M, ld)[:, :, :N].double()
    if centred:
        yy = (yy - mean.double()[:, None, :]) ** 2
    ref = 0.75 * yy.sum(1) + (0.5 if accum else 0.0)
    assert torch.allclose(outs[1][:, :N].double(), ref, rtol=1e-5, atol=1e-4)


def test_deferred_wgrad_batch_bitwise():
    torch.manual_seed(3)
    shapes = [(4, 1000, 256, 256, 3, 2), (2, 2048, 512, 128, 1, 1), (30, 256, 128, 192, 7, 1),
              (3, 600, 64, 40, 1, 1)]
    srcs = []
    for B, T, N, Kc, taps, dil in shapes:
        dy = K.cast_bf16(torch.randn(B * T, N, device=DEV), N, N, B * T)
        x = K.cast_bf16(torch.randn(B * T, Kc, device=DEV), Kc, Kc, B * T)
        srcs.append((B, T, N, Kc, taps, dil, dy, x))
    res = []
    for defer in (False, True):
        dsts = [torch.full((N, Kc, taps), 0.25, device=DEV) for (_, _, N, Kc, taps, _, _, _)
                in srcs]
        shared = torch.full((srcs[0][2], srcs[0][3], srcs[0][4]), 0.125, device=DEV)
        with K.deferred_wgrad():
            for (B, T, N, Kc, taps, dil, dy, x), d in zip(srcs, dsts):
                K.wgrad(dy, N, x, Kc, B, T, T, N, Kc, taps, dil, -dil * (taps // 2),
                        L.PAD_ZERO, d, Kc * taps, taps, 1, accum=True, scale=0.5, defer=defer)
            # two contributions into one destination: the queue flushes in between
            B, T, N, Kc, taps, dil, dy, x = srcs[0]
            for sc in (1.0, -0.5):
                K.wgrad(dy, N, x, Kc, B, T, T, N, Kc, taps, dil, -dil * (taps // 2), L.PAD_ZERO,
                        shared, Kc * taps, taps, 1, accum=True, scale=sc, defer=defer)
        torch.cuda.synchronize()
        res.append(dsts + [shared])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_colsum_batch_bitwise():
    """ensvs_colsum_batch (the deferred bias gradients): each descriptor's sums carry the bits
    of one ensvs_colsum with the same max_splits, accumulation and scale included, over row
    counts / widths / strides / alignments a step issues (and a ragged one)."""
    torch.manual_seed(9)
    specs = [(30720, 256, 256, 0), (30720, 128, 131, 0), (1024, 512, 512, 0), (200, 67, 70, 1),
             (30720, 5, 8, 0), (30, 1024, 1024, 0), (3000, 61, 64, 3)]
    st = torch.cuda.current_stream().cuda_stream
    outs, descs, keep = [], [], []
    for M, N, ld, yoff in specs:
        y = torch.randn(M * ld + yoff, device=DEV)
        out = torch.full((N,), 0.5, device=DEV)
        ref = out.clone()
        ms = max(1, min(256, M // 128, -(-2048 // (-(-N // 64)))))
        part = torch.empty(ms * N, device=DEV)
        L.call("ensvs_colsum", y.data_ptr() + 4 * yoff, ld, M, 1, N, None, 0.75, part.data_ptr(),
               ms, ref.data_ptr(), 0, 1, st)
        descs.append(K.ColsumDesc(y.data_ptr() + 4 * yoff, out.data_ptr(), ld, M, N, ms, 0.75, 1))
        outs.append((out, ref))
        keep.append(y)
    import ctypes
    arr = (K.ColsumDesc * len(descs))(*descs)
    nf = L.query("ensvs_colsum_batch_part_floats", ctypes.addressof(arr), len(descs))
    part = torch.empty(nf, device=DEV)
    L.call("ensvs_colsum_batch", ctypes.addressof(arr), len(descs), part.data_ptr(), nf, st)
    torch.cuda.synchronize()
    for out, ref in outs:
        assert torch.equal(out, ref)


@pytest.mark.parametrize("prec", ["bf16", "fp32"])
def test_deferred_colsum_train_step_bitwise(prec):
    """A training step with the bias-gradient column sums deferred and batched per branch
    (kernels.DEFER_COLSUM) leaves the bits of the step with one ensvs_colsum per bias:
    loss, gradient norm, every parameter and Adam moment."""
    import numpy as np
    from ensemble_svs_with_interactions_amd import configs, data, engine
    from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step
    engine.set_gemm_precision(prec)
    try:
        P, T = 4, 128
        b = data.synthetic_batch(P, T, 5)
        g = lambda k: torch.from_numpy(b[k]).cuda().contiguous()  # noqa: E731
        args = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
                b["lengths"].tolist())
        gen = torch.Generator(device=DEV).manual_seed(1)
        res = []
        for on in (True, False):
            K.DEFER_COLSUM["on"] = on
            try:
                torch.manual_seed(0)
                m = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).cuda()
                m.vuv_model.lstm.dropout = 0.0
                opt = FusedAdam(m)
                nm, nb = m.stream_sizes[0], m.stream_sizes[3]
                gen.manual_seed(1)
                draws = dict(
                    lf0_main=(torch.rand(P * T // 4, device=DEV, generator=gen) < .5).float() * 2,
                    lf0_sub=(torch.rand(P * T // 4, device=DEV, generator=gen) < .5).float() * 2,
                    mgc_t=torch.randint(0, 100, (P,), device=DEV, generator=gen),
                    bap_t=torch.randint(0, 100, (P,), device=DEV, generator=gen),
                    mgc_noise=torch.randn(P * T, nm, device=DEV, generator=gen),
                    bap_noise=torch.randn(P * T, nb, device=DEV, generator=gen))
                loss, norm = train_step(m, opt, *args, draws=draws)
                torch.cuda.synchronize()
                res.append((loss.clone(), norm.clone(), opt.flat.clone(), opt.gflat.clone(),
                            opt.m.clone(), opt.v.clone()))
            finally:
                K.DEFER_COLSUM["on"] = True
        for a, b_ in zip(*res):
            assert torch.equal(a, b_)
        assert np.isfinite(res[0][0].item())
    finally:
        engine.set_gemm_precision("bf16")


@pytest.mark.parametrize("M,C,G,ld,updates", [
    (30720, 128, 1, 128, 1), (30720, 256, 2, 256, 2), (30720, 512, 1, 512, 0),
    (2000, 60, 1, 61, 1),  # unaligned rows: the scalar loads
    (1000, 1024, 2, 1024, 1), (100, 8, 1, 8, 1),
])
def test_bn_stats_matches_two_pass(M, C, G, ld, updates):
    """ensvs_bn_stats (split sums / deviations, Chan merge in double) against the two-pass
    form it replaces (two column sums + ensvs_bn_finalize, `updates` calls): mean and variance
    within 1e-6 / 1e-5 relative of the two-pass values, rstd and running statistics likewise,
    num_batches_tracked advanced by G * updates."""
    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(M + C)
    y = (torch.randn(M, ld, device=dev, generator=g) * 3.0 + 5.0)  # |mean| >> std per column
    Mg = M // G
    eps, mom = 1e-5, 0.1
    rm0 = torch.randn(C, device=dev, generator=g)
    rv0 = torch.rand(C, device=dev, generator=g) + 0.5
    # two-pass reference
    mean_r, var_r, rstd_r = (torch.empty(G, C, device=dev) for _ in range(3))
    K.colsum(y, ld, Mg, C, mean_r, groups=G, scale=1.0 / Mg)
    K.colsum(y, ld, Mg, C, var_r, groups=G, mean=mean_r, scale=1.0 / Mg)
    rm_r, rv_r = rm0.clone(), rv0.clone()
    for _ in range(max(1, updates)):
        L.call("ensvs_bn_finalize", mean_r.data_ptr(), var_r.data_ptr(), G, C, Mg, eps,
               rstd_r.data_ptr(), rm_r.data_ptr(), rv_r.data_ptr(), mom, int(updates > 0), st)
    # fused
    n = L.query("ensvs_bn_stats_part_floats", M, C, Mg)
    part = torch.full((n,), float("nan"), device=dev)
    mean, var, rstd = (torch.full((G, C), float("nan"), device=dev) for _ in range(3))
    rm, rv = rm0.clone(), rv0.clone()
    nbt = torch.tensor([7], dtype=torch.int64, device=dev)
    L.call("ensvs_bn_stats", y.data_ptr(), ld, M, C, Mg, part.data_ptr(), n, eps, mean.data_ptr(),
           var.data_ptr(), rstd.data_ptr(), rm.data_ptr() if updates else None,
           rv.data_ptr() if updates else None, mom, updates, nbt.data_ptr() if updates else None,
           st)
    torch.cuda.synchronize()

    def close(a, b, tol):
        return ((a.double() - b.double()).abs().max() / b.double().abs().max()).item() <= tol

    assert close(mean, mean_r, 1e-6) and close(var, var_r, 1e-5) and close(rstd, rstd_r, 1e-5)
    if updates:
        assert close(rm, rm_r, 1e-6) and close(rv, rv_r, 1e-5)
        assert nbt.item() == 7 + G * updates
    else:
        assert torch.equal(rm, rm0) and torch.equal(rv, rv0)
