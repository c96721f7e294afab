"""Drop-in boundary on MI355X: the reference's train_step arithmetic, written with torch ops
exactly as nnsvs/bin/train_acoustic_multitrack.py:92-184 and 296-380 does it, on top of the
model's public forward(x_main, x_sub, spks_list, lengths, ys) and autograd, gives the same
loss and gradients as the fused train_step (both recipes: plain and interaction loss).

This is the path a reference user takes after swapping `_target_` strings: the
autograd.Function backward runs the HIP backward kernels and accumulates into .grad.
"""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, engine
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step
from golden_util import load_case
from gpu_util import build

pytestmark = pytest.mark.gpu


def _draws(a, B, T):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(a["draw0::" + k])).cuda()  # noqa: E731
    return dict(lf0_main=t("lf0_main").view(-1).contiguous(),
                lf0_sub=t("lf0_sub").view(-1).contiguous(), mgc_t=t("mgc_t"), bap_t=t("bap_t"),
                mgc_noise=t("mgc_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1),
                bap_noise=t("bap_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1))


def _reference_style_loss(model, xm, xs, ym, ys, spks, lengths, w_il, stream_sizes):
    """train_acoustic_multitrack.py:92-184, 289-298 (feats_criterion l1, no pitch reg)."""
    outs = model(xm, xs, spks_list=spks, lengths=lengths, ys=[ym, ys])
    (pred_main, _), (pred_sub, _) = outs
    mask = (torch.arange(ym.shape[1], device=ym.device)[None, :] < lengths[:, None]).unsqueeze(-1)
    crit = torch.nn.L1Loss(reduction="none")
    splits = lambda y: torch.split(y, stream_sizes, dim=-1)  # noqa: E731
    streams_main, streams_sub = splits(ym), splits(ys)
    loss_feats, N = 0, 0
    for pred, stream in zip(pred_main, streams_main):
        if isinstance(pred, tuple):
            noise, x_recon = pred
            l_ = crit(noise.masked_select(mask), x_recon.masked_select(mask))
        else:
            l_ = crit(pred.masked_select(mask), stream.masked_select(mask))
        loss_feats = loss_feats + l_.sum()
        N += len(l_.view(-1))
    loss = loss_feats / N
    if w_il > 0:
        vuv_flag = (streams_main[2] > 0) & (streams_sub[2] > 0)
        pred_diff = pred_main[1] - pred_sub[1]
        diff = streams_main[1] - streams_sub[1]
        loss = loss + w_il * crit(pred_diff.masked_select(mask & vuv_flag),
                                  diff.masked_select(mask & vuv_flag)).mean()
    return loss


@pytest.mark.parametrize("case", ["train_step_tiny", "train_step_tiny_il"])
def test_reference_style_step_equals_fused(case):
    engine.set_gemm_precision("fp32")
    a, meta = load_case(case)
    w_il = meta.get("logf0_diff_weight", 0.0)
    cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True, output_subtrack=w_il > 0)
    g = lambda k: torch.from_numpy(a[k]).cuda().contiguous()  # noqa: E731
    xm, xs, ym, ys, s0, s1 = g("x_main"), g("x_sub"), g("y_main"), g("y_sub"), g("spk_main"), \
        g("spk_sub")
    lengths = torch.from_numpy(a["lengths"]).cuda()
    B, T = xm.shape[:2]
    draws = _draws(a, B, T)
    results = []
    for fused in (False, True):
        model = build(cfg, meta["shapes"])
        model.vuv_model.lstm.dropout = 0.0
        opt = FusedAdam(model, lr=meta["lr"])
        if fused:
            loss, _ = train_step(model, opt, xm, xs, ym, s0, s1, a["lengths"].tolist(),
                                 draws=draws, y_sub=ys, logf0_diff_weight=w_il)
        else:
            model.train()
            opt.zero_grad()
            model._replay_draws = draws
            loss = _reference_style_loss(model, xm, xs, ym, ys, (s0, s1), lengths, w_il,
                                         cfg["stream_sizes"])
            loss.backward()
        torch.cuda.synchronize()
        results.append((loss.item(), opt.gflat.clone()))
    (l_ref, g_ref), (l_fused, g_fused) = results
    assert abs(l_ref - meta["losses"][0]) < 1e-5 * abs(meta["losses"][0])
    assert abs(l_fused - l_ref) <= 1e-6 * abs(l_ref)
    err = ((g_fused - g_ref).norm() / g_ref.norm()).item()
    assert err < 1e-5, err


def test_reference_step_amp_gradscaler_equals_fused():
    """The reference's own step shape (train_acoustic_multitrack.py:93-184, 358-380):
    prediction_type() dispatch, fp16 autocast around the forward, GradScaler scale ->
    backward -> unscale_ -> clip_grad_norm_ -> step -> update, torch.optim.Adam.  Parameter
    gradients come back through autograd (Function.backward returns them), so GradScaler
    and clip_grad_norm_ see them; the result equals the fused step."""
    from ensemble_svs_with_interactions_amd.base import PredictionType
    engine.set_gemm_precision("fp32")
    a, meta = load_case("train_step_tiny")
    cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True)
    g = lambda k: torch.from_numpy(a[k]).cuda().contiguous()  # noqa: E731
    xm, xs, ym, ys, s0, s1 = g("x_main"), g("x_sub"), g("y_main"), g("y_sub"), g("spk_main"), \
        g("spk_sub")
    lengths = torch.from_numpy(a["lengths"]).cuda()
    B, T = xm.shape[:2]
    draws = _draws(a, B, T)
    lr = meta["lr"]

    # reference-style
    model = build(cfg, meta["shapes"])
    model.vuv_model.lstm.dropout = 0.0
    p0 = {k: v.detach().clone() for k, v in model.named_parameters()}
    opt = torch.optim.Adam(model.parameters(), lr=lr, betas=(0.9, 0.999), weight_decay=0.0)
    scaler = torch.amp.GradScaler("cuda")
    model.train()
    opt.zero_grad()
    model._replay_draws = draws
    assert model.prediction_type() == PredictionType.MULTISTREAM_HYBRID
    with torch.autocast("cuda", dtype=torch.float16):
        loss = _reference_style_loss(model, xm, xs, ym, ys, (s0, s1), lengths, 0.0,
                                     cfg["stream_sizes"])
    scaler.scale(loss).backward()
    scaler.unscale_(opt)
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    scaler.step(opt)
    scaler.update()
    torch.cuda.synchronize()
    assert all(v is not None for v in grads.values())
    after_ref = {k: v.detach().clone() for k, v in model.named_parameters()}

    # fused
    model2 = build(cfg, meta["shapes"])
    model2.vuv_model.lstm.dropout = 0.0
    opt2 = FusedAdam(model2, lr=lr)
    loss2, norm2 = train_step(model2, opt2, xm, xs, ym, s0, s1, a["lengths"].tolist(),
                              draws=draws)
    torch.cuda.synchronize()
    assert abs(loss.item() - loss2.item()) <= 1e-6 * abs(loss2.item())
    assert abs(gn.item() - norm2.item()) <= 1e-5 * norm2.item()
    g2 = {k: p.grad.detach() for k, p in model2.named_parameters()}
    num = sum(((grads[k] - g2[k]) ** 2).sum().item() for k in grads) ** 0.5
    den = sum((g2[k] ** 2).sum().item() for k in grads) ** 0.5
    assert num / den < 1e-5, num / den
    bad = []
    for k, p in model2.named_parameters():
        d_ref = after_ref[k] - p0[k]
        d_f = p.detach() - p0[k]
        gk = g2[k].abs()
        err = (d_ref - d_f).abs().masked_fill(gk < 1e-7 * (1.0 + gk.max()), 0.0)
        if (err > 0.1 * lr).float().mean().item() > 0.02:
            bad.append(k)
    assert not bad, bad[:5]
