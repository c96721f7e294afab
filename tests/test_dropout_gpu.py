"""LSTM inter-layer dropout of the V/UV model on MI355X: mask replay vs the oracle.

The recipe sets ``dropout: 0.1`` on ``vuv_model`` (multitrack_acoustic_nnsvs_world_multi_
ar_f0_diff_mgcbap.yaml:188), so nn.LSTM(dropout=0.1) (nnsvs/model.py:862-869) scales the
first layer's output by a keep mask in training.  The reference draws that mask inside
torch's C++ LSTM, which cannot be replayed, so the goldens run it at p = 0; here the HIP
path's own masks (Ly.dropout_mask, captured) are replayed through the oracle's
``bilstm(..., layer_dropout_masks=...)`` at the fp32 tolerances, for the encoder at full
width (forward + every gradient) and for the whole fused training step.
"""
import numpy as np
import pytest
import torch

from oracle import ensvs_oracle as O
from ensemble_svs_with_interactions_amd import configs, engine
from ensemble_svs_with_interactions_amd import layers as Ly
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step
from golden_util import (load_case, full_shapes, params_from_shapes, rel, rel_l2, _pre_bn_bias,
                         record_errors)
from gpu_util import build
from test_encoders_gpu import relu_masks_from

pytestmark = pytest.mark.gpu
P_DROP = 0.1


class _Spy:
    """Records every mask Ly.dropout_mask hands out."""

    def __init__(self):
        self.masks = []
        self.real = Ly.dropout_mask

    def __enter__(self):
        def spy(n, p, device):
            m = self.real(n, p, device)
            self.masks.append((p, m))
            return m
        Ly.dropout_mask = spy
        return self

    def __exit__(self, *exc):
        Ly.dropout_mask = self.real


def test_dropout_mask_statistics():
    """Keep masks of F.dropout(p): values in {0, 1/(1-p)}, keep rate 1-p, fresh per draw."""
    n = 1 << 22
    a = Ly.dropout_mask(n, P_DROP, "cuda")
    b = Ly.dropout_mask(n, P_DROP, "cuda")
    torch.cuda.synchronize()
    scale = torch.tensor(1.0 / (1.0 - P_DROP), dtype=torch.float32)
    for m in (a, b):
        vals = torch.unique(m.cpu())
        assert set(vals.tolist()) <= {0.0, scale.item()}
        keep = (m > 0).float().mean().item()
        assert abs(keep - (1 - P_DROP)) < 5 * (P_DROP * (1 - P_DROP) / n) ** 0.5
    assert not torch.equal(a, b)


def test_vuv_encoder_dropout_replay_full_width():
    """V/UV FFConvLSTM at recipe width, train mode, p = 0.1: the default path draws one mask
    per inter-layer boundary; forward and every gradient equal the oracle replaying it."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("ffconvlstm_vuv")
    cfg = dict(configs.multitrack_diffusion(num_speakers=4)["vuv_model"])
    mod = build(cfg, full_shapes(), meta["prefix"])
    mod.train()
    mod.lstm.dropout = P_DROP
    P0 = {k: v.detach().cpu().clone() for k, v in mod.state_dict().items()}
    x = torch.from_numpy(a["x"]).cuda()
    B, T = x.shape[:2]
    H2 = 2 * mod.lstm.hidden_size
    spk = torch.from_numpy(a["spk"]).cuda().expand(B, T, -1)
    lens = torch.tensor(a["lengths"].tolist(), device="cuda")
    with _Spy() as spy:
        out, st = mod._fwd([(x, x.shape[2], 0, x.shape[2])], B, T, lens, spk, spk.stride(0))
    assert len(spy.masks) == mod.lstm.num_layers - 1 and spy.masks[0][0] == P_DROP
    R = torch.from_numpy(a["R"]).cuda().reshape(B * T, -1).contiguous()
    dX0, dspk = mod._bwd(st, R, want_spk=True)
    torch.cuda.synchronize()
    masks = [m.cpu().view(B, T, H2) for _, m in spy.masks]
    assert (masks[0] == 0).any()
    Pg = {k: (v.clone() if "running" in k else v.clone().requires_grad_())
          for k, v in P0.items() if v.dtype == torch.float32}
    spk_c = torch.from_numpy(a["spk"]).requires_grad_()
    oc = O.ffconvlstm(Pg, "", cfg, torch.from_numpy(a["x"]), a["lengths"],
                      spk_c.expand(B, T, -1), training=True,
                      lstm_dropout_masks=masks, relu_masks=relu_masks_from(st, B, T))
    assert rel(out.cpu().view(B, T, -1)[:, :oc.shape[1]], oc.detach()) < 1e-4
    # the dropout is live: without the mask the output differs
    o0 = O.ffconvlstm({k: v.detach() for k, v in Pg.items()}, "", cfg,
                      torch.from_numpy(a["x"]), a["lengths"], spk_c.detach().expand(B, T, -1),
                      training=True, bn_updates={})
    assert rel(o0, oc.detach()) > 1e-3
    (oc * torch.from_numpy(a["R"])[:, :oc.shape[1]]).sum().backward()
    assert rel(dspk.cpu(), spk_c.grad.view(B, -1)) < 1e-4
    for k, p in mod.named_parameters():
        if _pre_bn_bias(k):
            continue  # analytically zero (conv bias before training-mode BatchNorm)
        assert rel(p.grad.cpu(), Pg[k].grad) < 2e-4, k


def test_train_step_with_vuv_dropout_matches_oracle():
    """The fused training step (tiny widths) with V/UV LSTM dropout 0.1 and injected masks:
    loss, grad norm and every parameter gradient vs the oracle step replaying the same
    masks (train_acoustic_multitrack.py:40-392 around multistream.py:1594-1768)."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("train_step_tiny")
    cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True)
    model = build(cfg, meta["shapes"])
    model.vuv_model.lstm.dropout = P_DROP
    opt = FusedAdam(model, lr=meta["lr"])
    g = lambda k: torch.from_numpy(a[k]).cuda().contiguous()  # noqa: E731
    xm, xs, ym, s0, s1 = g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub")
    lens = a["lengths"].tolist()
    B, T = xm.shape[:2]
    H2 = 2 * model.vuv_model.lstm.hidden_size
    rng = np.random.default_rng(7)
    keep = (rng.random((B, T, H2)) >= P_DROP).astype(np.float32) / np.float32(1 - P_DROP)
    d = lambda k: torch.from_numpy(np.ascontiguousarray(a["draw0::" + k])).cuda()  # noqa: E731
    draws = dict(lf0_main=d("lf0_main").view(-1).contiguous(),
                 lf0_sub=d("lf0_sub").view(-1).contiguous(), mgc_t=d("mgc_t"),
                 bap_t=d("bap_t"),
                 mgc_noise=d("mgc_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1),
                 bap_noise=d("bap_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1),
                 vuv_lstm=[torch.from_numpy(keep).cuda().view(-1).contiguous()])
    loss, norm = train_step(model, opt, xm, xs, ym, s0, s1, lens, draws=draws)
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu() for k, p in model.named_parameters()}
    # oracle step with the same draws
    P = params_from_shapes(meta["shapes"])
    trainable = [k for k in P if "running" not in k and k.rsplit(".", 1)[-1] not in
                 O.diffusion_schedule()]
    for k in trainable:
        P[k].requires_grad_()
    T_ = torch.from_numpy
    od = dict(lf0_main=T_(a["draw0::lf0_main"]), lf0_sub=T_(a["draw0::lf0_sub"]),
              mgc_t=T_(a["draw0::mgc_t"]), mgc_noise=T_(a["draw0::mgc_noise"]),
              bap_t=T_(a["draw0::bap_t"]), bap_noise=T_(a["draw0::bap_noise"]),
              vuv_lstm=[T_(keep)])
    preds, _ = O.model_forward(P, cfg, T_(a["x_main"]), T_(a["x_sub"]),
                               (T_(a["spk_main"]), T_(a["spk_sub"])), a["lengths"],
                               (T_(a["y_main"]), T_(a["y_sub"])), od, bn_updates={})
    oloss = O.masked_l1_loss(preds, T_(a["y_main"]), a["lengths"], cfg["stream_sizes"])
    oloss.backward()
    onorm = torch.norm(torch.stack([P[k].grad.norm() for k in trainable]))
    assert abs(loss.item() - oloss.item()) < 1e-5 * abs(oloss.item())
    assert abs(norm.item() - onorm.item()) < 1e-4 * onorm.item()
    # the V/UV loss gradient differs from the p = 0 golden step: the mask is in the step
    assert abs(loss.item() - meta["losses"][0]) > 1e-6 * abs(meta["losses"][0])
    errs = {k: rel_l2(grads[k], P[k].grad) for k in trainable if not _pre_bn_bias(k)}
    record_errors("train_step_vuv_dropout", dict(loss=loss.item(), oracle_loss=oloss.item(),
                                                  grad_rel_l2=errs))
    bad = [(k, e) for k, e in errs.items() if e > 5e-5]  # measured <= 2.3e-6
    assert not bad, bad[:5]
