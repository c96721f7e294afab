"""Timing models on MI355X vs the reference goldens.

mdn.npz: nnsvs/mdn.py on a (G, D, dim_wise) grid incl. G = 30 and the -7 clamps / +-5 sigma
clip; nnsvs.model.MDN with the reference's tests/data/mdn_test.pth weights (BASELINE
config 1).  variance_predictor.npz: the recipe's multi-track duration / time-lag models,
eval forward + training forward with the reference's dropout masks, masked MDN loss and
backward.  Tolerances: fp32 GEMMs, rel 1e-5 forward / 1e-4 gradients; most-probable
selection exact.
"""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import engine, timing
from golden_util import load_case, params_from_shapes, rel

pytestmark = pytest.mark.gpu


def test_mdn_loss_grid_and_most_probable():
    engine.set_gemm_precision("fp32")
    a, meta = load_case("mdn")
    for key, G, D, dw in meta["grid"]:
        g = lambda k: torch.from_numpy(a[f"{key}::{k}"]).cuda()  # noqa: E731
        lp, ls, mu = (g(k).clone().requires_grad_() for k in ("lp", "ls", "mu"))
        loss = timing.mdn_loss(lp, ls, mu, g("tgt"), reduce=False)
        assert rel(loss.detach().cpu(), a[f"{key}::loss"]) < 1e-5, key
        (loss * g("R")).sum().backward()
        for n, t in (("lp", lp), ("ls", ls), ("mu", mu)):
            assert rel(t.grad.cpu(), a[f"{key}::d_{n}"]) < 1e-5, (key, n)
        sig, m = timing.mdn_get_most_probable_sigma_and_mu(g("lp"), g("ls"), g("mu"))
        assert torch.equal(m.cpu(), torch.from_numpy(a[f"{key}::mu_best"])), key
        assert rel(sig.cpu(), a[f"{key}::sigma"]) < 1e-6, key
        red = timing.mdn_loss(g("lp"), g("ls"), g("mu"), g("tgt"))
        assert rel(red.cpu(), a[f"{key}::loss_red"]) < 1e-5, key


def test_mdn_model_reference_fixture_weights():
    """nnsvs.model.MDN(331 -> 4 -> G 1) with the reference's mdn_test.pth state_dict."""
    engine.set_gemm_precision("fp32")
    a, _ = load_case("mdn")
    sd = {k[len("mdn_test::"):]: torch.from_numpy(v) for k, v in a.items()
          if k.startswith("mdn_test::model.") and "::grad::" not in k}
    model = timing.MDN(in_dim=331, hidden_dim=4, out_dim=1, num_layers=1, num_gaussians=1)
    model.load_state_dict(sd)
    model = model.cuda()
    x = torch.from_numpy(a["mdn_test::x"]).cuda()
    lp, ls, mu = model(x)
    assert rel(lp.detach().cpu(), a["mdn_test::lp"]) < 1e-5
    assert rel(ls.detach().cpu(), a["mdn_test::ls"]) < 1e-5
    assert rel(mu.detach().cpu(), a["mdn_test::mu"]) < 1e-5
    loss = timing.mdn_loss(lp, ls, mu, torch.from_numpy(a["mdn_test::y"]).cuda()).mean()
    assert rel(loss.detach().cpu(), a["mdn_test::loss"]) < 1e-5
    loss.backward()
    for k, p in model.named_parameters():
        assert rel(p.grad.cpu(), a["mdn_test::grad::" + k]) < 1e-4, k
    mu_i, sig_i = model.inference(x)
    assert rel(mu_i.cpu(), a["mdn_test::inf_mu"]) < 1e-5
    assert rel(sig_i.cpu(), a["mdn_test::inf_sigma"]) < 1e-5


@pytest.mark.parametrize("name", ["duration", "timelag"])
def test_variance_predictor_matches_reference(name):
    engine.set_gemm_precision("fp32")
    a, meta = load_case("variance_predictor")
    m, p = meta[name], name + "::"
    model = timing.MultiTrackVariancePredictor(**m["cfg"])
    model.load_state_dict(params_from_shapes(m["shapes"]))
    model = model.cuda()
    g = lambda k: torch.from_numpy(a[p + k]).cuda()  # noqa: E731
    x, s0, s1 = g("x"), g("s0"), g("s1")
    model.eval()
    with torch.no_grad():
        ev = model(x, (s0, s1))
        mu_i, sig_i = model.inference(x, (s0, s1))
    for k, v in zip(("lp", "ls", "mu"), ev):
        assert rel(v.cpu(), a[p + "eval_" + k]) < 1e-5, k
    assert rel(mu_i.cpu(), a[p + "inf_mu"]) < 1e-5 and rel(sig_i.cpu(), a[p + "inf_sigma"]) < 1e-5
    model.train()
    B, T = x.shape[:2]
    model._replay_masks = [g(f"mask{i}").transpose(1, 2).contiguous().view(-1)
                           for i in range(m["cfg"]["num_layers"])]
    lp, ls, mu = model(x, (s0, s1))
    lengths = torch.from_numpy(a[p + "lengths"]).cuda()
    mask = torch.arange(T, device="cuda")[None, :] < lengths[:, None]
    # train_multitrack.py:101-112 (mdn_loss(reduce=False).masked_select(mask).mean())
    loss = timing.mdn_loss(lp, ls, mu, g("y"), reduce=False).masked_select(mask).mean()
    assert rel(loss.detach().cpu(), a[p + "loss"]) < 1e-5
    loss.backward()
    for k, (s, ab, l2) in m["grad_summary"].items():
        gr = dict(model.named_parameters())[k].grad.double().cpu()
        assert abs(gr.norm().item() - l2) <= 1e-4 * l2 + 1e-9, (k, gr.norm().item(), l2)
        if p + "grad::" + k in a:
            assert rel(gr, a[p + "grad::" + k]) < 1e-4, k


@pytest.mark.parametrize("name", ["duration", "timelag"])
def test_timing_train_step(name):
    """bin/train_multitrack.py:46-154 through timing.timing_train_step: the masked-mean MDN
    loss and parameter gradients equal the reference-generated ones (variance_predictor
    golden, same dropout masks), and the first Adam step moves every parameter by
    lr * g / (|g| + eps) (no clipping in the timing step)."""
    from ensemble_svs_with_interactions_amd.train import FusedAdam

    engine.set_gemm_precision("fp32")
    a, meta = load_case("variance_predictor")
    m, p = meta[name], name + "::"
    model = timing.MultiTrackVariancePredictor(**m["cfg"])
    model.load_state_dict(params_from_shapes(m["shapes"]))
    model = model.cuda()
    g = lambda k: torch.from_numpy(a[p + k]).cuda()  # noqa: E731
    x, s0, s1 = g("x"), g("s0"), g("s1")
    B, T, D2 = x.shape
    x0, x1 = x[:, :, : D2 // 2].contiguous(), x[:, :, D2 // 2:].contiguous()
    model._replay_masks = [g(f"mask{i}").transpose(1, 2).contiguous().view(-1)
                           for i in range(m["cfg"]["num_layers"])]
    lengths = torch.from_numpy(a[p + "lengths"]).cuda()
    mask = (torch.arange(T, device="cuda")[None, :] < lengths[:, None]).unsqueeze(-1)
    lr = 1e-3
    opt = FusedAdam(model, lr=lr, clip_norm=float("inf"))
    before = {k: v.detach().clone() for k, v in model.named_parameters()}
    loss = timing.timing_train_step(model, opt, x0, x1, g("y"), s0, s1, mask)
    assert rel(loss.cpu(), a[p + "loss"]) < 1e-5
    for k, (s, ab, l2) in m["grad_summary"].items():
        gr = dict(model.named_parameters())[k].grad.double().cpu()
        assert abs(gr.norm().item() - l2) <= 1e-4 * l2 + 1e-9, (k, gr.norm().item(), l2)
    for k, v in model.named_parameters():
        gr = v.grad.detach()
        want = before[k] - lr * gr / (gr.abs() + 1e-8)
        assert torch.allclose(v.detach(), want, rtol=0, atol=1e-6), k


def test_masked_mean_matches_masked_select():
    x = torch.randn(3, 37, 2, device="cuda")
    mask = torch.rand(3, 37, 1, device="cuda") < 0.6
    xr = x.clone().requires_grad_()
    got = timing.masked_mean(xr, mask)
    want = x.masked_select(mask).mean()
    assert rel(got.detach().cpu(), want.cpu()) < 1e-6
    got.backward()
    ref = mask.expand_as(x).float() / mask.expand_as(x).sum()
    assert torch.allclose(xr.grad, ref, rtol=1e-6, atol=0)
    assert torch.isnan(timing.masked_mean(x, torch.zeros_like(mask)))
