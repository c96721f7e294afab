"""Multi-track lf0 model, full pairwise model and the fused train step on MI355X."""
import numpy as np
import pytest
import torch

from oracle import ensvs_oracle as O
from ensemble_svs_with_interactions_amd import configs, engine
from ensemble_svs_with_interactions_amd.train import FusedAdam, step_metrics, train_step
from golden_util import (load_case, full_shapes, rel, grad_close, rel_l2, _pre_bn_bias,
                         sampled_grad_errors, record_errors)
from gpu_util import build

pytestmark = pytest.mark.gpu
CFG = configs.multitrack_diffusion(num_speakers=4)


def _masks(st, B, T):
    m = {}
    for n, i in enumerate((0, 2, 4)):
        m[f"ff{i}"] = (st["hs"][n] > 0).float().cpu().view(B, T, -1)
    for li, bi in enumerate((2, 6, 10)):
        m[f"bn{bi}"] = (st["csv"][li]["out"] > 0).float().cpu().view(B, T, -1)
    return m


def test_lf0_model_matches_reference():
    engine.set_gemm_precision("fp32")
    a, meta = load_case("lf0_model")
    cfg = dict(CFG["lf0_model"])
    mod = build(cfg, full_shapes(), "lf0_model.")
    for k, v in meta["lf0_stats"].items():
        setattr(mod, k, v)
    mod.train()
    P0 = {k: v.detach().cpu().clone() for k, v in mod.state_dict().items()}
    B, T, D = a["x_main"].shape
    xm = torch.from_numpy(a["x_main"]).cuda()
    xs = torch.from_numpy(a["x_sub"]).cuda()
    s0 = torch.from_numpy(a["spk_main"]).cuda().view(B, -1).contiguous()
    s1 = torch.from_numpy(a["spk_sub"]).cuda().view(B, -1).contiguous()
    lens = torch.tensor(a["lengths"].tolist(), device="cuda")
    masks = torch.from_numpy(a["masks"]).cuda().view(-1).contiguous()
    lf0, res, st = mod._fwd([xm, xs], D, B, T, lens, (s0, s1), s0.shape[1], masks=masks)
    R1 = torch.from_numpy(a["R1"]).cuda().view(-1).contiguous()
    R2 = torch.from_numpy(a["R2"]).cuda().view(-1).contiguous()
    d0, d1, _ = mod._bwd(st, R1, R2)
    torch.cuda.synchronize()
    assert rel(lf0.cpu().view(B, T, 1), a["lf0"]) < 1e-4
    assert rel(res.cpu().view(B, T, 1), a["res"]) < 1e-4
    # mask-matched oracle backward
    ocfg = dict(cfg)
    ocfg.update(meta["lf0_stats"])
    Pg = {k: (v.clone() if "running" in k else v.clone().requires_grad_())
          for k, v in P0.items() if v.dtype == torch.float32}
    sm = torch.from_numpy(a["spk_main"]).requires_grad_()
    ss = torch.from_numpy(a["spk_sub"]).requires_grad_()
    ol, orr = O.lf0_model(Pg, "", ocfg, torch.from_numpy(a["x_main"]), torch.from_numpy(a["x_sub"]),
                          sm.expand(B, T, -1), ss.expand(B, T, -1), a["lengths"],
                          torch.from_numpy(a["masks"]), relu_masks=_masks(st, B, T))
    ((ol * torch.from_numpy(a["R1"])).sum() + (orr * torch.from_numpy(a["R2"])).sum()).backward()
    assert rel(d0.cpu(), sm.grad.view(B, -1)) < 2e-4
    for k, p in mod.named_parameters():
        if _pre_bn_bias(k):
            continue
        assert rel(p.grad.cpu(), Pg[k].grad) < 5e-4, k
    # end-to-end vs the reference (measured 2.3e-6 rel-L2)
    assert grad_close(d0.cpu(), torch.from_numpy(a["d_spk_main"]).view(B, -1), 2e-5,
                      name="lf0_model.d_spk_main")


def _draws(a, pfx, B, T):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(a[pfx + k])).cuda()  # noqa: E731
    return dict(
        lf0_main=t("lf0_main").view(-1).contiguous(),
        lf0_sub=t("lf0_sub").view(-1).contiguous(),
        mgc_t=t("mgc_t"), bap_t=t("bap_t"),
        mgc_noise=t("mgc_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1),
        bap_noise=t("bap_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1))


def _batch(a):
    g = lambda k: torch.from_numpy(a[k]).cuda().contiguous()  # noqa: E731
    return g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"), a["lengths"].tolist()


def test_model_forward_full():
    engine.set_gemm_precision("fp32")
    a, meta = load_case("model_forward_full")
    model = build(configs.multitrack_diffusion(num_speakers=4), meta["shapes"])
    model.train()
    model.vuv_model.lstm.dropout = 0.0
    xm, xs, ym, s0, s1, lens = _batch(a)
    B, T = xm.shape[:2]
    outs, st = model._train_fwd(xm, xs, ym, s0, s1, lens, _draws(a, "draw::", B, T))
    torch.cuda.synchronize()
    v = lambda k: outs[k].cpu().view(B, T, -1)  # noqa: E731
    assert rel(v("mgc_recon"), a["mgc_recon"]) < 1e-4
    assert rel(v("bap_recon"), a["bap_recon"]) < 1e-4
    assert rel(v("lf0"), a["lf0"]) < 1e-4
    assert rel(v("lf0_residual"), a["res"]) < 1e-4
    assert rel(v("vuv"), a["vuv"]) < 1e-4


@pytest.mark.parametrize("case", ["train_step_tiny", "train_step_tiny_il"])
def test_train_step_tiny_matches_reference(case):
    """2 fused training steps vs the reference train_step; _il: the interaction-loss recipe
    (output_subtrack model, logf0_diff_weight 0.5)."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case(case)
    w_il = meta.get("logf0_diff_weight", 0.0)
    model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True,
                                               output_subtrack=w_il > 0), meta["shapes"])
    model.vuv_model.lstm.dropout = 0.0
    opt = FusedAdam(model, lr=meta["lr"])
    xm, xs, ym, s0, s1, lens = _batch(a)
    ysub = torch.from_numpy(a["y_sub"]).cuda().contiguous()
    B, T = xm.shape[:2]
    p0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    for s in range(meta["steps"]):
        loss, norm = train_step(model, opt, xm, xs, ym, s0, s1, lens,
                                draws=_draws(a, f"draw{s}::", B, T), y_sub=ysub,
                                logf0_diff_weight=w_il)
        torch.cuda.synchronize()
        print(f"step {s}: loss {loss.item():.7f} ref {meta['losses'][s]:.7f} | "
              f"norm {norm.item():.6f} ref {meta['grad_norms'][s]:.6f}")
        assert abs(loss.item() - meta["losses"][s]) < 1e-5 * abs(meta["losses"][s])
        assert abs(norm.item() - meta["grad_norms"][s]) < 1e-4 * meta["grad_norms"][s]
        # the reference's per-step log metrics (train_acoustic_multitrack.py:382-390)
        mt = step_metrics(loss, opt)
        assert mt["Loss"] == loss.item() and mt["GradNorm"] == norm.item()
        if w_il > 0:
            il = meta["interaction_losses"][s]
            assert abs(mt["Loss_LogF0_Interaction"] - il) < 1e-5 * abs(il)
            assert abs(mt["Loss_Feats"] + w_il * mt["Loss_LogF0_Interaction"] - mt["Loss"]) \
                <= 1e-6 * abs(mt["Loss"])
        else:
            assert mt["Loss_LogF0_Interaction"] == 0.0 and mt["Loss_Feats"] == mt["Loss"]
        if s == 0:
            bad = []
            grads = {k: p.grad.detach().cpu() for k, p in model.named_parameters()}
            for k, v in model.state_dict().items():
                if v.dtype != torch.float32 or "delta0::" + k not in a or _pre_bn_bias(k):
                    continue
                d = (v - p0[k]).cpu()
                ref = torch.from_numpy(a["delta0::" + k])
                err = (d - ref).abs()
                if k in grads:
                    # gradient elements at the float noise floor (near-dead ReLU units) move
                    # Adam by a rounding-sensitive fraction of lr: not compared
                    g = grads[k].abs()
                    err = err.masked_fill(g < 1e-7 * (1.0 + g.max()), 0.0)
                # Adam's first step is ~lr*sign(g): count elements off by > lr/10
                frac = (err > 0.1 * meta["lr"]).float().mean().item()
                if frac > 0.02:
                    bad.append((k, frac))
            assert not bad, bad[:5]
    sd = model.state_dict()
    for k in sd:
        if "running" in k and "final::" + k in a:
            # running statistics carry the pre-BN conv biases, whose zero-gradient Adam
            # updates are noise-driven (~lr): absolute tolerance lr/10
            ref = torch.from_numpy(a["final::" + k])
            err = (sd[k].cpu() - ref).abs().max().item()
            assert err < 0.1 * meta["lr"] + 1e-5 * ref.abs().max().item(), k


def test_train_step_full_width_matches_reference():
    """Recipe-width model (the production recurrence instantiations lstm<64/128> and
    ardec<256>, C = 256 / 128 DiffNet epilogues, 20 + 10 residual layers) through 2 fused
    training steps vs the reference train_step (P = 2, T = 64): loss <= 1e-5, grad norm
    <= 1e-4, and every step-0 parameter gradient (sampled elements, exact L2) vs the
    reference's; the measured errors are recorded (record_errors)."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("train_step_full")
    model = build(configs.multitrack_diffusion(num_speakers=4), meta["shapes"])
    model.vuv_model.lstm.dropout = 0.0
    opt = FusedAdam(model, lr=meta["lr"])
    xm, xs, ym, s0, s1, lens = _batch(a)
    B, T = xm.shape[:2]
    rec = {}
    for s in range(meta["steps"]):
        loss, norm = train_step(model, opt, xm, xs, ym, s0, s1, lens,
                                draws=_draws(a, f"draw{s}::", B, T))
        torch.cuda.synchronize()
        rec[f"step{s}"] = dict(loss=loss.item(), ref_loss=meta["losses"][s], norm=norm.item(),
                               ref_norm=meta["grad_norms"][s])
        assert abs(loss.item() - meta["losses"][s]) < 1e-5 * abs(meta["losses"][s])
        assert abs(norm.item() - meta["grad_norms"][s]) < 1e-4 * meta["grad_norms"][s]
        if s == 0:
            errs = sampled_grad_errors({k: p.grad for k, p in model.named_parameters()}, a,
                                       meta)
            errs = {k: e for k, e in errs.items() if not _pre_bn_bias(k)}
            rec["grad_rel_l2"] = {k: e[0] for k, e in errs.items()}
            rec["grad_norm_rel"] = {k: e[1] for k, e in errs.items()}
            record_errors("train_step_full", rec)
            # measured: sampled rel-L2 <= 4.5e-6 (median 7.9e-7), L2 norms <= 4.9e-7
            bad = [(k, e) for k, e in errs.items() if e[0] > 5e-5 or e[1] > 1e-5]
            assert not bad, bad[:5]
    record_errors("train_step_full", rec)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_concurrent_branches_bitwise_equal_serial(prec):
    """The lf0 / mgc / bap / vuv branches on concurrent HIP streams give bit-identical
    loss, gradients and BN statistics to the serial schedule."""
    engine.set_gemm_precision(prec)
    a, meta = load_case("train_step_tiny")
    xm, xs, ym, s0, s1, lens = _batch(a)
    B, T = xm.shape[:2]
    res = []
    try:
        for conc in (False, True):
            engine.set_concurrency(conc)
            model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True), meta["shapes"])
            model.vuv_model.lstm.dropout = 0.0
            opt = FusedAdam(model, lr=meta["lr"])
            loss, norm = train_step(model, opt, xm, xs, ym, s0, s1, lens,
                                    draws=_draws(a, "draw0::", B, T))
            torch.cuda.synchronize()
            res.append((loss.item(), opt.gflat.clone(),
                        {k: v.clone() for k, v in model.state_dict().items()}))
    finally:
        engine.set_concurrency(True)
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
    for k in res[0][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k


@pytest.mark.parametrize("case", ["train_step_tiny", "train_step_tiny_il"])
def test_fused_branch_schedule_matches(case):
    """train.set_fused_branches(True) (each branch's forward, loss gradient and backward on
    its own stream) gives the same gradients bit for bit, and the loss up to the order of
    its per-branch partial sums, as the forward-all / loss / backward-all schedule."""
    from ensemble_svs_with_interactions_amd.train import set_fused_branches

    engine.set_gemm_precision("fp32")
    a, meta = load_case(case)
    w_il = meta.get("logf0_diff_weight", 0.0)
    xm, xs, ym, s0, s1, lens = _batch(a)
    ysub = torch.from_numpy(a["y_sub"]).cuda().contiguous()
    B, T = xm.shape[:2]
    res = []
    try:
        for fused in (False, True):
            set_fused_branches(fused)
            model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True,
                                                       output_subtrack=w_il > 0), meta["shapes"])
            model.vuv_model.lstm.dropout = 0.0
            opt = FusedAdam(model, lr=meta["lr"])
            loss, norm = train_step(model, opt, xm, xs, ym, s0, s1, lens,
                                    draws=_draws(a, "draw0::", B, T), y_sub=ysub,
                                    logf0_diff_weight=w_il)
            torch.cuda.synchronize()
            res.append((loss.item(), opt.gflat.clone()))
    finally:
        set_fused_branches(False)
    assert abs(res[0][0] - res[1][0]) <= 1e-6 * abs(res[0][0])
    assert torch.equal(res[0][1], res[1][1])
    assert abs(res[1][0] - meta["losses"][0]) < 1e-5 * abs(meta["losses"][0])
