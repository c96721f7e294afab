"""BASELINE config 2 on MI355X: the single-track NPSSMDNMultistreamParametricModel
(multistream.py:1025-1243) with the teacher-forced BiLSTMResF0NonAttentiveDecoder
(tacotron_f0.py:528-756), against reference-generated goldens."""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, data, engine
from ensemble_svs_with_interactions_amd.train import (FusedAdam, GraphedTrainStep,
                                                      train_step_single)
from golden_util import load_case, rel, _pre_bn_bias
from gpu_util import build

pytestmark = pytest.mark.gpu


def _draws(a, pfx, B, T):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(a[pfx + k])).cuda()  # noqa: E731
    return dict(
        lf0_main=t("lf0_main").view(-1).contiguous(),
        mgc_t=t("mgc_t"), bap_t=t("bap_t"),
        mgc_noise=t("mgc_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1),
        bap_noise=t("bap_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1))


def _g(a, k):
    return torch.from_numpy(a[k]).cuda().contiguous()


def test_st_forward_full():
    """Full-size training forward (teacher-forced lf0, both diffusions, V/UV) at fp32."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("st_forward_full")
    model = build(configs.singletrack_diffusion(), meta["shapes"])
    model.train()
    model.vuv_model.lstm.dropout = 0.0
    x, y = _g(a, "x"), _g(a, "y")
    B, T = x.shape[:2]
    outs, st = model._train_fwd(x, None, y, None, None, a["lengths"].tolist(),
                                _draws(a, "draw::", B, T))
    torch.cuda.synchronize()
    v = lambda k: outs[k].cpu().view(B, T, -1)  # noqa: E731
    assert rel(v("mgc_recon"), a["mgc_recon"]) < 1e-4
    assert rel(v("bap_recon"), a["bap_recon"]) < 1e-4
    assert rel(v("lf0"), a["lf0"]) < 1e-4
    assert rel(v("lf0_residual"), a["res"]) < 1e-4
    assert rel(v("vuv"), a["vuv"]) < 1e-4


def test_st_reference_api_forward():
    """The reference call signature model(x, lengths, y) -> ((mgc, lf0, vuv, bap), res)."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("st_forward_full")
    model = build(configs.singletrack_diffusion(), meta["shapes"])
    model.train()
    model.vuv_model.lstm.dropout = 0.0
    x, y = _g(a, "x"), _g(a, "y")
    B, T = x.shape[:2]
    model._replay_draws = _draws(a, "draw::", B, T)
    (mgc, lf0, vuv, bap), res = model(x, torch.from_numpy(a["lengths"]), y)
    del model._replay_draws
    torch.cuda.synchronize()
    assert rel(mgc[1].cpu(), a["mgc_recon"]) < 1e-4
    assert rel(lf0.cpu(), a["lf0"]) < 1e-4
    assert rel(res.cpu(), a["res"]) < 1e-4
    assert torch.equal(mgc[0].cpu(), torch.from_numpy(a["mgc_noise_out"]))


def test_st_train_step_tiny_matches_reference():
    """2 fused single-track training steps vs nnsvs/bin/train_acoustic.py train_step."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("st_train_step_tiny")
    model = build(configs.singletrack_diffusion(tiny=True), meta["shapes"])
    model.vuv_model.lstm.dropout = 0.0
    opt = FusedAdam(model, lr=meta["lr"])
    x, y = _g(a, "x"), _g(a, "y")
    B, T = x.shape[:2]
    p0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    for s in range(meta["steps"]):
        loss, norm = train_step_single(model, opt, x, y, a["lengths"].tolist(),
                                       draws=_draws(a, f"draw{s}::", B, T))
        torch.cuda.synchronize()
        print(f"step {s}: loss {loss.item():.7f} ref {meta['losses'][s]:.7f} | "
              f"norm {norm.item():.6f} ref {meta['grad_norms'][s]:.6f}")
        assert abs(loss.item() - meta["losses"][s]) < 1e-5 * abs(meta["losses"][s])
        assert abs(norm.item() - meta["grad_norms"][s]) < 1e-4 * meta["grad_norms"][s]
        if s == 0:
            bad = []
            grads = {k: p.grad.detach().cpu() for k, p in model.named_parameters()}
            for k, v in model.state_dict().items():
                if v.dtype != torch.float32 or "delta0::" + k not in a or _pre_bn_bias(k):
                    continue
                d = (v - p0[k]).cpu()
                err = (d - torch.from_numpy(a["delta0::" + k])).abs()
                if k in grads:
                    g = grads[k].abs()
                    err = err.masked_fill(g < 1e-7 * (1.0 + g.max()), 0.0)
                frac = (err > 0.1 * meta["lr"]).float().mean().item()
                if frac > 0.02:
                    bad.append((k, frac))
            assert not bad, bad[:5]


def test_st_inference_tiny_matches_reference():
    """pad_inference(mdn=True) + the lf0 model's own pad_inference, T mod 4 = 0..3."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("st_inference_tiny")
    model = build(configs.singletrack_diffusion(tiny=True), meta["shapes"])
    model.eval()
    for T in (28, 29, 30, 31):
        k = f"T{T}::"
        x = _g(a, k + "x")
        Tp = T + meta[f"T{T}"]["pad"]
        nz = lambda n: torch.from_numpy(a[k + n])[:, 0, 0].transpose(1, 2).contiguous() \
            .view(101, Tp, -1).cuda()  # noqa: E731
        draws = dict(noises={"mgc": nz("noise_mgc"), "bap": nz("noise_bap")},
                     masks=_g(a, k + "masks").view(-1))
        mu, sigma = model.inference(x, a[k + "lengths"].tolist(), draws=draws)
        torch.cuda.synchronize()
        assert tuple(mu.shape) == tuple(meta[f"T{T}"]["out_shape"])
        assert rel(mu.cpu(), a[k + "out"]) < 1e-4, T
        assert mu is sigma


def test_st_bench_size_bf16_graph():
    """bf16 production path at the bench workload (30 x 1024): graph-replayed steps are
    finite, the loss drops over 3 replays of one batch, and replay 1 matches an eager
    step from the same state to bf16 tolerance."""
    engine.set_gemm_precision("bf16")
    torch.manual_seed(5)
    model = configs.instantiate(configs.singletrack_diffusion()).cuda()
    opt = FusedAdam(model, lr=1e-4)
    b = data.synthetic_batch(30, 1024, 99)
    g = lambda k: torch.from_numpy(b[k]).cuda().contiguous()  # noqa: E731
    x, y = g("x_main"), g("y_main")
    lens = b["lengths"].tolist()
    step = GraphedTrainStep(model, opt, x, None, y, None, None, lens, warmup=1)
    losses = []
    for _ in range(3):
        loss, norm = step.step()
        losses.append(loss.item())
        assert np.isfinite(losses[-1]) and np.isfinite(norm.item())
    assert losses[-1] < step.warmup_result[0].item() * 1.05
