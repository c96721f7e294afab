"""Checkpoint / resume of the fused training path (train_util.py:1290-1335 save_checkpoint,
:1360-1384 _resume): {"state_dict", "optimizer_state", "lr_scheduler_state"} written with
torch.save, read back with torch.load(weights_only=True), and resumed

  * fused -> fused: the next step equals the uninterrupted run bit for bit (eager and
    HIP-graph replay), device step count included;
  * fused -> torch.optim.Adam through the drop-in (reference-style autograd) step, and
    torch.optim.Adam -> fused: the next update matches at Adam's lr scale;
  * StepLR (myconfig_notuseIL.yaml:49-53) drives FusedAdam's learning rate and its state
    round-trips.
"""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, engine
from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep, train_step
from golden_util import load_case
from gpu_util import build
from test_dropin_gpu import _draws, _reference_style_loss

pytestmark = pytest.mark.gpu
LR = 1e-3


def _setup():
    engine.set_gemm_precision("fp32")
    a, meta = load_case("train_step_tiny")
    cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True)
    g = lambda k: torch.from_numpy(a[k]).cuda().contiguous()  # noqa: E731
    batch = dict(xm=g("x_main"), xs=g("x_sub"), ym=g("y_main"), ys=g("y_sub"), s0=g("spk_main"),
                 s1=g("spk_sub"), lens=a["lengths"].tolist())
    B, T = batch["xm"].shape[:2]
    return a, meta, cfg, batch, _draws(a, B, T)


def _model(cfg, meta):
    m = build(cfg, meta["shapes"])
    m.vuv_model.lstm.dropout = 0.0
    return m


def _fused_step(model, opt, b, draws):
    return train_step(model, opt, b["xm"], b["xs"], b["ym"], b["s0"], b["s1"], b["lens"],
                      draws=draws)


def _torch_step(model, opt, b, draws, stream_sizes):
    """The reference's step (train_acoustic_multitrack.py:93-184, 358-380) on the drop-in
    model: autograd forward/backward, clip_grad_norm_(1.0), torch.optim.Adam."""
    model.train()
    opt.zero_grad()
    model._replay_draws = draws
    lengths = torch.tensor(b["lens"], device="cuda")
    loss = _reference_style_loss(model, b["xm"], b["xs"], b["ym"], b["ys"], (b["s0"], b["s1"]),
                                 lengths, 0.0, stream_sizes)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step()
    return loss


def _roundtrip(ckpt, tmp_path, name):
    path = tmp_path / f"{name}.pth"
    torch.save(ckpt, path)
    return torch.load(path, weights_only=True)


def _close_updates(before, after_a, after_b, grads, lr, tag):
    """Adam's update is ~lr * m / sqrt(v): count elements whose two updates differ by more
    than lr / 10 (gradient elements at the float noise floor are not compared)."""
    bad = []
    for k in before:
        gk = grads[k].abs()
        err = ((after_a[k] - before[k]) - (after_b[k] - before[k])).abs()
        err = err.masked_fill(gk < 1e-7 * (1.0 + gk.max()), 0.0)
        if (err > 0.1 * lr).float().mean().item() > 0.02:
            bad.append(k)
    assert not bad, (tag, bad[:5])


def test_fused_resume_bitwise(tmp_path):
    a, meta, cfg, b, draws = _setup()
    torch.manual_seed(0)
    ma = _model(cfg, meta)
    oa = FusedAdam(ma, lr=LR)
    sched_a = torch.optim.lr_scheduler.StepLR(oa, step_size=1, gamma=0.5)
    for _ in range(2):
        _fused_step(ma, oa, b, draws)
        sched_a.step()
    torch.cuda.synchronize()
    assert oa.lr == pytest.approx(LR * 0.25) and oa.device_step == 2
    ck = _roundtrip({"state_dict": ma.state_dict(), "optimizer_state": oa.state_dict(),
                     "lr_scheduler_state": sched_a.state_dict()}, tmp_path, "fused")
    # uninterrupted
    _fused_step(ma, oa, b, draws)
    torch.cuda.synchronize()
    # resumed
    mc = _model(cfg, meta)
    mc.load_state_dict(ck["state_dict"])
    oc = FusedAdam(mc, lr=LR)
    sched_c = torch.optim.lr_scheduler.StepLR(oc, step_size=1, gamma=0.5)
    oc.load_state_dict(ck["optimizer_state"])
    sched_c.load_state_dict(ck["lr_scheduler_state"])
    assert oc.lr == oa.lr and oc.device_step == 2
    _fused_step(mc, oc, b, draws)
    torch.cuda.synchronize()
    assert torch.equal(oc.flat, oa.flat) and torch.equal(oc.m, oa.m) and torch.equal(oc.v, oa.v)
    assert oc.device_step == oa.device_step == 3
    for k, v in ma.state_dict().items():
        assert torch.equal(v, mc.state_dict()[k]), k


def test_fused_resume_graph_replay(tmp_path):
    """GraphedTrainStep resumed from a checkpoint replays the same steps as the original."""
    a, meta, cfg, b, draws = _setup()
    runs = []
    for resume in (False, True):
        ma = _model(cfg, meta)
        oa = FusedAdam(ma, lr=LR)
        g = GraphedTrainStep(ma, oa, b["xm"], b["xs"], b["ym"], b["s0"], b["s1"], b["lens"],
                             warmup=1, draws=draws)
        g.step()
        torch.cuda.synchronize()
        if resume:
            ck = _roundtrip({"state_dict": ma.state_dict(),
                             "optimizer_state": oa.state_dict()}, tmp_path, "graph")
            ma = _model(cfg, meta)
            ma.load_state_dict(ck["state_dict"])
            oa = FusedAdam(ma, lr=LR)
            oa.load_state_dict(ck["optimizer_state"])
            assert oa.device_step == 2
            # capture on the resumed state: its warm-up step is the third step
            g = GraphedTrainStep(ma, oa, b["xm"], b["xs"], b["ym"], b["s0"], b["s1"], b["lens"],
                                 warmup=1, draws=draws)
        else:
            g.step()
        g.step()
        torch.cuda.synchronize()
        runs.append((oa.flat.clone(), oa.device_step))
    assert runs[0][1] == runs[1][1] == 4
    assert torch.equal(runs[0][0], runs[1][0])


def test_fused_to_torch_adam_and_back(tmp_path):
    a, meta, cfg, b, draws = _setup()
    sizes = cfg["stream_sizes"]
    # fused run: 2 steps, checkpoint
    ma = _model(cfg, meta)
    oa = FusedAdam(ma, lr=LR)
    for _ in range(2):
        _fused_step(ma, oa, b, draws)
    torch.cuda.synchronize()
    ck = _roundtrip({"state_dict": ma.state_dict(), "optimizer_state": oa.state_dict()},
                    tmp_path, "to_torch")
    st = ck["optimizer_state"]["state"]
    assert len(st) == len(list(ma.parameters()))
    assert all(float(s["step"]) == 2.0 for s in st.values())
    before = {k: v.detach().clone() for k, v in ma.named_parameters()}
    _fused_step(ma, oa, b, draws)  # the uninterrupted third step
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().clone() for k, p in ma.named_parameters()}
    after_fused = {k: v.detach().clone() for k, v in ma.named_parameters()}
    # resumed into torch.optim.Adam on the drop-in model
    mb = _model(cfg, meta)
    mb.load_state_dict(ck["state_dict"])
    ob = torch.optim.Adam(mb.parameters(), lr=LR)
    ob.load_state_dict(ck["optimizer_state"])
    _torch_step(mb, ob, b, draws, sizes)
    torch.cuda.synchronize()
    after_torch = {k: v.detach().clone() for k, v in mb.named_parameters()}
    _close_updates(before, after_fused, after_torch, grads, LR, "fused -> torch.optim.Adam")
    # and back: torch.optim.Adam's state (3 steps) resumed into FusedAdam
    ck2 = _roundtrip({"state_dict": mb.state_dict(), "optimizer_state": ob.state_dict()},
                     tmp_path, "to_fused")
    before2 = {k: v.detach().clone() for k, v in mb.named_parameters()}
    _torch_step(mb, ob, b, draws, sizes)
    torch.cuda.synchronize()
    after_torch2 = {k: v.detach().clone() for k, v in mb.named_parameters()}
    mc = _model(cfg, meta)
    mc.load_state_dict(ck2["state_dict"])
    oc = FusedAdam(mc, lr=LR)
    oc.load_state_dict(ck2["optimizer_state"])
    assert oc.device_step == 3
    _fused_step(mc, oc, b, draws)
    torch.cuda.synchronize()
    grads2 = {k: p.grad.detach().clone() for k, p in mc.named_parameters()}
    after_fused2 = {k: v.detach().clone() for k, v in mc.named_parameters()}
    _close_updates(before2, after_torch2, after_fused2, grads2, LR, "torch.optim.Adam -> fused")
    # the moments themselves agree with torch's after the same step
    sd_t, sd_f = ob.state_dict()["state"], oc.state_dict()["state"]
    num = sum(((sd_t[i]["exp_avg"].cpu() - sd_f[i]["exp_avg"]) ** 2).sum() for i in sd_t)
    den = sum((sd_t[i]["exp_avg"].cpu() ** 2).sum() for i in sd_t)
    assert (num / den).sqrt().item() < 1e-4
