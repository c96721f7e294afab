"""The training step captured as HIP graphs (train.GraphedTrainStep) on MI355X.

Replays with explicit draws are bit-identical to eager train_step calls with the same draws
(loss, gradient norm, parameters, Adam moments, BN statistics) and follow the reference's
losses (train_step_tiny golden); replays without draws take fresh random draws per step;
a non-finite gradient norm skips the update and the device-side Adam step count, as the
reference skips optimizer.step() (train_acoustic_multitrack.py:365-380).
"""
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, engine
from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep, train_step
from golden_util import load_case
from gpu_util import build
from test_multitrack_gpu import _batch, _draws

pytestmark = pytest.mark.gpu


def _tiny(meta):
    model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True), meta["shapes"])
    model.vuv_model.lstm.dropout = 0.0
    return model, FusedAdam(model, lr=meta["lr"])


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_graphed_steps_bitwise_equal_eager(prec):
    engine.set_gemm_precision(prec)
    a, meta = load_case("train_step_tiny")
    xm, xs, ym, s0, s1, lens = _batch(a)
    B, T = xm.shape[:2]
    seq = [_draws(a, f"draw{s}::", B, T) for s in range(meta["steps"])] + [_draws(a, "draw0::", B, T)]
    m_e, o_e = _tiny(meta)
    eager = []
    for d in seq:
        loss, norm = train_step(m_e, o_e, xm, xs, ym, s0, s1, lens, draws=d)
        eager.append((loss.item(), norm.item()))
    m_g, o_g = _tiny(meta)
    gs = GraphedTrainStep(m_g, o_g, xm, xs, ym, s0, s1, lens, warmup=1, draws=seq[0])
    graphed = [tuple(t.item() for t in gs.warmup_result)]  # the eager warm-up step = step 0
    for d in seq[1:]:
        loss, norm = gs.step(draws=d)
        graphed.append((loss.item(), norm.item()))
    torch.cuda.synchronize()
    assert graphed == eager, (graphed, eager)
    if prec == "fp32":
        for s in range(meta["steps"]):
            assert abs(graphed[s][0] - meta["losses"][s]) < 1e-5 * abs(meta["losses"][s])
    assert torch.equal(o_g.flat, o_e.flat) and torch.equal(o_g.m, o_e.m)
    assert torch.equal(o_g.v, o_e.v) and torch.equal(o_g.dev_state, o_e.dev_state)
    assert o_g.device_step == len(seq)
    se, sg = m_e.state_dict(), m_g.state_dict()
    for k in se:
        assert torch.equal(se[k], sg[k]), k


def test_graphed_replays_draw_fresh_noise_and_skip_nonfinite():
    engine.set_gemm_precision("bf16")
    a, meta = load_case("train_step_tiny")
    xm, xs, ym, s0, s1, lens = _batch(a)
    model, opt = _tiny(meta)
    gs = GraphedTrainStep(model, opt, xm, xs, ym, s0, s1, lens, warmup=1)
    losses = []
    for _ in range(4):
        loss, norm = gs.step()
        losses.append(loss.item())
        assert torch.isfinite(norm).item()
    assert len(set(losses)) == len(losses), losses  # new diffusion steps / noise per replay
    assert opt.device_step == 5
    p = opt.flat.clone()
    bad = xm.clone()
    bad[0, 0, 0] = float("nan")
    loss, norm = gs.step(x_main=bad)
    torch.cuda.synchronize()
    assert not torch.isfinite(norm).item()
    assert torch.equal(opt.flat, p) and opt.device_step == 5
    loss, norm = gs.step(x_main=xm)
    assert torch.isfinite(loss).item() and opt.device_step == 6
    # eager steps still work after replays (packed weights refreshed from the flat buffer)
    loss, norm = train_step(model, opt, xm, xs, ym, s0, s1, lens)
    assert torch.isfinite(loss).item() and opt.device_step == 7
