"""The bench configuration itself (BASELINE config 3 on one GPU: 30 pairs x 1024 frames,
full-size recipe model, bf16 GEMM operands), checked through size-independent properties:

* the HIP-graph replay that bench.py times computes exactly what eager train_step calls
  compute (loss, grad norm, parameters, Adam moments; two steps, explicit draws), with
  ragged lengths (U[T/2, T], multiples of 4) as SURVEY §8(d) prescribes for parity runs;
* the bf16-operand step stays within 1 % (loss) / 5 % (grad norm) of the fp32 step from
  the same weights and draws (the fp32 path is the one pinned to the reference goldens).

Both at the bench shape and at 8 pairs x 4096 frames: the multi-track pairing never filters
long segments (nnsvs/train_util.py:160-166 hard-codes filter_long_segments=False), so
4096-step recurrences (SURVEY §8(d)'s long-sequence case) reach the production step.
"""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, data, engine
from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep, train_step

pytestmark = pytest.mark.gpu

SHAPES = [(30, 1024), (8, 4096)]


def _model():
    torch.manual_seed(0)
    m = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).cuda()
    m.vuv_model.lstm.dropout = 0.0  # nn.LSTM's inter-layer dropout has no replayable draw
    return m


def _batch(P, T):
    rng = np.random.default_rng(7)
    lens = (rng.integers(T // 2, T + 1, size=P) // 4) * 4
    b = data.synthetic_batch(P, T, 11, lengths=lens)
    g = lambda k: torch.from_numpy(b[k]).cuda().contiguous()  # noqa: E731
    return (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
            b["lengths"].tolist())


def _draws(P, T, seed, nm, nb):
    g = torch.Generator(device="cuda").manual_seed(seed)
    keep = lambda: ((torch.rand(P * T // 4, device="cuda", generator=g) < 0.5).float() * 2.0)  # noqa: E731
    return dict(lf0_main=keep(), lf0_sub=keep(),
                mgc_t=torch.randint(0, 100, (P,), device="cuda", generator=g),
                bap_t=torch.randint(0, 100, (P,), device="cuda", generator=g),
                mgc_noise=torch.randn(P * T, nm, device="cuda", generator=g),
                bap_noise=torch.randn(P * T, nb, device="cuda", generator=g))


@pytest.mark.parametrize("P,T", SHAPES)
def test_bench_config_graph_replay_equals_eager(P, T):
    engine.set_gemm_precision("bf16")
    xm, xs, ym, s0, s1, lens = _batch(P, T)
    m_e = _model()
    nm, nb = m_e.stream_sizes[0], m_e.stream_sizes[3]
    seq = [_draws(P, T, s, nm, nb) for s in (1, 2)]
    o_e = FusedAdam(m_e)
    eager = []
    for d in seq:
        loss, norm = train_step(m_e, o_e, xm, xs, ym, s0, s1, lens, draws=d)
        eager.append((loss.item(), norm.item()))
    m_g = _model()
    o_g = FusedAdam(m_g)
    gs = GraphedTrainStep(m_g, o_g, xm, xs, ym, s0, s1, lens, warmup=1, draws=seq[0])
    graphed = [tuple(t.item() for t in gs.warmup_result)]
    loss, norm = gs.step(draws=seq[1])
    graphed.append((loss.item(), norm.item()))
    torch.cuda.synchronize()
    assert graphed == eager, (graphed, eager)
    assert all(np.isfinite(v) for step in eager for v in step)
    assert torch.equal(o_g.flat, o_e.flat) and torch.equal(o_g.m, o_e.m)
    assert torch.equal(o_g.v, o_e.v)


@pytest.mark.parametrize("P,T", SHAPES)
def test_bench_config_bf16_close_to_fp32(P, T):
    xm, xs, ym, s0, s1, lens = _batch(P, T)
    res = []
    try:
        for prec in ("fp32", "bf16"):
            engine.set_gemm_precision(prec)
            m = _model()
            d = _draws(P, T, 3, m.stream_sizes[0], m.stream_sizes[3])
            loss, norm = train_step(m, FusedAdam(m), xm, xs, ym, s0, s1, lens, draws=d)
            res.append((loss.item(), norm.item()))
    finally:
        engine.set_gemm_precision("bf16")
    (l32, n32), (l16, n16) = res
    print(f"P={P} T={T} loss fp32 {l32:.7f} bf16 {l16:.7f} norm fp32 {n32:.6f} bf16 {n16:.6f}")
    assert abs(l16 - l32) <= 1e-2 * abs(l32), res
    assert abs(n16 - n32) <= 5e-2 * n32, res
