"""Producer-side bf16 operand copies (layers.BF16_COPIES) on the recipe-width training step:
the FF GEMM epilogues, BatchNorm + ReLU passes, ReLU-mask passes and MFMA LSTM recurrences
write the bf16 rounding of their outputs, which the consuming GEMMs and weight gradients
take directly instead of rounding the fp32 tensors while staging.  The rounding is the same,
so the gradients must be the same bits; the LSTM biases alone change summation order
(per-sequence partial sums in the recurrence, then over sequences) and are compared at
1e-5."""
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, engine
from ensemble_svs_with_interactions_amd import layers as Ly
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step
from golden_util import load_case
from gpu_util import build
from test_multitrack_gpu import _batch, _draws

pytestmark = pytest.mark.gpu


def test_bf16_operand_copies_bitwise():
    engine.set_gemm_precision("bf16")
    a, meta = load_case("train_step_full")
    xm, xs, ym, s0, s1, lens = _batch(a)
    B, T = xm.shape[:2]
    res = []
    try:
        for on in (False, True):
            Ly.BF16_COPIES["on"] = on
            model = build(configs.multitrack_diffusion(num_speakers=4), meta["shapes"])
            model.vuv_model.lstm.dropout = 0.0
            opt = FusedAdam(model, lr=meta["lr"])
            loss, _ = train_step(model, opt, xm, xs, ym, s0, s1, lens,
                                 draws=_draws(a, "draw0::", B, T))
            torch.cuda.synchronize()
            res.append((loss.item(),
                        {k: p.grad.detach().clone() for k, p in model.named_parameters()},
                        {k: v.clone() for k, v in model.state_dict().items() if "running" in k}))
    finally:
        Ly.BF16_COPIES["on"] = True
    assert res[0][0] == res[1][0]
    lstm_bias = [k for k in res[0][1] if ".lstm." in k and ".bias_" in k]
    assert lstm_bias
    for k, g0 in res[0][1].items():
        g1 = res[1][1][k]
        if k in lstm_bias:
            assert (g1 - g0).norm().item() <= 1e-5 * g0.norm().item() + 1e-12, k
        else:
            assert torch.equal(g0, g1), k
    for k, v in res[0][2].items():
        assert torch.equal(v, res[1][2][k]), k
