"""Pin the timing-model oracle (oracle/timing_oracle.py) to the reference-generated goldens:
nnsvs/mdn.py on a (G, D, dim_wise) grid, nnsvs.model.MDN with the reference's
tests/data/mdn_test.pth weights (BASELINE config 1, CPU), MultiTrackVariancePredictor."""
import torch

from golden_util import load_case, params_from_shapes, rel
from oracle import timing_oracle as TO

T_ = torch.from_numpy


def test_mdn_grid():
    a, meta = load_case("mdn")
    for key, G, D, dw in meta["grid"]:
        g = lambda k: T_(a[f"{key}::{k}"])  # noqa: E731
        lp, ls, mu = (g(k).clone().requires_grad_() for k in ("lp", "ls", "mu"))
        loss = TO.mdn_loss(lp, ls, mu, g("tgt"), reduce=False)
        assert rel(loss.detach(), g("loss")) < 1e-6, key
        (loss * g("R")).sum().backward()
        for k in ("lp", "ls", "mu"):
            assert rel(locals()[k].grad, g("d_" + k)) < 1e-5, (key, k)
        sig, m = TO.mdn_most_probable(g("lp"), g("ls"), g("mu"))
        # component selection is exact (mu is a plain gather); sigma = exp(.) may differ by
        # an ulp between host CPUs' vectorised exp, so it is held to 1e-6 relative
        assert torch.equal(m, g("mu_best")), key
        assert torch.allclose(sig, g("sigma"), rtol=1e-6, atol=0), key
        assert rel(TO.mdn_loss(g("lp"), g("ls"), g("mu"), g("tgt")), g("loss_red")) < 1e-6


def test_mdn_model_reference_fixture_weights():
    """BASELINE config 1: the single-track MDN duration model on CPU with mdn_test.pth."""
    a, _ = load_case("mdn")
    P = {k[len("mdn_test::"):]: T_(v) for k, v in a.items()
         if k.startswith("mdn_test::") and "::grad::" not in k}
    P = {k: v.clone().requires_grad_() if v.is_floating_point() else v for k, v in P.items()}
    lp, ls, mu = TO.mdn_model(P, P.pop("x").detach(), 1, 1, 1)
    assert rel(lp.detach(), a["mdn_test::lp"]) < 1e-6
    assert rel(mu.detach(), a["mdn_test::mu"]) < 1e-6
    loss = TO.mdn_loss(lp, ls, mu, T_(a["mdn_test::y"])).mean()
    assert rel(loss.detach(), a["mdn_test::loss"]) < 1e-6
    loss.backward()
    for k in ("model.0.weight", "model.2.mu.weight", "model.2.log_sigma.bias"):
        assert rel(P[k].grad, a["mdn_test::grad::" + k]) < 1e-5, k


def test_variance_predictor_duration_and_timelag():
    a, meta = load_case("variance_predictor")
    for name in ("duration", "timelag"):
        m = meta[name]
        p = name + "::"
        P = params_from_shapes(m["shapes"], requires_grad=True)
        x, s0, s1 = T_(a[p + "x"]), T_(a[p + "s0"]), T_(a[p + "s1"])
        with torch.no_grad():
            ev = TO.variance_predictor(P, m["cfg"], x, (s0, s1))
        for k, v in zip(("lp", "ls", "mu"), ev):
            assert rel(v, a[p + "eval_" + k]) < 1e-5, (name, k)
        sig, mu = TO.mdn_most_probable(*ev)
        assert rel(mu, a[p + "inf_mu"]) < 1e-5 and rel(sig, a[p + "inf_sigma"]) < 1e-5
        masks = [T_(a[p + f"mask{i}"]).transpose(1, 2) for i in range(m["cfg"]["num_layers"])]
        lp, ls, mu = TO.variance_predictor(P, m["cfg"], x, (s0, s1), masks)
        loss = TO.masked_mdn_loss(lp, ls, mu, T_(a[p + "y"]), a[p + "lengths"])
        assert rel(loss.detach(), a[p + "loss"]) < 1e-5, name
        loss.backward()
        for k, (s, ab, l2) in m["grad_summary"].items():
            g = P[k].grad.double()
            assert abs(g.abs().sum().item() - ab) <= 1e-4 * ab + 1e-9, (name, k)
            if p + "grad::" + k in a:
                assert rel(P[k].grad, a[p + "grad::" + k]) < 1e-4, (name, k)
