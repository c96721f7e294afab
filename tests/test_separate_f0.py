"""The recipe's default acoustic model, MultiTrackMultistreamSeparateF0ParametricModel
(multistream.py:348-577) with MultiTrackLSTMEncoder (nnsvs/model.py:1435-1537) and
embedding-free FFConvLSTM decoders, against fixtures the reference itself produced
(tests/golden/gen_goldens.py sf0): training-mode forward through the reference API with
its backward (tiny model, every gradient; full recipe size at T = 32, outputs and gradient
summaries), two reference train steps, and inference with pad_inference_multitrack.

Tolerances: oracle (CPU fp32) outputs rel 1e-5, gradients 1e-4 of the gradient scale;
HIP path at fp32 GEMM precision outputs rel 1e-4 (AR decoder + 3 recurrences), gradients
1e-3 of the gradient scale, train-step loss rel 1e-5 and grad norm rel 1e-4.  The golden
models run the LSTMs' inter-layer dropout at 0 (torch's C++ RNG cannot be replayed)."""
import numpy as np
import pytest
import torch

from oracle import ensvs_oracle as O
from ensemble_svs_with_interactions_amd import configs, engine
from golden_util import (_pre_bn_bias, check_grad_summary, load_case, params_from_shapes, rel,
                         rel_l2)


def _cfg(tiny):
    return configs.multitrack_separate_f0(num_speakers=4, tiny=tiny)


def _grad_ok(got, ref, tol, floor):
    got = torch.as_tensor(got).double()
    ref = torch.as_tensor(ref).double()
    return (got - ref).abs().max().item() <= tol * max(ref.abs().max().item(), floor)


def _t(a, k):
    return torch.from_numpy(np.ascontiguousarray(a[k]))


def _spks(a, pfx=""):
    return _t(a, pfx + "spk_main").long(), _t(a, pfx + "spk_sub").long()


# ------------------------------------------------------------------ CPU: oracle, API

@pytest.mark.parametrize("tiny", [True, False])
def test_state_dict_matches_reference(tiny):
    a, meta = load_case("sf0_forward_tiny" if tiny else "sf0_forward_full")
    model = configs.instantiate(_cfg(tiny))
    mine = {k: list(v.shape) for k, v in model.state_dict().items()}
    assert mine == meta["shapes"]
    assert model.prediction_type().name == "DETERMINISTIC"
    assert model.has_residual_lf0_prediction()


@pytest.mark.parametrize("case", ["sf0_forward_tiny", "sf0_forward_full"])
def test_oracle_forward_matches_reference(case):
    a, meta = load_case(case)
    tiny = case.endswith("tiny")
    P = params_from_shapes(meta["shapes"], requires_grad=True)
    bn = {}
    draws = dict(lf0_main=_t(a, "draw::lf0_main"), lf0_sub=_t(a, "draw::lf0_sub"))
    (om, rm), (os_, rs) = O.separate_f0_forward(
        P, _cfg(tiny), _t(a, "x_main"), _t(a, "x_sub"), _spks(a), a["lengths"].tolist(),
        [_t(a, "y_main"), _t(a, "y_sub")], draws, training=True, bn_updates=bn)
    for got, k in ((om, "out_main"), (rm, "res_main"), (os_, "out_sub"), (rs, "res_sub")):
        assert rel(got.detach(), a[k]) < 1e-5, k
    for k in a:
        if k.startswith("bn::"):
            assert rel(P[k[4:]], a[k]) < 1e-5, k
    sum((t * _t(a, f"R{i}")).sum() for i, t in enumerate((om, rm, os_, rs))).backward()
    grads = {k: v.grad for k, v in P.items() if getattr(v, "grad", None) is not None}
    if tiny:
        refs = {k[6:]: a[k] for k in a if k.startswith("grad::")}
        floor = 1e-2 * max(float(np.abs(g).max()) for g in refs.values())
        bad = [k for k, g in refs.items() if not _pre_bn_bias(k) and
               not _grad_ok(grads.get(k, torch.zeros(g.shape)), g, 1e-4, floor)]
        assert not bad, bad
    else:
        assert not check_grad_summary(grads, meta["grad_summary"], "", rtol=1e-4, atol=1e-6)


def test_oracle_inference_matches_reference():
    a, meta = load_case("sf0_inference_tiny")
    P = params_from_shapes(load_case("sf0_forward_tiny")[1]["shapes"])
    for T in (29, 32):
        p = f"T{T}::"
        out = O.separate_f0_inference(P, _cfg(True), _t(a, p + "x_main"), _t(a, p + "x_sub"),
                                      _spks(a, p), a[p + "lengths"].tolist(),
                                      _t(a, p + "masks_main"), _t(a, p + "masks_sub"))
        assert rel(out, a[p + "out"]) < 1e-5


def test_rejects_unsupported_submodels():
    cfg = _cfg(True)
    cfg["mgc_model"]["_target_"] = f"{configs.PKG}.transformer.TransformerEncoder"
    with pytest.raises((NotImplementedError, TypeError)):
        configs.instantiate(cfg)


# ------------------------------------------------------------------ GPU: HIP path

def _build(tiny, shapes):
    from gpu_util import build
    model = build(_cfg(tiny), shapes)
    for m in (model.mgc_model, model.vuv_model, model.bap_model, model.encoder):
        m.lstm.dropout = 0.0
    return model


def _dev(a, k):
    return torch.from_numpy(np.ascontiguousarray(a[k])).cuda().contiguous()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["sf0_forward_tiny", "sf0_forward_full"])
def test_forward_backward_matches_reference(case):
    """The reference API (autograd): (out_main, res_main), (out_sub, res_sub) with teacher
    forcing, BatchNorm running statistics after the call, parameter gradients."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case(case)
    tiny = case.endswith("tiny")
    model = _build(tiny, meta["shapes"])
    model.train()
    B, T = a["x_main"].shape[:2]
    model._replay_draws = dict(lf0_main=_dev(a, "draw::lf0_main").view(-1),
                               lf0_sub=_dev(a, "draw::lf0_sub").view(-1))
    try:
        (om, rm), (os_, rs) = model(_dev(a, "x_main"), _dev(a, "x_sub"),
                                    (_dev(a, "spk_main"), _dev(a, "spk_sub")),
                                    lengths=a["lengths"].tolist(),
                                    ys=[_dev(a, "y_main"), _dev(a, "y_sub")])
    finally:
        model._replay_draws = None
    outs = (om, rm, os_, rs)
    for got, k in zip(outs, ("out_main", "res_main", "out_sub", "res_sub")):
        assert got.shape == a[k].shape, k
        assert rel(got.detach().cpu(), a[k]) < 1e-4, k
    sd = model.state_dict()
    for k in a:
        if k.startswith("bn::"):
            assert rel(sd[k[4:]].cpu(), a[k]) < 1e-4, k
    sum((t * _dev(a, f"R{i}")).sum() for i, t in enumerate(outs)).backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu() for k, p in model.named_parameters() if p.grad is not None}
    if tiny:
        refs = {k[6:]: a[k] for k in a if k.startswith("grad::")}
        floor = 1e-2 * max(float(np.abs(g).max()) for g in refs.values())
        bad = [(k, rel(grads.get(k, torch.zeros(g.shape)), g)) for k, g in refs.items()
               if not _pre_bn_bias(k) and
               not _grad_ok(grads.get(k, torch.zeros(g.shape)), g, 1e-3, floor)]
        assert not bad, bad
    else:
        # recipe size: the V/UV decoder's gradients sit ~3 % (rel L2, tools/sf0_grad_diag.py)
        # from the CPU oracle's while its outputs agree to 5e-6 -- ReLU decisions at the
        # kink flip between fp32 summation orders in its narrow 1-channel head; every
        # gradient's norm is held to 5e-2, the other decoders' and the lf0 model's to 1e-3
        bad = []
        for k, (_, _, l2) in meta["grad_summary"].items():
            if _pre_bn_bias(k):
                continue
            tol = 5e-2 if k.startswith(("vuv_model.", "encoder.", "speaker_")) else 1e-3
            got = grads[k].double().norm().item() if k in grads else 0.0
            if abs(got - l2) > tol * l2 + 1e-6:
                bad.append((k, got, l2))
        assert not bad, bad[:5]


@pytest.mark.gpu
def test_train_step_matches_reference():
    """Two fused train steps (train.train_step: loss on the main output, BatchNorm updates of
    the unobservable sub calls) vs two reference train steps."""
    from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step
    engine.set_gemm_precision("fp32")
    a, meta = load_case("sf0_train_tiny")
    model = _build(True, meta["shapes"])
    opt = FusedAdam(model, lr=meta["lr"])
    xm, xs, ym = _dev(a, "x_main"), _dev(a, "x_sub"), _dev(a, "y_main")
    s0, s1 = _dev(a, "spk_main"), _dev(a, "spk_sub")
    lens = a["lengths"].tolist()
    for s in range(meta["steps"]):
        d = dict(lf0_main=_dev(a, f"draw{s}::lf0_main").view(-1),
                 lf0_sub=_dev(a, f"draw{s}::lf0_sub").view(-1))
        loss, norm = train_step(model, opt, xm, xs, ym, s0, s1, lens, draws=d)
        torch.cuda.synchronize()
        print(f"step {s}: loss {loss.item():.7f} ref {meta['losses'][s]:.7f} | "
              f"norm {norm.item():.6f} ref {meta['grad_norms'][s]:.6f}")
        assert abs(loss.item() - meta["losses"][s]) < 1e-5 * abs(meta["losses"][s])
        assert abs(norm.item() - meta["grad_norms"][s]) < 1e-4 * meta["grad_norms"][s]
    sd = model.state_dict()
    for k, v in sd.items():
        if "final::" + k not in a or v.dtype != torch.float32:
            continue
        ref = torch.from_numpy(a["final::" + k])
        err = (v.cpu() - ref).abs().max().item()
        # Adam moves each element by ~lr per step: a sign flip of a noise-level gradient
        # element is at most 2 lr per step; BN running stats carry the pre-BN biases
        assert err < 4 * meta["lr"] + 1e-5 * ref.abs().max().item(), (k, err)


@pytest.mark.gpu
def test_inference_matches_reference():
    engine.set_gemm_precision("fp32")
    a, _ = load_case("sf0_inference_tiny")
    model = _build(True, load_case("sf0_forward_tiny")[1]["shapes"])
    model.eval()
    for T in (29, 32):
        p = f"T{T}::"
        out = model.inference(_dev(a, p + "x_main"), _dev(a, p + "x_sub"),
                              spks=(_dev(a, p + "spk_main"), _dev(a, p + "spk_sub")),
                              lengths=a[p + "lengths"].tolist(),
                              draws=dict(lf0_main=_dev(a, p + "masks_main").view(-1),
                                         lf0_sub=_dev(a, p + "masks_sub").view(-1)))
        assert tuple(out.shape) == a[p + "out"].shape
        assert rel(out.cpu(), a[p + "out"]) < 1e-4


@pytest.mark.gpu
def test_recipe_size_graph_replay_equals_eager_bf16():
    """Recipe-size model (encoder H = 512, decoders H = 256 / 64 / 62 on the per-step and
    persistent recurrences), 8 pairs x 1024 frames, ragged, bf16 GEMM operands, explicit
    draws: two HIP-graph-replayed train steps give exactly the eager steps' loss, grad
    norm and Adam state."""
    from ensemble_svs_with_interactions_amd import data
    from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep, train_step
    engine.set_gemm_precision("bf16")
    P, T = 8, 1024
    rng = np.random.default_rng(5)
    lens = sorted(((rng.integers(T // 2, T + 1, size=P) // 4) * 4).tolist(), reverse=True)
    lens[0] = T
    b = data.synthetic_batch(P, T, 77, lengths=lens)
    g = lambda k: torch.from_numpy(b[k]).cuda().contiguous()  # noqa: E731
    xm, xs, ym, s0, s1 = g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub")

    def draws(seed):
        gen = torch.Generator(device="cuda").manual_seed(seed)
        keep = lambda: ((torch.rand(P * T // 4, device="cuda", generator=gen) < 0.5)  # noqa
                        .float() * 2.0)
        return dict(lf0_main=keep(), lf0_sub=keep())

    def model():
        torch.manual_seed(0)
        m = configs.instantiate(_cfg(False)).cuda()
        for sub in (m.mgc_model, m.vuv_model, m.bap_model, m.encoder):
            sub.lstm.dropout = 0.0
        return m
    seq = [draws(s) for s in (1, 2)]
    m_e = model()
    o_e = FusedAdam(m_e)
    eager = []
    for d in seq:
        loss, norm = train_step(m_e, o_e, xm, xs, ym, s0, s1, lens, draws=d)
        eager.append((loss.item(), norm.item()))
    m_g = model()
    o_g = FusedAdam(m_g)
    gs = GraphedTrainStep(m_g, o_g, xm, xs, ym, s0, s1, lens, warmup=1, draws=seq[0])
    graphed = [tuple(t.item() for t in gs.warmup_result)]
    loss, norm = gs.step(draws=seq[1])
    graphed.append((loss.item(), norm.item()))
    torch.cuda.synchronize()
    assert graphed == eager, (graphed, eager)
    assert all(np.isfinite(v) for step in eager for v in step)
    assert torch.equal(o_g.flat, o_e.flat) and torch.equal(o_g.m, o_e.m)


@pytest.mark.gpu
def test_bf16_copies_match_cast_by_consumers():
    """Recipe-size model, bf16 GEMM operands: the production step -- the decoders' input in
    zero-padded 1 032-column rows with one bf16 copy (acoustic_models.DEC_PAD), the
    cooperative LSTMs' bf16 copies of y / dg and per-sequence bias partials
    (layers.COOP_BF16) -- against the same step with both off, where every consumer rounds the
    fp32 tensors itself.  The forward is the same bits (the same roundings feed the same
    GEMMs); the gradients agree within 1e-4 (rel L2, the whole flat gradient and each
    parameter with a norm above 1e-3 of the largest): the bias sums run in another order and
    the decoders' 1 026-column weight gradient runs on the bf16-operand kernel.  The
    decoders' parameter gradients issued after their input gradients (DEC_LATER) or between
    them, and the V/UV and bap decoders started after the mgc decoder's conv stack
    (DEC_ORDER) or with it: the same bits."""
    from ensemble_svs_with_interactions_amd import acoustic_models as AM, data
    from ensemble_svs_with_interactions_amd import layers as Ly
    from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step
    engine.set_gemm_precision("bf16")
    P, T = 8, 256
    lens = [T, 240, 200, 256, 128, 64, 180, 252]
    b = data.synthetic_batch(P, T, 91, lengths=lens)
    g = lambda k: torch.from_numpy(b[k]).cuda().contiguous()  # noqa: E731
    gen = torch.Generator(device="cuda").manual_seed(3)
    keep = [((torch.rand(P * T // 4, device="cuda", generator=gen) < 0.5).float() * 2.0)
            for _ in range(2)]
    res = []
    try:
        for on, later, order in ((True, True, True), (False, True, True), (True, False, True),
                                 (True, True, False)):
            AM.DEC_PAD["on"] = on
            Ly.COOP_BF16["on"] = on
            AM.DEC_LATER["on"] = later
            AM.DEC_ORDER["on"] = order
            torch.manual_seed(0)
            m = configs.instantiate(_cfg(False)).cuda()
            for sub in (m.mgc_model, m.vuv_model, m.bap_model, m.encoder):
                sub.lstm.dropout = 0.0
            opt = FusedAdam(m)
            loss, norm = train_step(m, opt, g("x_main"), g("x_sub"), g("y_main"), g("spk_main"),
                                    g("spk_sub"), lens, draws=dict(lf0_main=keep[0],
                                                                    lf0_sub=keep[1]))
            torch.cuda.synchronize()
            grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()
                     if p.grad is not None}
            res.append((loss.item(), norm.item(), opt.gflat.detach().clone(), grads))
    finally:
        AM.DEC_PAD["on"] = True
        Ly.COOP_BF16["on"] = True
        AM.DEC_LATER["on"] = True
        AM.DEC_ORDER["on"] = True
    (l1, n1, g1, p1), (l0, n0, g0, p0) = res[:2]
    for l2, n2, g2, _ in res[2:]:
        assert (l2, n2) == (l1, n1) and torch.equal(g2, g1)
    assert l1 == l0, (l1, l0)
    assert abs(n1 - n0) <= 1e-4 * n0
    assert rel_l2(g1.cpu(), g0.cpu()) < 1e-4
    big = max(v.norm().item() for v in p0.values())
    bad = [(k, rel_l2(p1[k].cpu(), v.cpu())) for k, v in p0.items()
           if v.norm().item() > 1e-3 * big and rel_l2(p1[k].cpu(), v.cpu()) > 1e-4]
    assert not bad, bad[:5]
