"""The torch.library boundary (torch_ops.py): every ensvs:: op passes
torch.library.opcheck (schema, autograd registration, fake-tensor shapes, AOT dispatch with
dynamic shapes -- forward and gradients against eager), and the drop-in model under
torch.compile(fullgraph=False) gives the eager loss and gradients.

Reference call sites the ops serve: nnsvs/bin/train_acoustic_multitrack.py:94-100 (the
model's forward with targets under autograd), gen.py:1290-1292 (inference)."""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, engine, torch_ops
from golden_util import load_case
from gpu_util import build

pytestmark = pytest.mark.gpu

FWD_TESTS = ("test_schema", "test_autograd_registration", "test_faketensor",
             "test_aot_dispatch_dynamic")
# The backward ops find their forward's saved state by the identity of the forward output they
# are handed (torch_ops._take), which opcheck's own tests copy; so a backward op is checked by
# hand: its fake implementation (FakeTensorMode) against one real call -- shapes, dtypes,
# devices.  Its arithmetic is what the forward ops' test_aot_dispatch_dynamic compares
# (gradients, eager vs AOT) and what the drop-in tests check against the fused step.


@pytest.fixture(autouse=True)
def _fp32():
    engine.set_gemm_precision("fp32")
    yield


def _tiny():
    a, meta = load_case("train_step_tiny")
    model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True), meta["shapes"])
    model.vuv_model.lstm.dropout = 0.0
    model.train()
    g = lambda k: torch.from_numpy(a[k]).cuda().contiguous()  # noqa: E731
    return model, a, meta, g


def _draws(a, B, T):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(a["draw0::" + k])).cuda()  # noqa: E731
    return dict(lf0_main=t("lf0_main").view(-1).contiguous(),
                lf0_sub=t("lf0_sub").view(-1).contiguous(), mgc_t=t("mgc_t"), bap_t=t("bap_t"),
                mgc_noise=t("mgc_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1),
                bap_noise=t("bap_noise")[:, 0].transpose(1, 2).contiguous().view(B * T, -1))


def _spk(B, T, E):
    """A per-sequence speaker vector expanded over frames, as the models pass it
    (multistream.py:1620-1628)."""
    return (0.3 * torch.randn(B, 1, E, device="cuda")).requires_grad_().expand(B, T, -1)


def _params(mod):
    return list(mod.parameters())


def _check_pair(fwd, fwd_args, bwd_name):
    """opcheck the forward op; returns the outputs of one more forward (whose saved state the
    backward op's check then uses)."""
    torch.library.opcheck(fwd, fwd_args, test_utils=FWD_TESTS)
    outs = fwd(*fwd_args)
    return outs


def _check_bwd(bwd, args):
    from torch._subclasses.fake_tensor import FakeTensorMode
    real = bwd(*args)
    real = real if isinstance(real, (tuple, list)) else (real,)
    with FakeTensorMode(allow_non_fake_inputs=True) as mode:
        fargs = [mode.from_tensor(a) if isinstance(a, torch.Tensor) else
                 ([None if t is None else mode.from_tensor(t) for t in a]
                  if isinstance(a, list) else a) for a in args]
        fake = bwd(*fargs)
    fake = fake if isinstance(fake, (tuple, list)) else (fake,)
    assert len(fake) == len(real)
    for f, r in zip(fake, real):
        assert tuple(f.shape) == tuple(r.shape) and f.dtype == r.dtype and \
            f.device == r.device, (tuple(f.shape), tuple(r.shape), f.dtype, r.dtype)


def test_opcheck_diffnet():
    model, a, meta, g = _tiny()
    net = model.mgc_model.denoise_fn
    B, T = 2, 48
    Mc = net.input_projection.in_channels
    E = net.residual_layers[0].conditioner_projection.in_channels
    r = torch.Generator(device="cuda").manual_seed(3)
    spec = (0.5 * torch.randn(B, 1, Mc, T, device="cuda", generator=r)).requires_grad_()
    cond = torch.randn(B, E, T, device="cuda", generator=r).requires_grad_()
    t = torch.tensor([3, 71], device="cuda")
    h = torch_ops.handle_of(net)
    out = _check_pair(torch.ops.ensvs.diffnet.default, (h, spec, t, cond, _params(net)),
                      "diffnet_bwd")
    _check_bwd(torch.ops.ensvs.diffnet_bwd.default,
               (h, out.detach(), torch.randn_like(out), E, torch_ops._flat_size(_params(net))))


@pytest.mark.parametrize("which", ["mgc", "vuv"])
def test_opcheck_ffconvlstm(which):
    model, a, meta, g = _tiny()
    enc = model.mgc_model.encoder if which == "mgc" else model.vuv_model
    if which == "vuv":
        enc.lstm.dropout = 0.1  # random: the op's seed makes it a pure function
    B, T = a["x_main"].shape[:2]
    x = torch.randn(B, T, enc.in_dim, device="cuda")
    spk = None
    if enc.embed_dim is not None:
        spk = _spk(B, T, enc.embed_dim)
    lens = torch.tensor(a["lengths"].tolist())
    h = torch_ops.handle_of(enc)
    out = _check_pair(torch.ops.ensvs.ffconvlstm.default,
                      (h, x, spk, lens, torch.tensor(12345), _params(enc)), "ffconvlstm_bwd")
    _check_bwd(torch.ops.ensvs.ffconvlstm_bwd.default,
               (h, out.detach(), torch.randn_like(out), torch_ops._flat_size(_params(enc))))


def test_opcheck_diffusion():
    model, a, meta, g = _tiny()
    gd = model.mgc_model
    B, T = a["x_main"].shape[:2]
    cond = torch.randn(B, T, gd.encoder.in_dim, device="cuda")
    y = torch.randn(B, T, gd.out_dim, device="cuda")
    spk = _spk(B, T, gd.encoder.embed_dim)
    lens = torch.tensor(a["lengths"].tolist())
    h = torch_ops.handle_of(gd)
    noise, xr = _check_pair(torch.ops.ensvs.diffusion_train.default,
                            (h, cond, y, spk, lens, torch.tensor(777), _params(gd)), "")
    _check_bwd(torch.ops.ensvs.diffusion_train_bwd.default,
               (h, xr.detach(), torch.randn_like(xr), torch_ops._flat_size(_params(gd))))


def test_opcheck_lf0():
    model, a, meta, g = _tiny()
    lm = model.lf0_model
    model._set_lf0_params()
    B, T = a["x_main"].shape[:2]
    E = lm.embed_dim
    s0, s1 = _spk(B, T, E), _spk(B, T, E)
    lens = torch.tensor(a["lengths"].tolist())
    h = torch_ops.handle_of(lm)
    lf0, res = _check_pair(torch.ops.ensvs.lf0_train.default,
                                   (h, g("x_main"), g("x_sub"), s0, s1, lens, None, torch.tensor(99),
                                    _params(lm)), "")
    _check_bwd(torch.ops.ensvs.lf0_train_bwd.default,
               (h, lf0.detach(), torch.randn_like(lf0), torch.randn_like(res),
                torch_ops._flat_size(_params(lm))))


def test_opcheck_multitrack():
    model, a, meta, g = _tiny()
    B, T = a["x_main"].shape[:2]
    model._replay_draws = _draws(a, B, T)
    lens = torch.from_numpy(a["lengths"]).cuda()
    h = torch_ops.handle_of(model)
    outs = _check_pair(torch.ops.ensvs.multitrack_train.default,
                               (h, g("x_main"), g("x_sub"), g("y_main"), g("spk_main"),
                                g("spk_sub"), lens, torch.tensor(5), _params(model)), "")
    grads = [None if i in (0, 4) else torch.randn_like(o) for i, o in enumerate(outs)]
    _check_bwd(torch.ops.ensvs.multitrack_train_bwd.default,
               (h, outs[1].detach(), grads, torch_ops._flat_size(_params(model))))


def test_opcheck_separate_f0_and_lstm_encoder():
    a, meta = load_case("sf0_train_tiny")
    model = build(configs.multitrack_separate_f0(num_speakers=4, tiny=True), meta["shapes"])
    for m in (model.mgc_model, model.vuv_model, model.bap_model, model.encoder):
        m.lstm.dropout = 0.0
    model.train()
    g = lambda k: torch.from_numpy(a[k]).cuda().contiguous()  # noqa: E731
    B, T = a["x_main"].shape[:2]
    model._replay_draws = dict(lf0_main=g("draw0::lf0_main").view(-1),
                               lf0_sub=g("draw0::lf0_sub").view(-1))
    lens = torch.from_numpy(a["lengths"]).cuda()
    h = torch_ops.handle_of(model)
    om, rm, os_, rs = _check_pair(
        torch.ops.ensvs.separate_f0_train.default,
        (h, g("x_main"), g("x_sub"), g("y_main"), g("y_sub"), g("spk_main"), g("spk_sub"), lens,
         torch.tensor(5), _params(model)), "")
    _check_bwd(torch.ops.ensvs.separate_f0_train_bwd.default,
               (h, om.detach(), torch.randn_like(om), torch.randn_like(rm), None, torch.randn_like(rs),
                torch_ops._flat_size(_params(model))))
    enc = model.encoder
    E = enc.embed_dim
    s0, s1 = _spk(B, T, E), _spk(B, T, E)
    he = torch_ops.handle_of(enc)
    out = _check_pair(torch.ops.ensvs.lstm_encoder.default,
                          (he, g("x_main"), g("x_sub"), s0, s1, lens.cpu(), _params(enc)), "")
    _check_bwd(torch.ops.ensvs.lstm_encoder_bwd.default,
               (he, out.detach(), torch.randn_like(out), torch_ops._flat_size(_params(enc))))


def test_opcheck_transformer_embedding_loss():
    from test_transformer import _case
    from ensemble_svs_with_interactions_amd.transformer import TransformerEncoder
    from golden_util import params_from_shapes
    _, m = _case("base")
    mod = TransformerEncoder(**dict(m["cfg"], dropout=0.2)).cuda()
    mod.load_state_dict(params_from_shapes(m["shapes"]))
    mod.train()
    B, T = 2, 40
    x = torch.randn(B, T, mod.in_dim, device="cuda").requires_grad_()
    lens = torch.tensor([40, 31])
    h = torch_ops.handle_of(mod)
    out = _check_pair(torch.ops.ensvs.transformer_encoder.default,
                      (h, x, lens, torch.tensor(4), _params(mod)), "")
    _check_bwd(torch.ops.ensvs.transformer_encoder_bwd.default,
               (h, out.detach(), torch.randn_like(out), T, True, torch_ops._flat_size(_params(mod))))
    table = torch.randn(4, 16, device="cuda").requires_grad_()
    idx = torch.tensor([[1], [3], [1]], device="cuda", dtype=torch.int32)
    torch.library.opcheck(torch.ops.ensvs.embedding_gather.default, (table, idx),
                          test_utils=FWD_TESTS)
    preds = [torch.randn(3, 24, n, device="cuda").requires_grad_() for n in (5, 1, 2)]
    targs = [torch.randn(3, 24, n, device="cuda") for n in (5, 1, 2)]
    torch.library.opcheck(torch.ops.ensvs.masked_l1.default,
                          (preds, targs, torch.tensor([24, 17, 9])), test_utils=FWD_TESTS)


def test_masked_l1_op_matches_reference_formula():
    """ensvs::masked_l1 = the reference's loss_feats / N (train_acoustic_multitrack.py:
    143-144, 173): L1 over the selected elements of every stream, summed, / their count."""
    r = torch.Generator(device="cuda").manual_seed(0)
    preds = [torch.randn(3, 24, n, device="cuda", generator=r).requires_grad_() for n in (5, 1, 2)]
    targs = [torch.randn(3, 24, n, device="cuda", generator=r) for n in (5, 1, 2)]
    lens = torch.tensor([24, 17, 9], device="cuda")
    loss = torch_ops.masked_l1_loss(preds, targs, lens)
    loss.backward()
    mask = (torch.arange(24, device="cuda")[None, :] < lens[:, None]).unsqueeze(-1)
    p2 = [p.detach().clone().requires_grad_() for p in preds]
    tot, n = 0, 0
    for p, q in zip(p2, targs):
        d = (p.masked_select(mask) - q.masked_select(mask)).abs()
        tot = tot + d.sum()
        n += d.numel()
    ref = tot / n
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-6 * abs(ref.item())
    for p, q in zip(preds, p2):
        assert torch.allclose(p.grad, q.grad, atol=1e-9, rtol=1e-6)


@pytest.mark.parametrize("backend", ["aot_eager", "inductor"])
def test_dropin_model_under_torch_compile(backend):
    """torch.compile(model, fullgraph=False) around the drop-in model: the reference-style
    loss (tests/test_dropin_gpu.py) and every parameter gradient equal the eager run's."""
    from test_dropin_gpu import _reference_style_loss
    torch._dynamo.reset()
    res = []
    for compiled in (False, True):
        model, a, meta, g = _tiny()
        B, T = a["x_main"].shape[:2]
        model._replay_draws = _draws(a, B, T)
        lens = torch.from_numpy(a["lengths"]).cuda()
        run = torch.compile(model, backend=backend, fullgraph=False) if compiled else model
        model.zero_grad(set_to_none=True)
        loss = _reference_style_loss(run, g("x_main"), g("x_sub"), g("y_main"), g("y_sub"),
                                     (g("spk_main"), g("spk_sub")), lens, 0.0, [60, 1, 1, 5])
        loss.backward()
        torch.cuda.synchronize()
        res.append((loss.item(), {k: p.grad.detach().clone() for k, p in
                                  model.named_parameters()}))
    (l0, g0), (l1, g1) = res
    assert abs(l0 - meta["losses"][0]) < 1e-5 * abs(meta["losses"][0])
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    num = sum(((g1[k] - g0[k]) ** 2).sum().item() for k in g0) ** 0.5
    den = sum((g0[k] ** 2).sum().item() for k in g0) ** 0.5
    assert num / den < 1e-6, num / den
