"""PyTorch custom ops (torch.library) over the HIP training path -- the boundary SURVEY §8(b)
names: every reference module whose forward runs our kernels is one op pair registered with
``torch.library.custom_op`` (forward) + ``register_autograd`` (its backward, itself an op)
+ ``register_fake`` (shape functions), so autograd, ``torch.compile`` / ``torch.export`` and
``torch.library.opcheck`` see ordinary operators instead of opaque Python.

    ensvs::multitrack_train   MultiTrackNPSSMDNMultistreamParametricModel / NPSSMDN... .forward
                              with targets (multistream.py:1594-1768, 1025-1243)
    ensvs::separate_f0_train  MultiTrackMultistreamSeparateF0ParametricModel.forward
                              (multistream.py:348-577)
    ensvs::lf0_train          MultiTrackBiLSTMResF0NonAttentiveDecoder.forward + its AR
                              residual-F0 decoder (tacotron_f0.py:924-991, 126-237)
    ensvs::ffconvlstm         FFConvLSTM.forward (nnsvs/model.py:891-918)
    ensvs::diffusion_train    GaussianDiffusion.forward (diffusion.py:269-300)
    ensvs::diffnet            DiffNet.forward (denoiser.py:101-124)
    ensvs::masked_l1          the masked L1 feature loss (train_acoustic_multitrack.py:92-184)
each with a ``*_bwd`` op.  The modules' forward methods call these (the reference's call
sites: train_acoustic_multitrack.py:94-100, gen.py:1290-1292).

Functional form.  A module is named by an integer handle (``handle_of``); its parameters are
an explicit ``Tensor[]`` input, so autograd returns their gradients (one flat buffer from the
backward op, split into views laid out like engine.GradCapture).  Randomness (diffusion
steps / noise, the AR decoder's always-on prenet dropout, the V/UV LSTM dropout) comes from
an explicit ``seed`` argument (engine.seed_scope), so an op is a pure function of its inputs.
What the backward kernels read (saved activations, gates, BN statistics) stays on the device,
filed under the forward's first output: the autograd formula saves that output and hands it
to the backward op, which finds the state by its storage (no extra output, so the forward's
results are deterministic functions of its inputs).
"""
import collections
import itertools
import weakref
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import engine
from .engine import GradCapture, lengths_pair

_MODS = {}
_NEXT = itertools.count(1)
_SAVED = collections.OrderedDict()  # (device, data_ptr) of the key output -> saved state
MAX_SAVED = 64  # forwards whose backward never ran are dropped past this many
ALIGN = 64       # engine.GradCapture's per-parameter alignment


def handle_of(mod) -> int:
    h = getattr(mod, "_ensvs_handle", None)
    if h is None or _MODS.get(h, lambda: None)() is not mod:
        h = next(_NEXT)
        mod._ensvs_handle = h
        _MODS[h] = weakref.ref(mod)
    return h


def _mod(handle):
    m = _MODS.get(int(handle), lambda: None)()
    if m is None:
        raise RuntimeError(f"ensvs op: module handle {handle} is gone")
    return m


def _key(t):
    return (str(t.device), t.untyped_storage().data_ptr())


def _keep(state, out):
    """File the forward's saved state under its output `out`; returns `out`."""
    k = _key(out)
    _SAVED.pop(k, None)
    _SAVED[k] = state
    while len(_SAVED) > MAX_SAVED:
        _SAVED.popitem(last=False)
    return out


def _take(key_out):
    k = _key(key_out)
    st = _SAVED.pop(k, None)
    if st is None:
        raise RuntimeError("ensvs op: the forward state of this backward is gone (backward "
                           "called twice, or more than MAX_SAVED forwards in flight)")
    return st


def peek(out):
    """The saved forward state filed under the output `out` (or a view of it), not consumed
    (tests read the device's intermediate decisions from it)."""
    st = _SAVED.get(_key(out))
    if st is None:
        raise KeyError("ensvs op: no forward state saved under this output")
    return st


def _flat_size(params):
    return max(sum((p.numel() + ALIGN - 1) // ALIGN * ALIGN for p in params), 1)


def _split_flat(g, shapes):
    """Per-parameter views of a flat gradient buffer (GradCapture's layout)."""
    out, o = [], 0
    for shp in shapes:
        n = 1
        for d in shp:
            n *= d
        out.append(g[o:o + n].view(shp))
        o += (n + ALIGN - 1) // ALIGN * ALIGN
    return out


def _new_seed():
    """The op's randomness: a CPU int64 tensor from torch's generator (torch.manual_seed makes
    it reproducible; a tensor, so torch.compile neither specialises nor graph-breaks on it)."""
    return torch.randint(0, 1 << 62, (), dtype=torch.int64)


def _spk_rows(spk, B, T):
    """Per-sequence speaker vectors (B, E) contiguous, and their row stride, from a (B, T, E)
    speaker input: the reference expands a (B, 1, E) vector over frames (multistream.py:
    1620-1628); a materialised copy of such an expansion is accepted after checking that every
    frame holds the first frame's vector (per-frame vectors are not on the path).  The op keeps
    the rows with its saved state."""
    if spk is None:
        return None, 0
    first = spk[:, 0, :]
    if spk.stride(1) != 0 and not torch.equal(spk, first.unsqueeze(1).expand_as(spk)):
        raise NotImplementedError("per-frame speaker embeddings are not on the path")
    rows = first.contiguous().float()
    return rows, rows.shape[1]


def _lengths_arg(lengths, B, T, device):
    """Module-call lengths (None / list / tensor) as the op's Optional[Tensor]."""
    if lengths is None or isinstance(lengths, torch.Tensor):
        return lengths
    return lengths_pair(lengths, B, T, device)[1]


def _setup_params(ctx, params, handle=None):
    """Per-parameter shapes and the flat gradient size, from the module's own (concrete)
    parameters: under symbolic tracing the `params` input carries symbolic sizes, and a sum
    over ~200 of them as nflat overflows the tracer's recursion."""
    src = list(_mod(handle).parameters()) if handle is not None else params
    ctx.param_shapes = [tuple(int(d) for d in p.shape) for p in src]
    ctx.nflat = _flat_size(src)


def _param_grads(ctx, gflat):
    needs = ctx.needs_input_grad[-1]
    if isinstance(needs, (list, tuple)) and not any(needs):
        return None
    return _split_flat(gflat, ctx.param_shapes)


# ============================================================================== DiffNet
@torch.library.custom_op("ensvs::diffnet", mutates_args=())
def diffnet(handle: int, spec: Tensor, t: Tensor, cond: Tensor,
            params: List[Tensor]) -> Tensor:
    """denoiser.py:101-124: spec (B, 1, M, T), diffusion step (B,), cond (B, E, T)."""
    mod = _mod(handle)
    B, _, Mc, T = spec.shape
    E = cond.shape[1]
    xin = spec[:, 0].transpose(1, 2).contiguous().view(B * T, Mc)
    cnd = cond.transpose(1, 2).contiguous().view(B * T, E)
    out, st = mod._fwd(xin, Mc, t.to(device=spec.device, dtype=torch.int64).contiguous(), cnd,
                       E, B, T)
    return _keep(st, out.view(B, T, Mc).transpose(1, 2).unsqueeze(1).contiguous())


@diffnet.register_fake
def _(handle, spec, t, cond, params):
    return torch.empty_like(spec, memory_format=torch.contiguous_format)


@torch.library.custom_op("ensvs::diffnet_bwd", mutates_args=())
def diffnet_bwd(handle: int, out: Tensor, grad: Tensor, E: int,
                nflat: int) -> Tuple[Tensor, Tensor]:
    mod = _mod(handle)
    st = _take(out)
    B, _, Mc, T = grad.shape
    dout = grad[:, 0].transpose(1, 2).contiguous().view(B * T, Mc)
    with GradCapture(list(mod.parameters())) as gc:
        dcond = mod._bwd(st, dout)
    return dcond.view(B, T, E).transpose(1, 2).contiguous(), gc.buf


@diffnet_bwd.register_fake
def _(handle, out, grad, E, nflat):
    B, _, _, T = grad.shape
    return grad.new_empty(B, E, T), grad.new_empty(nflat)


def _diffnet_setup(ctx, inputs, output):
    handle, spec, t, cond, params = inputs
    ctx.handle, ctx.E = handle, cond.shape[1]
    ctx.save_for_backward(output)
    _setup_params(ctx, params, handle)


def _diffnet_backward(ctx, g_out):
    (out,) = ctx.saved_tensors
    dcond, gflat = torch.ops.ensvs.diffnet_bwd(ctx.handle, out, g_out.contiguous(), ctx.E,
                                               ctx.nflat)
    return None, None, None, dcond, _param_grads(ctx, gflat)


diffnet.register_autograd(_diffnet_backward, setup_context=_diffnet_setup)


def diffnet_call(mod, spec, diffusion_step, cond):
    return torch.ops.ensvs.diffnet(handle_of(mod), spec, diffusion_step, cond,
                                   list(mod.parameters()))


# ============================================================================ FFConvLSTM
@torch.library.custom_op("ensvs::ffconvlstm", mutates_args=())
def ffconvlstm(handle: int, x: Tensor, spk_embs: Optional[Tensor], lengths: Optional[Tensor],
               seed: Tensor, params: List[Tensor]) -> Tensor:
    """model.py:891-918 over all T frames (the caller trims to max(lengths), as
    pad_packed_sequence does)."""
    mod = _mod(handle)
    B, T, D = x.shape
    x = x.contiguous().float()
    _, lens_dev = lengths_pair(lengths, B, T, x.device)
    spk, spk_ld = _spk_rows(spk_embs, B, T)
    with engine.seed_scope(int(seed)):
        out, st = mod._fwd([(x, D, 0, D)], B, T, lens_dev, spk, spk_ld, save=True)
    st["_keep_spk"] = spk
    return _keep(st, out.view(B, T, -1))


@ffconvlstm.register_fake
def _(handle, x, spk_embs, lengths, seed, params):
    B, T, _ = x.shape
    return x.new_empty(B, T, _mod(handle).out_dim, dtype=torch.float32)


@torch.library.custom_op("ensvs::ffconvlstm_bwd", mutates_args=())
def ffconvlstm_bwd(handle: int, out: Tensor, grad: Tensor, nflat: int) -> Tuple[Tensor, Tensor]:
    """Returns (d of the fused input per frame = d spk_embs (B, T, E) or (B, T, 0), flat
    parameter gradients)."""
    mod = _mod(handle)
    st = _take(out)
    B, T = st["B"], st["T"]
    with GradCapture(list(mod.parameters())) as gc:
        dX0, _ = mod._bwd(st, grad.contiguous().view(B * T, -1), want_spk=False)
    return dX0.view(B, T, -1).contiguous(), gc.buf


@ffconvlstm_bwd.register_fake
def _(handle, out, grad, nflat):
    B, T, _ = grad.shape
    m = _mod(handle)
    return grad.new_empty(B, T, m.embed_dim or m.in_dim), grad.new_empty(nflat)


def _ffconvlstm_setup(ctx, inputs, output):
    handle, x, spk_embs, lengths, seed, params = inputs
    ctx.handle = handle
    ctx.save_for_backward(output)
    ctx.spk = spk_embs is not None
    _setup_params(ctx, params, handle)


def _ffconvlstm_backward(ctx, g_out):
    (out,) = ctx.saved_tensors
    d, gflat = torch.ops.ensvs.ffconvlstm_bwd(ctx.handle, out, g_out, ctx.nflat)
    dspk = d if ctx.spk and ctx.needs_input_grad[2] else None
    return None, None, dspk, None, None, _param_grads(ctx, gflat)


ffconvlstm.register_autograd(_ffconvlstm_backward, setup_context=_ffconvlstm_setup)


def ffconvlstm_call(mod, x, spk_embs, lengths):
    B, T, _ = x.shape
    lens = _lengths_arg(lengths, B, T, x.device)
    out = torch.ops.ensvs.ffconvlstm(handle_of(mod), x, spk_embs, lens, _new_seed(),
                                     list(mod.parameters()))
    Tm = T if lengths is None else int(max(lengths_pair(lengths, B, T, x.device)[0]))
    return out[:, :Tm] if Tm < T else out


# ================================================================= GaussianDiffusion
@torch.library.custom_op("ensvs::diffusion_train", mutates_args=())
def diffusion_train(handle: int, cond: Tensor, y: Tensor, spk_embs: Optional[Tensor],
                    lengths: Optional[Tensor], seed: Tensor,
                    params: List[Tensor]) -> Tuple[Tensor, Tensor]:
    """diffusion.py:269-300: (noise, x_recon); t ~ U{0..K-1} and the noise from `seed`."""
    mod = _mod(handle)
    B, T, D = cond.shape
    cond = cond.contiguous().float()
    y = y.contiguous().float()
    _, lens_dev = lengths_pair(lengths, B, T, cond.device)
    spk, spk_ld = _spk_rows(spk_embs, B, T)
    with engine.seed_scope(int(seed)):
        noise, xr, st = mod._fwd([(cond, D, 0, D)], B, T, lens_dev, (y, y.shape[2], 0), spk,
                                 spk_ld)
    st["_keep_spk"] = (spk, y)
    return noise.view(B, T, -1), _keep(st, xr.view(B, T, -1))


@diffusion_train.register_fake
def _(handle, cond, y, spk_embs, lengths, seed, params):
    B, T, _ = cond.shape
    M = _mod(handle).out_dim
    return cond.new_empty(B, T, M), cond.new_empty(B, T, M)


@torch.library.custom_op("ensvs::diffusion_train_bwd", mutates_args=())
def diffusion_train_bwd(handle: int, x_recon: Tensor, grad_recon: Tensor,
                        nflat: int) -> Tuple[Tensor, Tensor]:
    mod = _mod(handle)
    st = _take(x_recon)
    B, T, _ = grad_recon.shape
    with GradCapture(list(mod.parameters())) as gc:
        dcond = mod.denoise_fn._bwd(st["dst"], grad_recon.contiguous().view(B * T, -1))
        dX0, _ = mod.encoder._bwd(st["est"], dcond, want_spk=False)
    return dX0.view(B, T, -1).contiguous(), gc.buf


@diffusion_train_bwd.register_fake
def _(handle, x_recon, grad_recon, nflat):
    B, T, _ = grad_recon.shape
    enc = _mod(handle).encoder
    return grad_recon.new_empty(B, T, enc.embed_dim or enc.in_dim), grad_recon.new_empty(nflat)


def _diffusion_setup(ctx, inputs, output):
    handle, cond, y, spk_embs, lengths, seed, params = inputs
    ctx.handle = handle
    ctx.save_for_backward(output[1])
    ctx.spk = spk_embs is not None
    _setup_params(ctx, params, handle)


def _diffusion_backward(ctx, g_noise, g_recon):
    # the noise output is the random target (not differentiable): its gradient is dropped
    (xr,) = ctx.saved_tensors
    if g_recon is None:
        g_recon = torch.zeros_like(xr)
    d, gflat = torch.ops.ensvs.diffusion_train_bwd(ctx.handle, xr, g_recon, ctx.nflat)
    dspk = d if ctx.spk and ctx.needs_input_grad[3] else None
    return None, None, None, dspk, None, None, _param_grads(ctx, gflat)


diffusion_train.register_autograd(_diffusion_backward, setup_context=_diffusion_setup)


def diffusion_call(mod, cond, lengths, y, spk_embs):
    B, T, _ = cond.shape
    noise, xr = torch.ops.ensvs.diffusion_train(
        handle_of(mod), cond, y, spk_embs, _lengths_arg(lengths, B, T, cond.device),
        _new_seed(), list(mod.parameters()))
    return noise, xr


# ============================================================== multi-track lf0 model
@torch.library.custom_op("ensvs::lf0_train", mutates_args=())
def lf0_train(handle: int, x_main: Tensor, x_sub: Optional[Tensor], spk_emb_main: Optional[Tensor],
              spk_emb_sub: Optional[Tensor], lengths: Optional[Tensor], y: Optional[Tensor],
              seed: Tensor, params: List[Tensor]) -> Tuple[Tensor, Tensor]:
    """tacotron_f0.py:924-991 (+ the AR decoder, free-running unless y is given): (lf0,
    lf0_residual), each (B, T, 1); the prenet dropout masks from `seed`."""
    mod = _mod(handle)
    B, T, D = x_main.shape
    xs = [x_main.contiguous().float()]
    if x_sub is not None:
        xs.append(x_sub.contiguous().float())
    _, lens_dev = lengths_pair(lengths, B, T, x_main.device)
    p0, ld0 = _spk_rows(spk_emb_main, B, T)
    p1, ld1 = _spk_rows(spk_emb_sub, B, T)
    teacher = None
    if y is not None:
        if y.shape[1] != T:
            raise ValueError("decoder targets must have the input's frame count "
                             "(tacotron_f0.py:139)")
        yc = y.contiguous().float()
        teacher = (yc, yc.shape[2], mod.decoder.out_lf0_idx)
    with engine.seed_scope(int(seed)):
        lf0, res, st = mod._fwd(xs, D, B, T, lens_dev, (p0, p1), ld0, teacher=teacher)
    st["_keep"] = (teacher, p0, p1)  # buffers the saved state points into
    return _keep(st, lf0.view(B, T, 1)), res.view(B, T, 1)


@lf0_train.register_fake
def _(handle, x_main, x_sub, spk_emb_main, spk_emb_sub, lengths, y, seed, params):
    B, T, _ = x_main.shape
    return (x_main.new_empty(B, T, 1, dtype=torch.float32),
            x_main.new_empty(B, T, 1, dtype=torch.float32))


@torch.library.custom_op("ensvs::lf0_train_bwd", mutates_args=())
def lf0_train_bwd(handle: int, lf0: Tensor, grad_lf0: Tensor, grad_res: Optional[Tensor],
                  nflat: int) -> Tuple[Tensor, Tensor]:
    """(d of the fused per-frame input = d of each expanded speaker embedding (B, T, E), flat
    parameter gradients)."""
    mod = _mod(handle)
    st = _take(lf0)
    B, T = st["B"], st["T"]
    gl = grad_lf0.contiguous().view(-1)
    gr = grad_res.contiguous().view(-1) if grad_res is not None else None
    with GradCapture(list(mod.parameters())) as gc:
        _, _, dX0 = mod._bwd(st, gl, gr, want_spk=False)
    return dX0.view(B, T, -1).contiguous(), gc.buf


@lf0_train_bwd.register_fake
def _(handle, lf0, grad_lf0, grad_res, nflat):
    B, T, _ = grad_lf0.shape
    return grad_lf0.new_empty(B, T, _mod(handle).embed_dim), grad_lf0.new_empty(nflat)


def _lf0_setup(ctx, inputs, output):
    handle, x_main, x_sub, s0, s1, lengths, y, seed, params = inputs
    ctx.handle = handle
    ctx.save_for_backward(output[0])
    ctx.spk = (s0 is not None, s1 is not None)
    _setup_params(ctx, params, handle)


def _lf0_backward(ctx, g_lf0, g_res):
    (lf0,) = ctx.saved_tensors
    if g_lf0 is None:
        g_lf0 = torch.zeros_like(lf0)
    d, gflat = torch.ops.ensvs.lf0_train_bwd(ctx.handle, lf0, g_lf0, g_res, ctx.nflat)
    d0 = d if ctx.spk[0] and ctx.needs_input_grad[3] else None
    d1 = d if ctx.spk[1] and ctx.needs_input_grad[4] else None
    return None, None, None, d0, d1, None, None, None, _param_grads(ctx, gflat)


lf0_train.register_autograd(_lf0_backward, setup_context=_lf0_setup)


def lf0_call(mod, x_main, x_sub, spk_emb_main, spk_emb_sub, lengths, y):
    B, T, _ = x_main.shape
    lf0, res = torch.ops.ensvs.lf0_train(
        handle_of(mod), x_main, x_sub, spk_emb_main, spk_emb_sub,
        _lengths_arg(lengths, B, T, x_main.device), y, _new_seed(), list(mod.parameters()))
    return lf0, res


# ===================================================== multi-track acoustic model (pair step)
def _mt_widths(mod):
    s = mod.stream_sizes
    return [s[0], s[0], 1, 1, s[3], s[3], 1]


def _mt_has_sub(mod):
    return bool(getattr(mod, "output_subtrack", False)) and getattr(mod, "_MULTI", False)


@torch.library.custom_op("ensvs::multitrack_train", mutates_args=())
def multitrack_train(handle: int, x_main: Tensor, x_sub: Optional[Tensor], y_main: Tensor,
                     spk_main: Optional[Tensor], spk_sub: Optional[Tensor],
                     lengths: Optional[Tensor], seed: Tensor,
                     params: List[Tensor]) -> List[Tensor]:
    """multistream.py:1594-1768 training forward: [mgc noise, mgc x_recon, lf0, vuv, bap
    noise, bap x_recon, lf0_residual (+ lf0_sub, lf0_residual_sub with output_subtrack)], each
    (B, T, n).  Random draws from `seed` (or the module's _replay_draws, tests)."""
    mod = _mod(handle)
    B, T, _ = x_main.shape
    with engine.seed_scope(int(seed)):
        outs, st = mod._train_fwd(x_main.contiguous().float(),
                                  None if x_sub is None else x_sub.contiguous().float(),
                                  y_main.contiguous().float(), spk_main, spk_sub, lengths,
                                  getattr(mod, "_replay_draws", None))
    v = lambda t: t.view(B, T, -1)  # noqa: E731
    ret = [v(outs["mgc_noise"]), _keep(st, v(outs["mgc_recon"])), v(outs["lf0"]), v(outs["vuv"]),
           v(outs["bap_noise"]), v(outs["bap_recon"]), v(outs["lf0_residual"])]
    if "lf0_sub" in outs:
        ret += [v(outs["lf0_sub"]), v(outs["lf0_residual_sub"])]
    return ret


@multitrack_train.register_fake
def _(handle, x_main, x_sub, y_main, spk_main, spk_sub, lengths, seed, params):
    mod = _mod(handle)
    B, T, _ = x_main.shape
    w = _mt_widths(mod) + ([1, 1] if _mt_has_sub(mod) else [])
    return [x_main.new_empty(B, T, n, dtype=torch.float32) for n in w]


@torch.library.custom_op("ensvs::multitrack_train_bwd", mutates_args=())
def multitrack_train_bwd(handle: int, mgc_recon: Tensor, grads: List[Optional[Tensor]],
                         nflat: int) -> Tensor:
    """Flat parameter gradients of the pair step for the output gradients `grads` (the
    forward's order; None = zero)."""
    mod = _mod(handle)
    st = _take(mgc_recon)
    B, T = st["B"], st["T"]
    dev = st["lens_dev"].device
    widths = _mt_widths(mod)

    def flat(g, n):
        return torch.zeros(B * T, n, device=dev) if g is None else g.contiguous().view(B * T, n)
    grads = list(grads) + [None] * (9 - len(grads))
    g = dict(mgc_recon=flat(grads[1], widths[1]), lf0=flat(grads[2], 1).view(-1),
             vuv=flat(grads[3], 1), bap_recon=flat(grads[5], widths[5]))
    if grads[6] is not None:
        g["lf0_residual"] = grads[6].contiguous().view(-1)
    if grads[7] is not None:
        g["lf0_sub"] = grads[7].contiguous().view(-1)
    if grads[8] is not None:
        g["lf0_residual_sub"] = grads[8].contiguous().view(-1)
    with GradCapture(list(mod.parameters())) as gc:
        mod._train_bwd(st, g)
    return gc.buf


@multitrack_train_bwd.register_fake
def _(handle, mgc_recon, grads, nflat):
    return mgc_recon.new_empty(nflat)


def _mt_setup(ctx, inputs, output):
    ctx.handle = inputs[0]
    ctx.save_for_backward(output[1])
    _setup_params(ctx, inputs[-1], inputs[0])


def _mt_backward(ctx, g_outs):
    (mgc_recon,) = ctx.saved_tensors
    gs = list(g_outs)
    gs[0] = gs[4] = None  # the diffusion noise targets are not differentiable
    if all(g is None for g in gs):
        gs[1] = torch.zeros_like(mgc_recon)
    gflat = torch.ops.ensvs.multitrack_train_bwd(ctx.handle, mgc_recon, gs, ctx.nflat)
    return None, None, None, None, None, None, None, None, _param_grads(ctx, gflat)


multitrack_train.register_autograd(_mt_backward, setup_context=_mt_setup)


def multitrack_call(mod, x_main, x_sub, y_main, spk_main, spk_sub, lengths):
    B, T, _ = x_main.shape
    outs = torch.ops.ensvs.multitrack_train(
        handle_of(mod), x_main, x_sub, y_main, spk_main, spk_sub,
        _lengths_arg(lengths, B, T, x_main.device), _new_seed(), list(mod.parameters()))
    return outs


# ========================================================= SeparateF0 recipe model (pair step)
@torch.library.custom_op("ensvs::separate_f0_train", mutates_args=())
def separate_f0_train(handle: int, x_main: Tensor, x_sub: Tensor, y_main: Tensor, y_sub: Tensor,
                      spk_main: Optional[Tensor], spk_sub: Optional[Tensor],
                      lengths: Optional[Tensor], seed: Tensor,
                      params: List[Tensor]) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """multistream.py:348-577 training forward: (main out, main lf0 residual, sub out, sub lf0
    residual)."""
    mod = _mod(handle)
    B, T, _ = x_main.shape
    f = lambda t: t.contiguous().float()  # noqa: E731
    with engine.seed_scope(int(seed)):
        outs, st = mod._fwd_core(f(x_main), f(x_sub), f(y_main), f(y_sub), spk_main, spk_sub,
                                 lengths, mod.training, True, getattr(mod, "_replay_draws", None))
    v = lambda t: t.view(B, T, -1)  # noqa: E731
    return (_keep(st, v(mod._assemble(outs))), v(outs["lf0_residual"]),
            v(mod._assemble(outs, "_sub")), v(outs["lf0_residual_sub"]))


@separate_f0_train.register_fake
def _(handle, x_main, x_sub, y_main, y_sub, spk_main, spk_sub, lengths, seed, params):
    mod = _mod(handle)
    B, T, _ = x_main.shape
    D = mod.out_dim
    e = lambda n: x_main.new_empty(B, T, n, dtype=torch.float32)  # noqa: E731
    return e(D), e(1), e(D), e(1)


@torch.library.custom_op("ensvs::separate_f0_train_bwd", mutates_args=())
def separate_f0_train_bwd(handle: int, out_main: Tensor, g_out_main: Optional[Tensor],
                          g_res_main: Optional[Tensor], g_out_sub: Optional[Tensor],
                          g_res_sub: Optional[Tensor], nflat: int) -> Tensor:
    mod = _mod(handle)
    st = _take(out_main)
    B, T = st["B"], st["T"]
    g = {}
    for gg, sfx in ((g_out_main, ""), (g_out_sub, "_sub")):
        if gg is not None:
            mod._split(gg.contiguous().view(B * T, -1), sfx, g)
    if g_res_main is not None:
        g["lf0_residual"] = g_res_main.contiguous().view(-1)
    if g_res_sub is not None:
        g["lf0_residual_sub"] = g_res_sub.contiguous().view(-1)
    with GradCapture(list(mod.parameters())) as gc:
        mod._bwd_core(st, g)
    return gc.buf


@separate_f0_train_bwd.register_fake
def _(handle, out_main, g_out_main, g_res_main, g_out_sub, g_res_sub, nflat):
    return out_main.new_empty(nflat)


def _sf0_setup(ctx, inputs, output):
    ctx.handle = inputs[0]
    ctx.save_for_backward(output[0])
    _setup_params(ctx, inputs[-1], inputs[0])


def _sf0_backward(ctx, g_om, g_rm, g_os, g_rs):
    (om,) = ctx.saved_tensors
    if all(g is None for g in (g_om, g_rm, g_os, g_rs)):
        g_om = torch.zeros_like(om)
    gflat = torch.ops.ensvs.separate_f0_train_bwd(ctx.handle, om, g_om, g_rm, g_os, g_rs,
                                                  ctx.nflat)
    return (None,) * 9 + (_param_grads(ctx, gflat),)


separate_f0_train.register_autograd(_sf0_backward, setup_context=_sf0_setup)


def separate_f0_call(mod, x_main, x_sub, y_main, y_sub, spk_main, spk_sub, lengths):
    B, T, _ = x_main.shape
    om, rm, os_, rs = torch.ops.ensvs.separate_f0_train(
        handle_of(mod), x_main, x_sub, y_main, y_sub, spk_main, spk_sub,
        _lengths_arg(lengths, B, T, x_main.device), _new_seed(), list(mod.parameters()))
    return om, rm, os_, rs


# ==================================================================== masked L1 loss
@torch.library.custom_op("ensvs::masked_l1", mutates_args=())
def masked_l1(preds: List[Tensor], targets: List[Tensor],
              lengths: Tensor) -> Tuple[Tensor, List[Tensor]]:
    """train_acoustic_multitrack.py:92-184 (feats_criterion l1): the L1 distance of every
    (pred, target) pair over the first lengths[b] frames, SUMMED over all selected elements of
    all streams and divided by their total count (not a mean of per-stream means).  preds /
    targets (B, T, n_i); returns (loss (), d loss / d pred_i for each stream)."""
    from .train import masked_l1 as _kernel
    B, T, _ = preds[0].shape
    host, lens_dev = lengths_pair(lengths, B, T, preds[0].device)
    P = [p.contiguous().float() for p in preds]
    Q = [q.contiguous().float() for q in targets]
    loss, grads = _kernel([(p, p.shape[2], 0, p.shape[2]) for p in P],
                          [(q, q.shape[2], 0) for q in Q], lens_dev, sum(host), B, T)
    return loss.view(()), [g.view(B, T, -1) for g in grads]


@masked_l1.register_fake
def _(preds, targets, lengths):
    return preds[0].new_empty((), dtype=torch.float32), \
        [p.new_empty(p.shape, dtype=torch.float32) for p in preds]


def _ml1_setup(ctx, inputs, output):
    ctx.save_for_backward(*output[1])


def _ml1_backward(ctx, g_loss, g_grads):
    gs = ctx.saved_tensors
    dp = [g_loss * g for g in gs]
    return dp, [-d for d in dp], None  # (L1: the targets' gradient is the negation)


masked_l1.register_autograd(_ml1_backward, setup_context=_ml1_setup)


def masked_l1_loss(preds, targets, lengths):
    """The reference's masked L1 feature loss over (pred, target) stream pairs as one op."""
    loss, _ = torch.ops.ensvs.masked_l1(list(preds), list(targets), lengths)
    return loss


# ================================================== MultiTrackLSTMEncoder (concat fusion)
@torch.library.custom_op("ensvs::lstm_encoder", mutates_args=())
def lstm_encoder(handle: int, x_main: Tensor, x_sub: Tensor, spk_main: Optional[Tensor],
                 spk_sub: Optional[Tensor], lengths: Optional[Tensor],
                 params: List[Tensor]) -> Tensor:
    """nnsvs/model.py:1435-1537 over all T frames (the caller trims to max(lengths))."""
    mod = _mod(handle)
    B, T, D = x_main.shape
    _, lens_dev = lengths_pair(lengths, B, T, x_main.device)
    p0, ld0 = _spk_rows(spk_main, B, T)
    p1, ld1 = _spk_rows(spk_sub, B, T)
    if ld0 != ld1:
        raise NotImplementedError("the two speaker inputs must share one layout")
    out, st = mod._fwd(x_main.contiguous().float(), x_sub.contiguous().float(), D, B, T,
                       lens_dev, (p0, p1), ld0)
    st["_keep_spk"] = (p0, p1)
    return _keep(st, out.view(B, T, -1))


@lstm_encoder.register_fake
def _(handle, x_main, x_sub, spk_main, spk_sub, lengths, params):
    B, T, _ = x_main.shape
    return x_main.new_empty(B, T, _mod(handle).out_dim, dtype=torch.float32)


@torch.library.custom_op("ensvs::lstm_encoder_bwd", mutates_args=())
def lstm_encoder_bwd(handle: int, out: Tensor, grad: Tensor,
                     nflat: int) -> Tuple[Tensor, Tensor]:
    """(d of the fused (B, T, 2E) LSTM input: [d spk_main | d spk_sub] per frame, flat
    parameter gradients)."""
    mod = _mod(handle)
    st = _take(out)
    B, T = st["B"], st["T"]
    with GradCapture(list(mod.parameters())) as gc:
        _, _, dX = mod._bwd(st, grad.contiguous().view(B * T, -1), want_spk=False)
    return dX.view(B, T, -1).contiguous(), gc.buf


@lstm_encoder_bwd.register_fake
def _(handle, out, grad, nflat):
    B, T, _ = grad.shape
    return grad.new_empty(B, T, 2 * _mod(handle).embed_dim), grad.new_empty(nflat)


def _lstm_enc_setup(ctx, inputs, output):
    handle, x_main, x_sub, s0, s1, lengths, params = inputs
    ctx.handle = handle
    ctx.save_for_backward(output)
    ctx.spk = (s0 is not None, s1 is not None)
    ctx.E = _mod(handle).embed_dim
    _setup_params(ctx, params, handle)


def _lstm_enc_backward(ctx, g_out):
    (out,) = ctx.saved_tensors
    d, gflat = torch.ops.ensvs.lstm_encoder_bwd(ctx.handle, out, g_out, ctx.nflat)
    E = ctx.E
    d0 = d[:, :, :E] if ctx.spk[0] and ctx.needs_input_grad[3] else None
    d1 = d[:, :, E:] if ctx.spk[1] and ctx.needs_input_grad[4] else None
    return None, None, None, d0, d1, None, _param_grads(ctx, gflat)


lstm_encoder.register_autograd(_lstm_enc_backward, setup_context=_lstm_enc_setup)


def lstm_encoder_call(mod, x_main, x_sub, spk_main, spk_sub, lengths):
    B, T, _ = x_main.shape
    out = torch.ops.ensvs.lstm_encoder(handle_of(mod), x_main, x_sub, spk_main, spk_sub,
                                       _lengths_arg(lengths, B, T, x_main.device),
                                       list(mod.parameters()))
    Tm = T if lengths is None else int(max(lengths_pair(lengths, B, T, x_main.device)[0]))
    return out[:, :Tm] if Tm < T else out


# ============================================================ Transformer encoder (tier 2)
@torch.library.custom_op("ensvs::transformer_encoder", mutates_args=())
def transformer_encoder(handle: int, x: Tensor, lengths: Optional[Tensor], seed: Tensor,
                        params: List[Tensor]) -> Tensor:
    """nnsvs/model.py:1540-1671 (transformer/encoder.py:82-142): (B, T / r, out * r)."""
    mod = _mod(handle)
    B, T, D = x.shape
    if D != mod.in_dim:
        raise ValueError(f"TransformerEncoder: input has {D} channels, expected {mod.in_dim}")
    lens_host, _ = lengths_pair(lengths, B, T, x.device)
    with engine.seed_scope(int(seed)):
        out, st = mod._fwd(x.contiguous().float().view(B * T, D), B, T, lens_host)
    return _keep(st, out.view(B, -1, mod.out_dim))


def _tf_frames(mod, T):
    r = mod.reduction_factor
    return (T // r) * r if r > 1 else T


@transformer_encoder.register_fake
def _(handle, x, lengths, seed, params):
    mod = _mod(handle)
    B, T, _ = x.shape
    return x.new_empty(B, _tf_frames(mod, T), mod.out_dim, dtype=torch.float32)


@torch.library.custom_op("ensvs::transformer_encoder_bwd", mutates_args=())
def transformer_encoder_bwd(handle: int, out: Tensor, grad: Tensor, T: int, need_dx: bool,
                            nflat: int) -> Tuple[Tensor, Tensor]:
    """(d input (B, T, in_dim) -- zeros when not needed --, flat parameter gradients)."""
    mod = _mod(handle)
    st = _take(out)
    g = grad.contiguous().float().view(st["B"] * st["Tp"], -1)
    with GradCapture(list(mod.parameters())) as gc:
        dx = mod._bwd(st, g, need_dx=need_dx)
    if dx is None:
        dx = grad.new_zeros(st["B"], T, mod.in_dim)
    return dx.view(st["B"], T, -1).contiguous(), gc.buf


@transformer_encoder_bwd.register_fake
def _(handle, out, grad, T, need_dx, nflat):
    return grad.new_empty(grad.shape[0], T, _mod(handle).in_dim), grad.new_empty(nflat)


def _tf_setup(ctx, inputs, output):
    handle, x, lengths, seed, params = inputs
    ctx.handle, ctx.T = handle, x.shape[1]
    ctx.save_for_backward(output)
    _setup_params(ctx, params, handle)


def _tf_backward(ctx, g_out):
    (out,) = ctx.saved_tensors
    need = bool(ctx.needs_input_grad[1])
    dx, gflat = torch.ops.ensvs.transformer_encoder_bwd(ctx.handle, out, g_out, ctx.T, need,
                                                        ctx.nflat)
    return None, dx if need else None, None, None, _param_grads(ctx, gflat)


transformer_encoder.register_autograd(_tf_backward, setup_context=_tf_setup)


def transformer_call(mod, x, lengths):
    B, T, _ = x.shape
    return torch.ops.ensvs.transformer_encoder(handle_of(mod), x,
                                               _lengths_arg(lengths, B, T, x.device),
                                               _new_seed(), list(mod.parameters()))


# ======================================================== speaker embedding (row gather)
@torch.library.custom_op("ensvs::embedding_gather", mutates_args=())
def embedding_gather(table: Tensor, idx: Tensor) -> Tensor:
    """nnsvs/model.py:35-53: table[idx] (rows), idx any shape -> idx.shape + (E,)."""
    from ._lib import call
    from .layers import stream
    flat = idx.reshape(-1).to(torch.int64).contiguous()
    out = torch.empty(flat.numel(), table.shape[1], dtype=torch.float32, device=table.device)
    call("ensvs_gather_rows", table.data_ptr(), flat.data_ptr(), flat.numel(), table.shape[1],
         out.data_ptr(), stream())
    return out.view(*idx.shape, table.shape[1])


@embedding_gather.register_fake
def _(table, idx):
    return table.new_empty(*idx.shape, table.shape[1])


@torch.library.custom_op("ensvs::embedding_scatter", mutates_args=())
def embedding_scatter(grad: Tensor, idx: Tensor, num_rows: int) -> Tensor:
    """d table: rows of grad summed into their table rows (deterministic order)."""
    from ._lib import call
    from .layers import stream
    E = grad.shape[-1]
    flat = idx.reshape(-1).to(torch.int64).contiguous()
    dt = torch.zeros(num_rows, E, dtype=torch.float32, device=grad.device)
    g = grad.reshape(-1, E).contiguous().float()
    call("ensvs_spk_scatter", g.data_ptr(), flat.numel(), E, flat.data_ptr(), dt.data_ptr(),
         stream())
    return dt


@embedding_scatter.register_fake
def _(grad, idx, num_rows):
    return grad.new_empty(num_rows, grad.shape[-1])


def _emb_setup(ctx, inputs, output):
    table, idx = inputs
    ctx.save_for_backward(idx)
    ctx.rows = table.shape[0]


def _emb_backward(ctx, g):
    (idx,) = ctx.saved_tensors
    return torch.ops.ensvs.embedding_scatter(g, idx, ctx.rows), None


embedding_gather.register_autograd(_emb_backward, setup_context=_emb_setup)


OPS = ("diffnet", "diffnet_bwd", "ffconvlstm", "ffconvlstm_bwd", "diffusion_train",
       "diffusion_train_bwd", "lf0_train", "lf0_train_bwd", "multitrack_train",
       "multitrack_train_bwd", "separate_f0_train", "separate_f0_train_bwd", "masked_l1",
       "lstm_encoder", "lstm_encoder_bwd", "transformer_encoder", "transformer_encoder_bwd",
       "embedding_gather", "embedding_scatter")
