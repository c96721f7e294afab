"""Forward/backward building blocks shared by the encoders of the path.

Each block runs entirely in libensvs.so kernels (MFMA GEMMs, persistent
recurrences, memory-bound kernels); tensors here are only allocations and
views.  All activations are channels-last frame rows (B*T, C) fp32.

Blocks mirror the reference layer stacks:
  * phoneme embedding input   nnsvs/model.py:895-910, tacotron_f0.py:929-965
  * FF stack 3x(Linear+ReLU)  nnsvs/model.py:837-844, tacotron_f0.py:852-859
  * conv stack 3x(ReflectionPad1d(3)+Conv1d k7+BatchNorm1d+ReLU)
                              nnsvs/model.py:846-859, tacotron_f0.py:861-874
  * packed bi-LSTM            nnsvs/model.py:862-869,914-916
"""
import torch

from . import _lib
from . import kernels as K
from ._lib import call, ptr, query
from .engine import empty, gemm_dtype, grad_of, next_seed


# row splits of the BatchNorm backward reduction (>= 64 rows each): 256 fills the chip
BN_SPLITS = 256

def stream():
    return torch.cuda.current_stream().cuda_stream


DEBUG = None  # set to a dict to capture intermediates (tests / tools only)


def _dbg(name, t):
    if DEBUG is not None:
        DEBUG[name] = t.detach().clone()


def dropout_mask(n, p, device):
    """Scaled keep mask of F.dropout(p, training=True) from the counter-based RNG kernel."""
    m = empty(n, device=device)
    call("ensvs_dropout_mask", m.data_ptr(), n, float(p), next_seed(), stream())
    return m


def randn(n, device):
    z = empty(n, device=device)
    call("ensvs_randn", z.data_ptr(), n, next_seed(), stream())
    return z


def colsum_into(dy, ld, M, N, param, groups=1, scale=1.0, off=0, yoff=0, defer=False):
    """param.grad[off:off+N] += scale * column sums of dy.  defer: inside
    kernels.deferred_wgrad(), queue the sum for the branch's batched flush -- it then reads dy
    at the flush, so only callers that never write dy again in the same branch may ask for it
    (the transformer / timing backward passes reuse their buffers and sum at once)."""
    g = grad_of(param)
    if off == 0 and groups == 1:
        K.colsum(dy, ld, M, N, g, scale=scale, accum=True, yoff=yoff, defer=defer)
    else:
        tmp = empty(groups * N, device=dy.device)
        K.colsum(dy, ld, M // groups, N, tmp, groups=groups, scale=scale, yoff=yoff)
        call("ensvs_axpy", g.data_ptr() + 4 * off, tmp.data_ptr(), 1.0, N, stream())


def issue(later, fn):
    """Run fn (parameter-gradient work only) now, or append it to `later` for the caller to
    issue once the critical input gradient is out (see FFConvLSTM._bwd)."""
    if later is None:
        fn()
    else:
        later.append(fn)


def add_into_pair(src, N, p1, p2):
    """p1.grad[:N] += src[:N] and p2.grad[:N] += src[:N] (src: device pointer) in one launch
    (the b_ih / b_hh pairs of the recurrent layers share their gradient)."""
    g1, g2 = grad_of(p1), grad_of(p2)
    step = g2.data_ptr() - g1.data_ptr()
    if step % 4 == 0:
        call("ensvs_axpy_strided", g1.data_ptr(), step // 4, src, 0, 1.0, N, 2, stream())
    else:
        for g in (g1, g2):
            call("ensvs_axpy", g.data_ptr(), src, 1.0, N, stream())


def wgrad_into(param, dy, ldy, x, ldx, B, Tout, Tin, N, Kc, taps=1, dil=1, shift0=0,
               pad=_lib.PAD_ZERO, col0=0, scale=1.0, radd=None, radd_ld=0, dyoff=0, xoff=0,
               row0=0):
    """param.grad (+)= dy^T x for a Linear (N, K) or Conv1d (N, K, taps) weight, optionally
    into an input-column range starting at col0 / output rows from row0."""
    g = grad_of(param)
    if g.dim() == 2:
        sn, sk, sj = g.shape[1], 1, 1
    else:
        sn, sk, sj = g.shape[1] * g.shape[2], g.shape[2], 1
    K.wgrad(dy, ldy, x, ldx, B, Tout, Tin, N, Kc, taps, dil, shift0, pad, g, sn, sk, sj,
            accum=True, dtype=gemm_dtype(), radd=radd, radd_ld=radd_ld, dyoff=dyoff, xoff=xoff,
            scale=scale, dstoff=row0 * sn + col0 * sk, defer=True)


# ----------------------------------------------------------------- input

def phoneme_input_register(pk, emb_mod, fc_in):
    pk.linear("fc_in", fc_in.weight, bwd=False)
    pk.bias_vec("fc_in.b", fc_in.bias)


def gather_input(sources, ph0, ph1, M, device):
    """Split logical input columns into (phoneme one-hot source, contiguous non-phoneme
    copy).  sources: list of (tensor, ld, col_offset, ncols) covering columns in order."""
    Kin = sum(s[3] for s in sources) - (ph1 - ph0)
    ldx = (Kin + 3) // 4 * 4
    X = empty(M, ldx, device=device)  # columns >= Kin are masked by the GEMM loaders
    ph_src = None
    col = 0  # logical column of the current source start
    out = 0
    for (t, ld, off, n) in sources:
        lo, hi = col, col + n
        pieces = []
        if hi <= ph0 or lo >= ph1:
            pieces.append((lo, hi))
        else:
            if lo < ph0:
                pieces.append((lo, ph0))
            if hi > ph1:
                pieces.append((ph1, hi))
            assert lo <= ph0 and hi >= ph1, "phoneme columns must lie in one source"
            ph_src = (t, ld, off + (ph0 - lo))
        for a, b in pieces:
            call("ensvs_copy_cols", t.data_ptr() + 4 * (off + a - lo), ld,
                 X.data_ptr() + 4 * out, ldx, M, b - a, stream())
            out += b - a
        col = hi
    return ph_src, X, Kin, ldx


def fc_in_seg(pk, X, ldx, Kin, M, T):
    """GEMM operand of the phoneme-input Linear: with bf16 operands a zero-padded bf16 copy
    (K = in_dim - 47 is not a multiple of 8, which would leave the launch on the
    register-staged fp32 kernel: 38.6 us at 30 x 1024 frames)."""
    if Kin % 8 and K.bf16_operands(pk.fwd, M):
        ld8 = (Kin + 7) // 8 * 8
        xb = K.cast_bf16(X, ldx, Kin, M,
                         out=torch.empty(M, ld8, dtype=torch.bfloat16, device=X.device),
                         out_ld=ld8)
        return K.Seg(xb, ld8, Kin, pk["fc_in"], T)
    return K.Seg(X, ldx, Kin, pk["fc_in"], T)


def embed_fwd(pk, emb_weight, sources, ph0, ph1, B, T, spk_seq=None, spk_ld=0, device=None,
              out=None):
    """x = emb(argmax onehot) + fc_in(other cols) [+ spk]  -> (M, E); returns saved dict.
    out: (tensor, ld, col) to write into a column range of a wider buffer instead."""
    M = B * T
    ph_src, X, Kin, ldx = gather_input(sources, ph0, ph1, M, device)
    ids = torch.empty(M, dtype=torch.int32, device=device)
    t, ld, off = ph_src
    call("ensvs_phoneme_ids", t.data_ptr() + 4 * off, ld, M, 0, ph1 - ph0, ids.data_ptr(), stream())
    E = emb_weight.shape[1]
    if out is None:
        Y, ldY, col = empty(M, E, device=device), E, 0
    else:
        Y, ldY, col = out
    K.gemm([fc_in_seg(pk, X, ldx, Kin, M, T)], B, T, E, pk.fwd, Y, ldY, yoff=col,
           **pk.bias_ptr_args("fc_in.b"))
    call("ensvs_embed_add", Y.data_ptr() + 4 * col, ldY, M, E, T, emb_weight.data_ptr(),
         ids.data_ptr(), None, ptr(spk_seq), None, spk_ld, stream())
    return Y, dict(ids=ids, X=X, Kin=Kin, ldx=ldx)


def embed_bwd(emb_mod, fc_in, sv, dY, B, T, dspk_seq=None, ld=None, col=0):
    """Grads of emb / fc_in (and per-sequence speaker vectors, summed over frames).
    dY: (M, E), or columns [col, col + E) of a (M, ld) buffer."""
    M = B * T
    E = emb_mod.weight.shape[1]
    ld = E if ld is None else ld
    V = emb_mod.weight.shape[0]
    part = K.scratch(_lib.query("ensvs_embed_bwd_workspace", M, E, V), dY.device, key="emb")
    call("ensvs_embed_bwd", dY.data_ptr() + 4 * col, ld, M, E, sv["ids"].data_ptr(), V,
         part.data_ptr(), grad_of(emb_mod.weight).data_ptr(), stream())
    wgrad_into(fc_in.weight, dY, ld, sv["X"], sv["ldx"], B, T, T, E, sv["Kin"], dyoff=col)
    colsum_into(dY, ld, M, E, fc_in.bias, yoff=col, defer=True)
    if dspk_seq is not None:
        K.colsum(dY, ld, T, E, dspk_seq, groups=B, accum=True, yoff=col)


# ----------------------------------------------------------------- FF stack

def ff_register(pk, ff):
    for i in (0, 2, 4):
        pk.linear(f"ff{i}", ff[i].weight)
        pk.bias_vec(f"ff{i}.b", ff[i].bias)


# Producers write bf16 copies of their outputs for the bf16-operand GEMMs that consume them
# (FF / BatchNorm+ReLU / ReLU-mask passes, MFMA LSTM recurrences).  Off: the consumers round
# the fp32 tensors themselves -- the same bits (tests compare the two).
BF16_COPIES = {"on": True}
# the cooperative LSTMs' bf16 copies of y / dg and per-sequence bias partials
# (ensvs_lstm_coop_fwd_ex / _bwd_ex); off: fp32 outputs cast by their consumers (A/B switch)
COOP_BF16 = {"on": True}
# BatchNorm training statistics by ensvs_bn_stats (two launches: split sums / deviations, then
# the merge + rstd + running updates) or by two column sums + ensvs_bn_finalize (A/B switch)
BN_STATS = {"on": True}


def bf16_copy(pk, M, C, device):
    """A bf16 [M, C] buffer for a producer's rounded copy of its output when the packed
    weights take bf16 operands (the copy is the operand rounding the consuming GEMMs apply,
    so it only saves their cast / register staging), else None."""
    if not BF16_COPIES["on"] or C % 8 or not K.bf16_operands(pk.fwd, M):
        return None
    return torch.empty(M, C, dtype=torch.bfloat16, device=device)


def ff_fwd(pk, ff, X, B, T, device, x16=None):
    """The three Linear + ReLU layers.  Returns (outputs, their bf16 copies or None): each
    GEMM epilogue also writes its output rounded to bf16 -- the next layer's operand and the
    backward's weight-gradient operand.  x16: an optional bf16 copy of X (rows zero-padded to
    a multiple of 8 columns when the input width is not one) for the first GEMM."""
    M = B * T
    hs, hs16 = [], []
    h, ldh = (X, X.shape[1]) if x16 is None else (x16, x16.shape[1])
    for i in (0, 2, 4):
        N = ff[i].weight.shape[0]
        Kc = ff[i].weight.shape[1]
        out = empty(M, N, device=device)
        ob = bf16_copy(pk, M, N, device)
        K.gemm([K.Seg(h, ldh, Kc, pk[f"ff{i}"], T)], B, T, N, pk.fwd, out, N, relu=True,
               ybf=ob, ybf_ld=N, **pk.bias_ptr_args(f"ff{i}.b"))
        hs.append(out)
        hs16.append(ob)
        h, ldh = (out, N) if ob is None else (ob, N)
    return hs, hs16


def ff_bwd(pk, ff, X, hs, hs16, dH3, B, T, device, need_dx=True, x16=None, dx_ld=None,
           later=None):
    """dH3: grad of the last ReLU output.  Returns grad w.r.t. X.  The layer gradients d
    also come as bf16 copies (ReLU mask pass, ReLU-mask dgrad epilogue) for the weight
    gradients against the forward's bf16 copies and for the dgrad GEMMs.  x16: ff_fwd's bf16
    copy of X; dx_ld: row stride of the returned grad (default: the input width); later:
    a list that receives the weight / bias gradients as closures (issue())."""
    M = B * T
    ins, ins16 = [X, hs[0], hs[1]], [None if x16 is None else x16, hs16[0], hs16[1]]
    d = empty(M, dH3.shape[1], device=device)
    d16 = bf16_copy(pk, M, dH3.shape[1], device) if hs16[2] is not None else None
    call("ensvs_relu_mask", d.data_ptr(), ptr(d16), dH3.data_ptr(), hs[2].data_ptr(), d.numel(),
         stream())
    dx = None
    for li, i in enumerate((4, 2, 0)):
        lay = ff[i]
        N, Kc = lay.weight.shape
        xin, xin16 = ins[2 - li], ins16[2 - li]
        if d16 is not None and xin16 is not None:
            issue(later, lambda w=lay.weight, g=d16, x=xin16, N=N, Kc=Kc:
                  wgrad_into(w, g, N, x, x.shape[1], B, T, T, N, Kc))
        else:
            issue(later, lambda w=lay.weight, g=d, x=xin, N=N, Kc=Kc:
                  wgrad_into(w, g, N, x, x.shape[1], B, T, T, N, Kc))
        issue(later, lambda g=d, N=N, b=lay.bias: colsum_into(g, N, M, N, b, defer=True))
        if i == 0 and not need_dx:
            break
        nd = empty(M, Kc, device=device)
        dseg = K.Seg(d if d16 is None else d16, N, N, pk[f"ff{i}^T"], T)
        nd16 = None
        if i > 0:
            nd16 = bf16_copy(pk, M, Kc, device) if ins16[2 - li] is not None else None
            K.gemm([dseg], B, T, Kc, pk.bwd, nd, Kc, epi=_lib.EPI_RELU_MASK,
                   aux1=hs[2 - li - 1], ld1=Kc, ybf=nd16, ybf_ld=Kc)
        else:
            if dx_ld is not None and dx_ld != Kc:
                nd = empty(M, dx_ld, device=device)
            K.gemm([dseg], B, T, Kc, pk.bwd, nd, nd.shape[1])
            dx = nd
        d, d16 = nd, nd16
    return dx


# ----------------------------------------------------------------- conv stack

CONV_IDX = ((1, 2), (5, 6), (9, 10))


def conv_register(pk, conv, first_cols=None, first_bwd_cols=None):
    """first_cols: list of (name, (c0, c1)) input-column ranges of conv.1 (segments; ranges
    may overlap: a forward-only operand over several narrow segments' columns)."""
    for li, (ci, bi) in enumerate(CONV_IDX):
        w = conv[ci].weight
        if li == 0 and first_cols is not None:
            for name, cols in first_cols:
                pk.conv(f"conv{ci}@{name}", w, cols=cols,
                        bwd=first_bwd_cols is not None and name in first_bwd_cols)
        else:
            pk.conv(f"conv{ci}", w)
        pk.bias_vec(f"conv{ci}.b", conv[ci].bias)


def conv_fwd(pk, conv, first_segs, B, T, device, training, groups=1, save=True,
             update_running=True, running_updates=1, first_b16=None):
    """first_segs: list of (name, tensor, ld, K, xoff) for conv.1.  Returns (out, saved).
    running_updates: BatchNorm running-statistic updates with this batch's statistics (2
    stands for a second call of the stack on the same input whose outputs are unused).
    first_b16: optional list of (name, bf16 tensor, ld, K) operands of conv.1's forward GEMM
    in place of first_segs (caller-rounded copies, e.g. narrow columns gathered into one
    zero-padded segment); first_segs stay the fp32 inputs of the weight gradient, and a
    first_b16 operand with a first_segs segment's name and width is also its bf16 weight-
    gradient operand.  With bf16 operands every later layer's BatchNorm + ReLU pass writes
    its output's bf16 copy too (the next convolution's operand; the last layer's is
    returned in saved[-1]["out16"] for the caller's next GEMM)."""
    M = B * T
    Mg = M // groups
    sv = []
    key = lambda name: pk[f"conv1@{name}"] if name else pk["conv1"]  # noqa: E731
    segs = [K.Seg(t, ld, Kc, key(name), T, taps=7, dil=1, shift0=-3, pad=_lib.PAD_REFLECT,
                  xoff=xoff)
            for (name, t, ld, Kc, xoff) in first_segs]
    fsegs = segs if first_b16 is None else [
        K.Seg(t, ld, Kc, key(name), T, taps=7, dil=1, shift0=-3, pad=_lib.PAD_REFLECT)
        for (name, t, ld, Kc) in first_b16]
    twin = {name: (t, ld) for (name, t, ld, Kc) in (first_b16 or [])
            if any(n == name and k == Kc for (n, _, _, k, _) in first_segs)}
    segs16 = [twin.get(name) for (name, _, _, _, _) in first_segs]
    a = a16 = None
    for li, (ci, bi) in enumerate(CONV_IDX):
        C = conv[ci].weight.shape[0]
        if li > 0:
            segs = [K.Seg(a, C_prev, C_prev, pk[f"conv{ci}"], T, taps=7, dil=1,
                          shift0=-3, pad=_lib.PAD_REFLECT)]
            fsegs = segs if a16 is None else [
                K.Seg(a16, C_prev, C_prev, pk[f"conv{ci}"], T, taps=7, dil=1, shift0=-3,
                      pad=_lib.PAD_REFLECT)]
            segs16 = [None if a16 is None else (a16, C_prev)]
        y = empty(M, C, device=device)
        K.gemm(fsegs, B, T, C, pk.fwd, y, C, **pk.bias_ptr_args(f"conv{ci}.b"))
        bn = conv[bi]
        mean = empty(groups, C, device=device)
        rstd = empty(groups, C, device=device)
        # a BatchNorm module put in eval mode inside a training step (torch semantics:
        # bn.training decides batch vs running statistics) normalises with its running
        # statistics and is differentiated with them held constant (ensvs_bn_bwd_frozen)
        frozen = training and not bn.training
        if training and not frozen:
            var = empty(groups, C, device=device)
            upd = int(update_running and bn.track_running_stats)
            if BN_STATS["on"]:
                # statistics, rstd, running updates and num_batches_tracked in two launches
                n = query("ensvs_bn_stats_part_floats", M, C, Mg)
                part = K.scratch(n, device, key="bnstats")
                call("ensvs_bn_stats", y.data_ptr(), C, M, C, Mg, part.data_ptr(), n,
                     float(bn.eps), mean.data_ptr(), var.data_ptr(), rstd.data_ptr(),
                     bn.running_mean.data_ptr() if upd else None,
                     bn.running_var.data_ptr() if upd else None, float(bn.momentum),
                     max(1, running_updates) if upd else 0,
                     bn.num_batches_tracked.data_ptr() if upd else None, stream())
            else:
                K.colsum(y, C, Mg, C, mean, groups=groups, scale=1.0 / Mg)
                K.colsum(y, C, Mg, C, var, groups=groups, mean=mean, scale=1.0 / Mg)
                for _ in range(max(1, running_updates if upd else 1)):
                    call("ensvs_bn_finalize", mean.data_ptr(), var.data_ptr(), groups, C, Mg,
                         float(bn.eps), rstd.data_ptr(), bn.running_mean.data_ptr(),
                         bn.running_var.data_ptr(), float(bn.momentum), upd, stream())
                    if upd:
                        bn.num_batches_tracked.add_(groups)
            Mg_apply = Mg
        else:
            # eval: running statistics, one group
            mean = bn.running_mean
            call("ensvs_bn_finalize", mean.data_ptr(), bn.running_var.data_ptr(), 1, C, M,
                 float(bn.eps), rstd.data_ptr(), None, None, 0.0, 0, stream())
            Mg_apply = M
        out = empty(M, C, device=device)
        out16 = bf16_copy(pk, M, C, device) if save or li < len(CONV_IDX) - 1 else None
        call("ensvs_bn_apply_relu", y.data_ptr(), C, M, C, Mg_apply, mean.data_ptr(),
             rstd.data_ptr(), bn.weight.data_ptr(), bn.bias.data_ptr(), out.data_ptr(), C,
             ptr(out16), C, stream())
        if save:
            sv.append(dict(y=y, mean=mean, rstd=rstd, out=out, segs=segs, segs16=segs16,
                           frozen=frozen, out16=out16))
        a, a16, C_prev = out, out16, C
    return a, sv


def conv_bwd(pk, conv, sv, dout, B, T, device, groups=1, first_dx=None, later=None):
    """dout: grad of the stack output.  first_dx: list of (name, K) of conv.1 segments whose
    input gradient is wanted (returned in order as a list).  later: a list that receives the
    conv weight / bias gradients as closures (issue())."""
    M = B * T
    Mg = M // groups
    d = dout
    res = []
    for li in (2, 1, 0):
        ci, bi = CONV_IDX[li]
        s = sv[li]
        C = conv[ci].weight.shape[0]
        bn = conv[bi]
        dy = empty(M, C, device=device)
        dy16 = None if s.get("frozen") else bf16_copy(pk, M, C, device)
        part = K.scratch(groups * BN_SPLITS * 2 * C, device, key="bn")
        sums = empty(groups * 2 * C, device=device)
        if s.get("frozen"):
            call("ensvs_bn_bwd_frozen", d.data_ptr(), C, s["y"].data_ptr(), C, M, C,
                 s["mean"].data_ptr(), s["rstd"].data_ptr(), bn.weight.data_ptr(),
                 bn.bias.data_ptr(), part.data_ptr(), BN_SPLITS, sums.data_ptr(),
                 grad_of(bn.weight).data_ptr(), grad_of(bn.bias).data_ptr(), dy.data_ptr(), C,
                 stream())
        else:
            call("ensvs_bn_bwd", d.data_ptr(), C, s["y"].data_ptr(), C, M, C, Mg,
                 s["mean"].data_ptr(), s["rstd"].data_ptr(), bn.weight.data_ptr(),
                 bn.bias.data_ptr(), part.data_ptr(), BN_SPLITS, sums.data_ptr(),
                 grad_of(bn.weight).data_ptr(), grad_of(bn.bias).data_ptr(), dy.data_ptr(), C,
                 ptr(dy16), C, stream())
        _dbg(f"conv{li}.dout", d)
        _dbg(f"conv{li}.dy", dy)
        issue(later, lambda g=dy, C=C, b=conv[ci].bias: colsum_into(g, C, M, C, b, defer=True))
        w = conv[ci].weight
        col = 0
        for seg, seg16 in zip(s["segs"], s.get("segs16") or [None] * len(s["segs"])):
            if dy16 is not None and seg16 is not None:
                issue(later, lambda w=w, g=dy16, C=C, x=seg16, K_=seg.K, col=col:
                      wgrad_into(w, g, C, x[0], x[1], B, T, T, C, K_, taps=7, dil=1, shift0=-3,
                                 pad=_lib.PAD_REFLECT, col0=col))
            else:
                issue(later, lambda w=w, g=dy, C=C, sg=seg, col=col:
                      wgrad_into(w, g, C, sg.x, sg.ld, B, T, T, C, sg.K, taps=7, dil=1,
                                 shift0=-3, pad=_lib.PAD_REFLECT, col0=col, xoff=sg.xoff))
            col += seg.K
        dyo = dy if dy16 is None else dy16
        if li > 0:
            Cin = w.shape[1]
            dxp = empty(B * (T + 6), Cin, device=device)
            K.gemm([K.Seg(dyo, C, C, pk[f"conv{ci}^T"], T, taps=7, dil=1, shift0=-6)], B, T + 6,
                   Cin, pk.bwd, dxp, Cin)
            dprev = empty(M, Cin, device=device)
            call("ensvs_reflect_fold", dxp.data_ptr(), B, T, 3, Cin, dprev.data_ptr(), stream())
            d = dprev
        else:
            for (name, Kc) in (first_dx or []):
                ref = pk[f"conv{ci}@{name}^T"] if name else pk[f"conv{ci}^T"]
                dxp = empty(B * (T + 6), Kc, device=device)
                K.gemm([K.Seg(dyo, C, C, ref, T, taps=7, dil=1, shift0=-6)], B, T + 6, Kc,
                       pk.bwd, dxp, Kc)
                dx = empty(M, Kc, device=device)
                call("ensvs_reflect_fold", dxp.data_ptr(), B, T, 3, Kc, dx.data_ptr(), stream())
                res.append(dx)
    return res


# ----------------------------------------------------------------- bi-LSTM

def lstm_register(pk, lstm):
    """Per layer: both directions' W_ih stacked as one forward operand "ih{l}" (one input-
    projection GEMM of N = 8H reads the layer input once) when 4H is a multiple of the
    128-row packing (the summed bias pairs b_ih + b_hh are then consecutive, so "b{l}"
    addresses all 8H); otherwise one operand per direction.  Their transposes for the
    input-gradient GEMM."""
    H = lstm.hidden_size
    for l in range(lstm.num_layers):
        ws = [getattr(lstm, f"weight_ih_l{l}{sfx}") for sfx in ("", "_reverse")]
        if lstm_fused_proj(H):
            pk.refs[f"ih{l}"] = pk.fwd.add_rowcat(ws, 4 * H, ws[0].shape[1])
        for sfx, w in zip(("", "_reverse"), ws):
            pk.linear(f"ih{l}{sfx}", w, fwd=not lstm_fused_proj(H))
            pk.bias_vec(f"b{l}{sfx}", getattr(lstm, f"bias_ih_l{l}{sfx}"),
                        b2=getattr(lstm, f"bias_hh_l{l}{sfx}"))


def lstm_fused_proj(H):
    return (4 * H) % K.BM == 0


def lstm_coop(B, H):
    """Whether the layer's recurrence runs the cooperative kernels (lstm_coop.hip: H = 256 /
    512, any B in tiles of 32 sequences (8 tiles per launch), production bf16 precision; fp16 / bf16 recurrent products with fp32
    accumulation and cell state).  The fp32 parity mode keeps lstm.hip's exact kernels."""
    return gemm_dtype() == _lib.DT_BF16 and query("ensvs_lstm_coop_supported", B, H) == 1


def _coop_pack(lstm, l, bwd):
    """W_hh of layer l (both directions) as the cooperative kernels' MFMA fragments,
    repacked whenever the weights changed (engine epoch / parameter versions, as the GEMM
    ModulePacks: inside a captured step the repack is part of the graph)."""
    from .engine import _sig
    ws = [getattr(lstm, f"weight_hh_l{l}"), getattr(lstm, f"weight_hh_l{l}_reverse")]
    cache = lstm.__dict__.setdefault("_ensvs_coop", {})
    sig = _sig(ws)
    ent = cache.get((l, bwd))
    if ent is None or ent[0] != sig:
        H = lstm.hidden_size
        buf = ent[1] if ent is not None else torch.empty(
            2 * 4 * H * H, dtype=torch.bfloat16 if bwd else torch.float16, device=ws[0].device)
        call("ensvs_lstm_coop_pack", ws[0].data_ptr(), ws[1].data_ptr(), H, int(bwd),
             buf.data_ptr(), stream())
        ent = cache[(l, bwd)] = (sig, buf)
    return ent[1]


def lstm_mfma(H):
    """Whether a layer of hidden size H (after zero padding, lstm_pad) runs the MFMA
    recurrences (lstm_mfma.hip: H = 64 / 128 in production bf16 precision; fp16 / bf16
    recurrent products with fp32 accumulation, gates and cell state).  The fp32 parity mode
    keeps lstm.hip's exact kernels."""
    return gemm_dtype() == _lib.DT_BF16 and query("ensvs_lstm_mfma_supported", H) == 1


def _mfma_pack(lstm, l, bwd, HP=None):
    """W_hh of layer l (both directions; zero-padded to HP when given) as the MFMA
    recurrences' fragments, repacked whenever the weights changed (as _coop_pack)."""
    from .engine import _sig
    ws = [getattr(lstm, f"weight_hh_l{l}"), getattr(lstm, f"weight_hh_l{l}_reverse")]
    cache = lstm.__dict__.setdefault("_ensvs_mfma", {})
    sig = _sig(ws)
    ent = cache.get((l, bwd))
    if ent is None or ent[0] != sig:
        H = HP or lstm.hidden_size
        src = _whh_pad(lstm, l, HP) if HP else ws
        buf = ent[1] if ent is not None else torch.empty(
            2 * 4 * H * H, dtype=torch.bfloat16 if bwd else torch.float16, device=ws[0].device)
        call("ensvs_lstm_mfma_pack", src[0].data_ptr(), src[1].data_ptr(), H, int(bwd),
             buf.data_ptr(), stream())
        ent = cache[(l, bwd)] = (sig, buf)
    return ent[1]


_PERSIST_H = (8, 16, 32, 64, 128)


def lstm_pad(H):
    """Hidden size of the exact fp32 persistent kernel that runs a layer of size H on
    zero-padded gates (the SeparateF0 bap decoder's H = 62 -> 64: padded units have zero
    weights and inputs, so their c and h stay exactly 0), or None (H has its own kernel)."""
    if H in _PERSIST_H or H > _PERSIST_H[-1]:
        return None
    return next(p for p in _PERSIST_H if p >= H)


def _regroup(src, lds, dst, ldd, M, nblk, sw, dw):
    call("ensvs_regroup_cols", src.data_ptr(), lds, dst.data_ptr(), ldd, M, nblk, sw, dw, stream())


def _whh_pad(lstm, l, HP):
    """W_hh of layer l (both directions) zero-padded to [4 HP][HP], cached per weight
    version (engine epoch / parameter versions; captured into a step graph like the packs)."""
    from .engine import _sig
    ws = [getattr(lstm, f"weight_hh_l{l}"), getattr(lstm, f"weight_hh_l{l}_reverse")]
    cache = lstm.__dict__.setdefault("_ensvs_pad", {})
    sig = _sig(ws)
    ent = cache.get(l)
    if ent is None or ent[0] != sig:
        H = lstm.hidden_size
        dev = ws[0].device
        bufs = ent[1] if ent is not None else [empty(4 * HP, HP, device=dev) for _ in ws]
        tmp = empty(4 * H, HP, device=dev)
        for w, b in zip(ws, bufs):
            _regroup(w, H, tmp, HP, 4 * H, 1, H, HP)            # columns k: H -> HP
            _regroup(tmp, H * HP, b, HP * HP, 4, 1, H * HP, HP * HP)  # rows per gate: H -> HP
        ent = cache[l] = (sig, bufs)
    return ent[1]


def _coop_work(H, B, device):
    """Workspace of one cooperative launch (ceil(B/32) tile headers + slabs); the process's
    coop error word is registered first (engine.coop_error_word)."""
    from .engine import coop_error_word
    coop_error_word(device)
    n = query("ensvs_lstm_coop_work_bytes", H, B)
    return empty(n, device=device, dtype=torch.uint8), n


def lstm_fwd(pk, lstm, X, ldx, B, T, lens_dev, device, dropout_masks=None, save=True,
             x16=None):
    """Packed bidirectional multi-layer LSTM.  Returns (Y (M, 2H), saved list).  x16: an
    optional bf16 copy of X (row stride = the input width) from its producer."""
    M = B * T
    H = lstm.hidden_size
    sv = []
    h, ldh = X, ldx
    h16 = x16  # bf16 copy of h (the producer's, or the previous layer's recurrence output)
    for l in range(lstm.num_layers):
        Kc = getattr(lstm, f"weight_ih_l{l}").shape[1]
        HP = lstm_pad(H)
        # MFMA / cooperative recurrences on unpadded H: the layer input and output also kept
        # as bf16 for the bf16-operand GEMMs that read them (the next layer's input projection,
        # the backward's) -- the same roundings those GEMMs apply to fp32
        coop = lstm_coop(B, H)
        direct = BF16_COPIES["on"] and not HP and (
            (coop and COOP_BF16["on"]) or (not coop and lstm_mfma(H)))
        x16 = None
        if direct:
            if h16 is not None:
                x16 = h16
            elif Kc % 8 == 0 and K._castable(K.Seg(h, ldh, Kc, None, T)):
                x16 = K.cast_bf16(h, ldh, Kc, M)
        xa, lda = (x16, Kc) if x16 is not None else (h, ldh)
        gx = empty(M, 8 * H, device=device)
        if lstm_fused_proj(H):
            assert pk[f"b{l}_reverse"].offset == pk[f"b{l}"].offset + 4 * H
            K.gemm([K.Seg(xa, lda, Kc, pk[f"ih{l}"], T)], B, T, 8 * H, pk.fwd, gx, 8 * H,
                   **pk.bias_ptr_args(f"b{l}"))
        else:
            for d, sfx in enumerate(("", "_reverse")):
                K.gemm([K.Seg(xa, lda, Kc, pk[f"ih{l}{sfx}"], T)], B, T, 4 * H, pk.fwd, gx,
                       8 * H, yoff=d * 4 * H, **pk.bias_ptr_args(f"b{l}{sfx}"))
        y = empty(M, 2 * H, device=device)
        last = l == lstm.num_layers - 1
        drop = dropout_masks is not None and not last
        y16 = None
        if direct and (save or not (last or drop)):
            y16 = torch.empty(M, 2 * H, dtype=torch.bfloat16, device=device)
        saved = empty(M * 2 * 5 * (HP or H), device=device)
        if coop:
            work, nbytes = _coop_work(H, B, device)
            call("ensvs_lstm_coop_fwd_ex", gx.data_ptr(), 8 * H,
                 _coop_pack(lstm, l, False).data_ptr(), lens_dev.data_ptr(), B, T, H, y.data_ptr(),
                 2 * H, saved.data_ptr(), ptr(y16), 2 * H, work.data_ptr(), nbytes, stream())
        elif HP:
            gxp = empty(M, 8 * HP, device=device)
            _regroup(gx, 8 * H, gxp, 8 * HP, M, 8, H, HP)
            yp = empty(M, 2 * HP, device=device)
            if lstm_mfma(HP):
                call("ensvs_lstm_mfma_fwd", gxp.data_ptr(), 8 * HP,
                     _mfma_pack(lstm, l, False, HP).data_ptr(), lens_dev.data_ptr(), B, T, HP,
                     yp.data_ptr(), 2 * HP, saved.data_ptr(), None, 0, stream())
            else:
                w0, w1 = _whh_pad(lstm, l, HP)
                call("ensvs_lstm_fwd", gxp.data_ptr(), 8 * HP, w0.data_ptr(), w1.data_ptr(),
                     lens_dev.data_ptr(), B, T, HP, yp.data_ptr(), 2 * HP, saved.data_ptr(),
                     stream())
            _regroup(yp, 2 * HP, y, 2 * H, M, 2, HP, H)
            del gxp, yp
        elif lstm_mfma(H):
            call("ensvs_lstm_mfma_fwd", gx.data_ptr(), 8 * H, _mfma_pack(lstm, l, False).data_ptr(),
                 lens_dev.data_ptr(), B, T, H, y.data_ptr(), 2 * H, saved.data_ptr(),
                 ptr(y16), 2 * H, stream())
        else:
            call("ensvs_lstm_fwd", gx.data_ptr(), 8 * H,
                 getattr(lstm, f"weight_hh_l{l}").data_ptr(),
                 getattr(lstm, f"weight_hh_l{l}_reverse").data_ptr(), lens_dev.data_ptr(), B, T,
                 H, y.data_ptr(), 2 * H, saved.data_ptr(), stream())
        del gx
        yin = y
        mask = None
        if dropout_masks is not None and l < lstm.num_layers - 1:
            mask = dropout_masks[l]
            yin = empty(M, 2 * H, device=device)
            call("ensvs_mul_out", yin.data_ptr(), y.data_ptr(), mask.data_ptr(), yin.numel(),
                 stream())
        if save:
            sv.append(dict(x=h, ldx=ldh, y=y, saved=saved, mask=mask, yin=yin, hp=HP, x16=x16,
                           y16=y16))
        h, ldh = yin, 2 * H
        h16 = None if mask is not None else y16
    return h, sv


def lstm_bwd(pk, lstm, sv, dY, B, T, lens_dev, device, need_dx=True, later=None):
    """Packed bidirectional LSTM backward; returns the input gradient.  later: a list that
    receives each layer's weight / bias gradients as closures (issue())."""
    M = B * T
    H = lstm.hidden_size
    d = dY
    dx = None
    for l in reversed(range(lstm.num_layers)):
        s = sv[l]
        Kc = getattr(lstm, f"weight_ih_l{l}").shape[1]
        x16, y16 = s.get("x16"), s.get("y16")
        # bf16 dg for the GEMMs (fp32 dg only when the layer input has no bf16 copy) and the
        # bias gradient's per-sequence partial sums, all from the MFMA / cooperative recurrence
        dgb = bpart = None
        if y16 is not None:
            dgb = torch.empty(M, 8 * H, dtype=torch.bfloat16, device=device)
            bpart = empty(B, 8 * H, device=device)
        dg = empty(M, 8 * H, device=device) if dgb is None or x16 is None else None
        if lstm_coop(B, H):
            work, nbytes = _coop_work(H, B, device)
            call("ensvs_lstm_coop_bwd_ex", d.data_ptr(), 2 * H,
                 _coop_pack(lstm, l, True).data_ptr(), lens_dev.data_ptr(), B, T, H,
                 s["saved"].data_ptr(), ptr(dg), 8 * H, ptr(dgb), 8 * H, ptr(bpart),
                 work.data_ptr(), nbytes, stream())
        elif s.get("hp"):
            HP = s["hp"]
            dp = empty(M, 2 * HP, device=device)
            _regroup(d, 2 * H, dp, 2 * HP, M, 2, H, HP)
            dgp = empty(M, 8 * HP, device=device)
            if lstm_mfma(HP):
                call("ensvs_lstm_mfma_bwd", dp.data_ptr(), 2 * HP,
                     _mfma_pack(lstm, l, True, HP).data_ptr(), lens_dev.data_ptr(), B, T, HP,
                     s["saved"].data_ptr(), dgp.data_ptr(), 8 * HP, None, 0, None, stream())
            else:
                w0, w1 = _whh_pad(lstm, l, HP)
                nw = query("ensvs_lstm_bwd_work_floats", B, HP)
                work = empty(max(nw, 1), device=device)
                call("ensvs_lstm_bwd", dp.data_ptr(), 2 * HP, w0.data_ptr(), w1.data_ptr(),
                     lens_dev.data_ptr(), B, T, HP, s["saved"].data_ptr(), dgp.data_ptr(),
                     8 * HP, work.data_ptr(), nw, stream())
            _regroup(dgp, 8 * HP, dg, 8 * H, M, 8, HP, H)
            del dp, dgp
        elif lstm_mfma(H):
            call("ensvs_lstm_mfma_bwd", d.data_ptr(), 2 * H, _mfma_pack(lstm, l, True).data_ptr(),
                 lens_dev.data_ptr(), B, T, H, s["saved"].data_ptr(), ptr(dg), 8 * H, ptr(dgb),
                 8 * H, ptr(bpart), stream())
        else:
            nw = query("ensvs_lstm_bwd_work_floats", B, H)
            work = empty(max(nw, 1), device=device)
            call("ensvs_lstm_bwd", d.data_ptr(), 2 * H,
                 getattr(lstm, f"weight_hh_l{l}").data_ptr(),
                 getattr(lstm, f"weight_hh_l{l}_reverse").data_ptr(), lens_dev.data_ptr(), B, T,
                 H, s["saved"].data_ptr(), dg.data_ptr(), 8 * H, work.data_ptr(), nw, stream())
        gy, yy = (dgb, y16) if dgb is not None else (dg, s["y"])
        gi, xi, ldi = (dgb, x16, x16.shape[1]) if x16 is not None and dgb is not None else \
            (dg, s["x"], s["ldx"])

        def params(l=l, Kc=Kc, gy=gy, yy=yy, gi=gi, xi=xi, ldi=ldi, dg=dg, bpart=bpart):
            for di, sfx in enumerate(("", "_reverse")):
                wgrad_into(getattr(lstm, f"weight_ih_l{l}{sfx}"), gi, 8 * H, xi, ldi, B, T, T,
                           4 * H, Kc, dyoff=di * 4 * H)
                # h_{t-1} in processing order: t-1 forward, t+1 reverse (zero outside [0, L))
                wgrad_into(getattr(lstm, f"weight_hh_l{l}{sfx}"), gy, 8 * H, yy, 2 * H, B, T, T,
                           4 * H, H, shift0=(-1 if di == 0 else 1), dyoff=di * 4 * H,
                           xoff=di * H)
            # b_ih and b_hh of both directions share one gradient: the column sums of dg, once
            bsum = empty(8 * H, device=device)
            if bpart is not None:
                K.colsum(bpart, 8 * H, B, 8 * H, bsum)
            else:
                K.colsum(dg, 8 * H, M, 8 * H, bsum)
            for di, sfx in enumerate(("", "_reverse")):
                add_into_pair(bsum.data_ptr() + di * 16 * H, 4 * H,
                              getattr(lstm, f"bias_ih_l{l}{sfx}"),
                              getattr(lstm, f"bias_hh_l{l}{sfx}"))
        issue(later, params)
        if l == 0 and not need_dx:
            break
        nd = empty(M, Kc, device=device)
        gd = dgb if dgb is not None else dg
        K.gemm([K.Seg(gd, 8 * H, 4 * H, pk[f"ih{l}^T"], T),
                K.Seg(gd, 8 * H, 4 * H, pk[f"ih{l}_reverse^T"], T, xoff=4 * H)],
               B, T, Kc, pk.bwd, nd, Kc)
        if l > 0:
            prev_mask = sv[l - 1].get("mask")
            if prev_mask is not None:
                call("ensvs_mul", nd.data_ptr(), prev_mask.data_ptr(), nd.numel(), stream())
        d = nd
        dx = nd
    return dx
