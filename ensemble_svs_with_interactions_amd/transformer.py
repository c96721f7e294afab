"""Transformer encoder on MI355X kernels.

Drop-in for nnsvs.model.TransformerEncoder (nnsvs/model.py:1540-1671) and the VITS-style
encoder it wraps (nnsvs/transformer/encoder.py:9-142, nnsvs/transformer/attentions.py:22-214):
same constructor arguments, ``forward`` signature and ``state_dict`` keys
(``encoder.attn_layers.{i}.conv_q.weight``, ``...emb_rel_k``, ``encoder.norm_layers_1.{i}.gamma``,
``encoder.ffn_layers.{i}.conv_1.weight`` ...).  The nn.Conv1d / nn.Linear members are parameter
containers; every op runs in libensvs.so:

  * 1x1 q / k / v / o projections, FFN convolutions ("same" zero padding), fc / fc_in /
    fc_out: the MFMA implicit-GEMM engine (ReLU and the residual add fused in epilogues);
  * relative-position attention (window_size, heads share the relative tables): per-head
    score / context products on a batched GEMM, the relative-key band, key mask and softmax
    in one wavefront per score row, relative values as a banded sum (attention.hip);
  * LayerNorm over channels (eps 1e-5) per frame row, the frame masks x * x_mask, dropout
    keep-masks from the counter-based RNG; backward of all of it under autograd
    (the ensvs::transformer_encoder op, torch_ops.py, returns the parameter gradients).
"""
import math

import torch
from torch import nn

from . import _lib
from . import engine
from . import kernels as K
from . import layers as Ly
from ._lib import call, ptr
from .base import BaseModel
from . import torch_ops
from .engine import ModulePacks, empty, grad_of, lengths_pair
from .model import init_weights


def stream():
    return torch.cuda.current_stream().cuda_stream


class LayerNorm(nn.Module):
    """nnsvs/transformer/encoder.py:9-21 (channel LayerNorm of (B, C, T), eps 1e-5)."""

    def __init__(self, channels, eps=1e-5):
        super().__init__()
        self.channels = channels
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))


class FFN(nn.Module):
    """nnsvs/transformer/encoder.py:24-79 (ReLU, "same" padding: the Encoder's use)."""

    def __init__(self, in_channels, out_channels, filter_channels, kernel_size, p_dropout=0.0,
                 activation=None, causal=False):
        super().__init__()
        if activation == "gelu" or causal:
            raise NotImplementedError("FFN(activation='gelu' / causal=True) is not used by the "
                                      "Transformer encoder (encoder.py:119-127)")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.filter_channels = filter_channels
        self.kernel_size = kernel_size
        self.p_dropout = p_dropout
        self.activation = activation
        self.causal = causal
        self.conv_1 = nn.Conv1d(in_channels, filter_channels, kernel_size)
        self.conv_2 = nn.Conv1d(filter_channels, out_channels, kernel_size)
        self.drop = nn.Dropout(p_dropout)


class MultiHeadAttention(nn.Module):
    """nnsvs/transformer/attentions.py:22-84 (self-attention with relative positions; the
    Encoder's configuration: window_size set, heads_share, no block_length / proximal)."""

    def __init__(self, channels, out_channels, n_heads, p_dropout=0.0, window_size=None,
                 heads_share=True, block_length=None, proximal_bias=False, proximal_init=False):
        super().__init__()
        assert channels % n_heads == 0
        if window_size is None or not heads_share or block_length is not None or proximal_bias:
            raise NotImplementedError("MultiHeadAttention: the encoder's relative-position "
                                      "self-attention (window_size, heads_share) only")
        self.channels = channels
        self.out_channels = out_channels
        self.n_heads = n_heads
        self.p_dropout = p_dropout
        self.window_size = window_size
        self.heads_share = heads_share
        self.block_length = block_length
        self.proximal_bias = proximal_bias
        self.proximal_init = proximal_init
        self.attn = None
        self.k_channels = channels // n_heads
        self.conv_q = nn.Conv1d(channels, channels, 1)
        self.conv_k = nn.Conv1d(channels, channels, 1)
        self.conv_v = nn.Conv1d(channels, channels, 1)
        self.conv_o = nn.Conv1d(channels, out_channels, 1)
        self.drop = nn.Dropout(p_dropout)
        rel_stddev = self.k_channels ** -0.5
        self.emb_rel_k = nn.Parameter(torch.randn(1, window_size * 2 + 1, self.k_channels)
                                      * rel_stddev)
        self.emb_rel_v = nn.Parameter(torch.randn(1, window_size * 2 + 1, self.k_channels)
                                      * rel_stddev)
        nn.init.xavier_uniform_(self.conv_q.weight)
        nn.init.xavier_uniform_(self.conv_k.weight)
        nn.init.xavier_uniform_(self.conv_v.weight)
        if proximal_init:
            with torch.no_grad():
                self.conv_k.weight.copy_(self.conv_q.weight)
                self.conv_k.bias.copy_(self.conv_q.bias)


class Encoder(nn.Module):
    """nnsvs/transformer/encoder.py:82-128 (container; run by TransformerEncoder)."""

    def __init__(self, hidden_channels, filter_channels, n_heads, n_layers, kernel_size=1,
                 p_dropout=0.0, window_size=4, **kwargs):
        super().__init__()
        self.hidden_channels = hidden_channels
        self.filter_channels = filter_channels
        self.n_heads = n_heads
        self.n_layers = n_layers
        self.kernel_size = kernel_size
        self.p_dropout = p_dropout
        self.window_size = window_size
        self.drop = nn.Dropout(p_dropout)
        self.attn_layers = nn.ModuleList()
        self.norm_layers_1 = nn.ModuleList()
        self.ffn_layers = nn.ModuleList()
        self.norm_layers_2 = nn.ModuleList()
        for _ in range(n_layers):
            self.attn_layers.append(MultiHeadAttention(hidden_channels, hidden_channels, n_heads,
                                                       p_dropout=p_dropout,
                                                       window_size=window_size))
            self.norm_layers_1.append(LayerNorm(hidden_channels))
            self.ffn_layers.append(FFN(hidden_channels, hidden_channels, filter_channels,
                                       kernel_size, p_dropout=p_dropout))
            self.norm_layers_2.append(LayerNorm(hidden_channels))


def _bg(t, off, sb, sh, sr, sc):
    """Batched-GEMM operand descriptor: (pointer, batch/head/row/col strides in floats)."""
    return (t.data_ptr() + 4 * off, sb, sh, sr, sc)


def _bgemm(a, b, c, Bn, H, M, N, Kd, alpha=1.0, accum=False):
    """Per-head products: bf16-operand MFMA in production precision, exact fp32 in parity
    mode (engine.set_gemm_precision)."""
    fn = "ensvs_bgemm_bf16" if engine.gemm_precision() == "bf16" else "ensvs_bgemm"
    call(fn, *a, *b, *c, Bn, H, M, N, Kd, float(alpha), int(accum), stream())


def _mask(x, ld, B, T, C, lens, out=None, out_ld=None):
    """out = x * x_mask over frame rows (in place when out is None)."""
    out = x if out is None else out
    call("ensvs_mask_rows", x.data_ptr(), ld, out.data_ptr(), ld if out_ld is None else out_ld,
         B, T, C, lens.data_ptr(), stream())
    return out


def _add(a, b, n, device):
    out = empty(n, device=device)
    call("ensvs_axpby_to", out.data_ptr(), a.data_ptr(), 1.0, b.data_ptr(), 1.0, n, stream())
    return out


class TransformerEncoder(BaseModel):
    """nnsvs/model.py:1540-1671: [phoneme embedding +] [reduction] -> fc -> relative-position
    Transformer encoder (masked) -> fc_out, output viewed (B, T'*r, out_dim)."""

    def __init__(self, in_dim, out_dim, hidden_dim, attention_dim, num_heads=2, num_layers=2,
                 kernel_size=3, dropout=0.1, reduction_factor=1, init_type="none",
                 downsample_by_conv=False, in_ph_start_idx: int = 1, in_ph_end_idx: int = 50,
                 embed_dim=None):
        super().__init__()
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.in_ph_start_idx = in_ph_start_idx
        self.in_ph_end_idx = in_ph_end_idx
        self.num_vocab = in_ph_end_idx - in_ph_start_idx
        self.embed_dim = embed_dim
        if self.embed_dim is not None:
            assert in_dim > self.num_vocab
            self.emb = nn.Embedding(self.num_vocab, embed_dim)
            self.fc_in = nn.Linear(in_dim - self.num_vocab, embed_dim)
            self.fc = nn.Linear(embed_dim, hidden_dim)
        else:
            self.emb = None
            self.fc_in = None
            self.fc = nn.Linear(in_dim, hidden_dim)
        self.reduction_factor = reduction_factor
        self.encoder = Encoder(hidden_channels=hidden_dim, filter_channels=attention_dim,
                               n_heads=num_heads, n_layers=num_layers, kernel_size=kernel_size,
                               p_dropout=dropout)
        self.fc_out = nn.Linear(hidden_dim, out_dim * reduction_factor)
        if reduction_factor > 1 and downsample_by_conv:
            if embed_dim is not None:
                # the reference runs Conv1d(in_dim, ...) on the embed_dim-wide embedding
                raise NotImplementedError("downsample_by_conv with embed_dim")
            self.conv_downsample = nn.Conv1d(in_dim, in_dim, kernel_size=reduction_factor,
                                             stride=reduction_factor, groups=in_dim)
        else:
            self.conv_downsample = None
        for f in [self.fc_in, self.emb, self.fc, self.fc_out]:
            if f is not None:
                init_weights(f, init_type)
        self._packs = ModulePacks()

    # ---- kernels -------------------------------------------------------------------
    def _register(self, pk):
        if self.embed_dim is not None:
            pk.linear("fc_in", self.fc_in.weight)
            pk.bias_vec("fc_in.b", self.fc_in.bias)
        pk.linear("fc", self.fc.weight)
        pk.bias_vec("fc.b", self.fc.bias)
        enc = self.encoder
        for i in range(enc.n_layers):
            att, ffn = enc.attn_layers[i], enc.ffn_layers[i]
            for n in ("q", "k", "v", "o"):
                conv = getattr(att, "conv_" + n)
                pk.conv(f"{i}.{n}", conv.weight)
                pk.bias_vec(f"{i}.{n}.b", conv.bias)
            for n in ("1", "2"):
                conv = getattr(ffn, "conv_" + n)
                pk.conv(f"{i}.c{n}", conv.weight)
                pk.bias_vec(f"{i}.c{n}.b", conv.bias)
        pk.linear("fc_out", self.fc_out.weight)
        pk.bias_vec("fc_out.b", self.fc_out.bias)

    def _pads(self):
        k = self.encoder.kernel_size
        return (k - 1) // 2, k // 2  # _same_padding (encoder.py:72-79)

    def _attn_fwd(self, i, x, B, T, lens, training):
        """attn_layers[i](x, x, attn_mask) up to the context O (before conv_o)."""
        enc = self.encoder
        att = enc.attn_layers[i]
        pk = self._packs
        dev = x.device
        M, C, H, dk, w = B * T, enc.hidden_channels, enc.n_heads, att.k_channels, att.window_size
        qkv = empty(M, 3 * C, device=dev)
        for j, n in enumerate(("q", "k", "v")):
            K.gemm([K.Seg(x, C, C, pk[f"{i}.{n}"], T)], B, T, C, pk.fwd, qkv, 3 * C,
                   yoff=j * C, **pk.bias_ptr_args(f"{i}.{n}.b"))
        qs = empty(M, C, device=dev)
        call("ensvs_div", qkv.data_ptr(), 3 * C, qs.data_ptr(), C, M, C, math.sqrt(dk), stream())
        TT = T * T
        S = empty(B * H * TT, device=dev)
        _bgemm(_bg(qs, 0, T * C, dk, C, 1), _bg(qkv, C, T * 3 * C, dk, 1, 3 * C),
               _bg(S, 0, H * TT, TT, T, 1), B, H, T, T, dk)
        keep = Pd = None
        if training and att.p_dropout > 0:
            keep = Ly.dropout_mask(B * H * TT, att.p_dropout, dev)
            Pd = empty(B * H * TT, device=dev)
        call("ensvs_attn_softmax", S.data_ptr(), qs.data_ptr(), C, att.emb_rel_k.data_ptr(),
             lens.data_ptr(), B, H, T, dk, w, ptr(keep), ptr(Pd), stream())
        P = S if Pd is None else Pd
        O = empty(M, C, device=dev)
        _bgemm(_bg(P, 0, H * TT, TT, T, 1), _bg(qkv, 2 * C, T * 3 * C, dk, 3 * C, 1),
               _bg(O, 0, T * C, dk, C, 1), B, H, T, dk, T)
        call("ensvs_attn_relv", P.data_ptr(), att.emb_rel_v.data_ptr(), O.data_ptr(), C, B, H,
             T, dk, w, stream())
        return dict(x=x, qkv=qkv, qs=qs, S=S, keep=keep, Pd=Pd, O=O)

    def _attn_bwd(self, i, a, dO, B, T, lens):
        """Backward of _attn_fwd: parameter grads (emb_rel_k / emb_rel_v) and dQKV."""
        enc = self.encoder
        att = enc.attn_layers[i]
        dev = dO.device
        M, C, H, dk, w = B * T, enc.hidden_channels, enc.n_heads, att.k_channels, att.window_size
        TT = T * T
        qkv, qs, S, keep = a["qkv"], a["qs"], a["S"], a["keep"]
        P = S if a["Pd"] is None else a["Pd"]
        dqkv = empty(M, 3 * C, device=dev)
        part = K.scratch(_lib.query("ensvs_attn_table_grad_workspace", dk, w), dev, key="attn")
        # dV = Pd^T dO ; d emb_rel_v
        _bgemm(_bg(P, 0, H * TT, TT, 1, T), _bg(dO, 0, T * C, dk, C, 1),
               _bg(dqkv, 2 * C, T * 3 * C, dk, 3 * C, 1), B, H, T, dk, T)
        call("ensvs_attn_table_grad", P.data_ptr(), dO.data_ptr(), C, B, H, T, dk, w,
             part.data_ptr(), grad_of(att.emb_rel_v).data_ptr(), 1, stream())
        # dPd = dO V^T + band(dO . ev) ; softmax backward -> dS
        dS = empty(B * H * TT, device=dev)
        _bgemm(_bg(dO, 0, T * C, dk, C, 1), _bg(qkv, 2 * C, T * 3 * C, dk, 1, 3 * C),
               _bg(dS, 0, H * TT, TT, T, 1), B, H, T, T, dk)
        call("ensvs_attn_band_dot", dS.data_ptr(), dO.data_ptr(), C, att.emb_rel_v.data_ptr(),
             B, H, T, dk, w, stream())
        call("ensvs_attn_softmax_bwd", dS.data_ptr(), S.data_ptr(), ptr(keep), lens.data_ptr(),
             B, H, T, stream())
        # d emb_rel_k ; dQS = dS K + band(dS) ek ; dQ = dQS / sqrt(dk) ; dK = dS^T QS
        call("ensvs_attn_table_grad", dS.data_ptr(), qs.data_ptr(), C, B, H, T, dk, w,
             part.data_ptr(), grad_of(att.emb_rel_k).data_ptr(), 1, stream())
        dqs = empty(M, C, device=dev)
        _bgemm(_bg(dS, 0, H * TT, TT, T, 1), _bg(qkv, C, T * 3 * C, dk, 3 * C, 1),
               _bg(dqs, 0, T * C, dk, C, 1), B, H, T, dk, T)
        call("ensvs_attn_band_rows", dS.data_ptr(), att.emb_rel_k.data_ptr(), dqs.data_ptr(), C,
             B, H, T, dk, w, stream())
        call("ensvs_div", dqs.data_ptr(), C, dqkv.data_ptr(), 3 * C, M, C, math.sqrt(dk),
             stream())
        _bgemm(_bg(dS, 0, H * TT, TT, 1, T), _bg(qs, 0, T * C, dk, C, 1),
               _bg(dqkv, C, T * 3 * C, dk, 3 * C, 1), B, H, T, dk, T)
        return dqkv

    def _fwd(self, x, B, T, lens_host, training=None):
        """x (B*T, in_dim) rows.  Returns (out (B*T', out_dim*r), saved state)."""
        training = self.training if training is None else training
        pk = self._packs.ensure(self, self._register)
        dev = x.device
        enc = self.encoder
        r = self.reduction_factor
        Din = self.in_dim
        st = dict(B=B, T=T)
        if r > 1:
            Tp = T // r
            lens_host = [int(v) // r for v in lens_host]
            xr = empty(B * Tp, Din, device=dev)
            if self.conv_downsample is not None:
                call("ensvs_dwdown_fwd", x.data_ptr(), Din, self.conv_downsample.weight.data_ptr(),
                     self.conv_downsample.bias.data_ptr(), xr.data_ptr(), Din, B, T, Din, r,
                     stream())
            else:
                call("ensvs_stride_rows", x.data_ptr(), Din, xr.data_ptr(), Din, B, T, Din, r,
                     r - 1, 0, stream())
            st["x_full"] = x
        else:
            Tp, xr = T, x
        _, lens = lengths_pair(lens_host, B, Tp, dev)
        M = B * Tp
        C = enc.hidden_channels
        if self.embed_dim is not None:
            hin, esv = Ly.embed_fwd(pk, self.emb.weight, [(xr, Din, 0, Din)],
                                    self.in_ph_start_idx, self.in_ph_end_idx, B, Tp, device=dev)
            Kin = self.embed_dim
            st["esv"] = esv
        else:
            hin, Kin = xr, Din
        h = empty(M, C, device=dev)
        K.gemm([K.Seg(hin, Kin, Kin, pk["fc"], Tp)], B, Tp, C, pk.fwd, h, C,
               **pk.bias_ptr_args("fc.b"))
        _mask(h, C, B, Tp, C, lens)  # x * x_mask (model.py:1666, encoder.py:132)
        st.update(Tp=Tp, lens=lens, xr=xr, hin=hin, Kin=Kin, layers=[])
        F = enc.filter_channels
        kz = enc.kernel_size
        pl, _ = self._pads()
        p = enc.p_dropout
        drop = training and p > 0
        for i in range(enc.n_layers):
            ln1, ln2 = enc.norm_layers_1[i], enc.norm_layers_2[i]
            a = self._attn_fwd(i, h, B, Tp, lens, training)
            y = empty(M, C, device=dev)
            K.gemm([K.Seg(a["O"], C, C, pk[f"{i}.o"], Tp)], B, Tp, C, pk.fwd, y, C,
                   **pk.bias_ptr_args(f"{i}.o.b"))
            k1 = Ly.dropout_mask(M * C, p, dev) if drop else None
            if k1 is not None:
                call("ensvs_mul", y.data_ptr(), k1.data_ptr(), M * C, stream())
            z1 = _add(h, y, M * C, dev).view(M, C)
            x1 = empty(M, C, device=dev)
            m1, r1 = empty(M, device=dev), empty(M, device=dev)
            call("ensvs_layer_norm_fwd", z1.data_ptr(), C, M, C, ln1.gamma.data_ptr(),
                 ln1.beta.data_ptr(), float(ln1.eps), x1.data_ptr(), C, m1.data_ptr(),
                 r1.data_ptr(), stream())
            # FFN (encoder.py:53-61): conv_1(pad(x*m)) -> relu -> drop -> conv_2(pad(.*m)) * m
            xm = _mask(x1, C, B, Tp, C, lens, out=empty(M, C, device=dev))
            h1 = empty(M, F, device=dev)
            K.gemm([K.Seg(xm, C, C, pk[f"{i}.c1"], Tp, taps=kz, shift0=-pl)], B, Tp, F, pk.fwd,
                   h1, F, relu=True, **pk.bias_ptr_args(f"{i}.c1.b"))
            kf = Ly.dropout_mask(M * F, p, dev) if drop else None
            hm = empty(M, F, device=dev)
            if kf is not None:
                call("ensvs_mul_out", hm.data_ptr(), h1.data_ptr(), kf.data_ptr(), M * F,
                     stream())
                _mask(hm, F, B, Tp, F, lens)
            else:
                _mask(h1, F, B, Tp, F, lens, out=hm)
            y2 = empty(M, C, device=dev)
            K.gemm([K.Seg(hm, F, F, pk[f"{i}.c2"], Tp, taps=kz, shift0=-pl)], B, Tp, C, pk.fwd,
                   y2, C, **pk.bias_ptr_args(f"{i}.c2.b"))
            _mask(y2, C, B, Tp, C, lens)
            k2 = Ly.dropout_mask(M * C, p, dev) if drop else None
            if k2 is not None:
                call("ensvs_mul", y2.data_ptr(), k2.data_ptr(), M * C, stream())
            z2 = _add(x1, y2, M * C, dev).view(M, C)
            x2 = empty(M, C, device=dev)
            m2, r2 = empty(M, device=dev), empty(M, device=dev)
            call("ensvs_layer_norm_fwd", z2.data_ptr(), C, M, C, ln2.gamma.data_ptr(),
                 ln2.beta.data_ptr(), float(ln2.eps), x2.data_ptr(), C, m2.data_ptr(),
                 r2.data_ptr(), stream())
            st["layers"].append(dict(a=a, k1=k1, z1=z1, m1=m1, r1=r1, xm=xm, h1=h1, kf=kf, hm=hm,
                                     k2=k2, z2=z2, m2=m2, r2=r2))
            h = x2
        xf = _mask(h, C, B, Tp, C, lens, out=empty(M, C, device=dev))  # encoder.py:141
        NO = self.fc_out.out_features
        out = empty(M, NO, device=dev)
        K.gemm([K.Seg(xf, C, C, pk["fc_out"], Tp)], B, Tp, NO, pk.fwd, out, NO,
               **pk.bias_ptr_args("fc_out.b"))
        st["xf"] = xf
        return out, st

    def _bwd(self, st, dout, need_dx=False):
        """dout (B*T', out_dim*r).  Accumulates parameter grads (grad_of); returns dx (B*T,
        in_dim) when need_dx."""
        pk = self._packs
        enc = self.encoder
        dev = dout.device
        B, Tp, lens = st["B"], st["Tp"], st["lens"]
        M, C, F = B * Tp, enc.hidden_channels, enc.filter_channels
        kz = enc.kernel_size
        pl, pr = self._pads()
        NO = self.fc_out.out_features
        Ly.wgrad_into(self.fc_out.weight, dout, NO, st["xf"], C, B, Tp, Tp, NO, C)
        Ly.colsum_into(dout, NO, M, NO, self.fc_out.bias)
        d = empty(M, C, device=dev)
        K.gemm([K.Seg(dout, NO, NO, pk["fc_out^T"], Tp)], B, Tp, C, pk.bwd, d, C)
        _mask(d, C, B, Tp, C, lens)
        for i in reversed(range(enc.n_layers)):
            L = st["layers"][i]
            att, ffn = enc.attn_layers[i], enc.ffn_layers[i]
            ln1, ln2 = enc.norm_layers_1[i], enc.norm_layers_2[i]
            # LayerNorm 2
            dz2, dyx = empty(M, C, device=dev), empty(M, C, device=dev)
            call("ensvs_layer_norm_bwd", d.data_ptr(), C, L["z2"].data_ptr(), C, M, C,
                 ln2.gamma.data_ptr(), L["m2"].data_ptr(), L["r2"].data_ptr(), dz2.data_ptr(), C,
                 dyx.data_ptr(), stream())
            Ly.colsum_into(dyx, C, M, C, ln2.gamma)
            Ly.colsum_into(d, C, M, C, ln2.beta)
            # FFN
            dy2 = empty(M, C, device=dev)
            if L["k2"] is not None:
                call("ensvs_mul_out", dy2.data_ptr(), dz2.data_ptr(), L["k2"].data_ptr(), M * C,
                     stream())
                _mask(dy2, C, B, Tp, C, lens)
            else:
                _mask(dz2, C, B, Tp, C, lens, out=dy2)
            Ly.wgrad_into(ffn.conv_2.weight, dy2, C, L["hm"], F, B, Tp, Tp, C, F, taps=kz,
                          shift0=-pl)
            Ly.colsum_into(dy2, C, M, C, ffn.conv_2.bias)
            dh = empty(M, F, device=dev)
            K.gemm([K.Seg(dy2, C, C, pk[f"{i}.c2^T"], Tp, taps=kz, shift0=-pr)], B, Tp, F,
                   pk.bwd, dh, F, epi=_lib.EPI_RELU_MASK, aux1=L["h1"], ld1=F)
            _mask(dh, F, B, Tp, F, lens)
            if L["kf"] is not None:
                call("ensvs_mul", dh.data_ptr(), L["kf"].data_ptr(), M * F, stream())
            Ly.wgrad_into(ffn.conv_1.weight, dh, F, L["xm"], C, B, Tp, Tp, F, C, taps=kz,
                          shift0=-pl)
            Ly.colsum_into(dh, F, M, F, ffn.conv_1.bias)
            dxm = empty(M, C, device=dev)
            K.gemm([K.Seg(dh, F, F, pk[f"{i}.c1^T"], Tp, taps=kz, shift0=-pr)], B, Tp, C,
                   pk.bwd, dxm, C)
            _mask(dxm, C, B, Tp, C, lens)
            dx1 = _add(dz2, dxm, M * C, dev).view(M, C)
            # LayerNorm 1
            dz1 = empty(M, C, device=dev)
            call("ensvs_layer_norm_bwd", dx1.data_ptr(), C, L["z1"].data_ptr(), C, M, C,
                 ln1.gamma.data_ptr(), L["m1"].data_ptr(), L["r1"].data_ptr(), dz1.data_ptr(), C,
                 dyx.data_ptr(), stream())
            Ly.colsum_into(dyx, C, M, C, ln1.gamma)
            Ly.colsum_into(dx1, C, M, C, ln1.beta)
            # conv_o
            a = L["a"]
            dy1 = dz1
            if L["k1"] is not None:
                dy1 = empty(M, C, device=dev)
                call("ensvs_mul_out", dy1.data_ptr(), dz1.data_ptr(), L["k1"].data_ptr(), M * C,
                     stream())
            Ly.wgrad_into(att.conv_o.weight, dy1, C, a["O"], C, B, Tp, Tp, C, C)
            Ly.colsum_into(dy1, C, M, C, att.conv_o.bias)
            dO = empty(M, C, device=dev)
            K.gemm([K.Seg(dy1, C, C, pk[f"{i}.o^T"], Tp)], B, Tp, C, pk.bwd, dO, C)
            dqkv = self._attn_bwd(i, a, dO, B, Tp, lens)
            segs = []
            for j, n in enumerate(("q", "k", "v")):
                conv = getattr(att, "conv_" + n)
                Ly.wgrad_into(conv.weight, dqkv, 3 * C, a["x"], C, B, Tp, Tp, C, C, dyoff=j * C)
                Ly.colsum_into(dqkv, 3 * C, M, C, conv.bias, yoff=j * C)
                segs.append(K.Seg(dqkv, 3 * C, C, pk[f"{i}.{n}^T"], Tp, xoff=j * C))
            dxa = empty(M, C, device=dev)
            K.gemm(segs, B, Tp, C, pk.bwd, dxa, C)
            d = _add(dz1, dxa, M * C, dev).view(M, C)
        _mask(d, C, B, Tp, C, lens)
        # fc (+ phoneme embedding / fc_in)
        Kin = st["Kin"]
        Ly.wgrad_into(self.fc.weight, d, C, st["hin"], Kin, B, Tp, Tp, C, Kin)
        Ly.colsum_into(d, C, M, C, self.fc.bias)
        if self.embed_dim is None and not need_dx:
            return None
        dh = empty(M, Kin, device=dev)
        K.gemm([K.Seg(d, C, C, pk["fc^T"], Tp)], B, Tp, Kin, pk.bwd, dh, Kin)
        Din = self.in_dim
        if self.embed_dim is not None:
            Ly.embed_bwd(self.emb, self.fc_in, st["esv"], dh, B, Tp)
            if not need_dx:
                return None
            # d x: fc_in^T d for the non-phoneme columns, 0 for the one-hot (argmax) columns
            nin = Din - self.num_vocab
            dn = empty(M, nin, device=dev)
            E = self.embed_dim
            K.gemm([K.Seg(dh, E, E, pk["fc_in^T"], Tp)], B, Tp, nin, pk.bwd, dn, nin)
            dxr = torch.zeros(M, Din, device=dev)
            p0, p1 = self.in_ph_start_idx, self.in_ph_end_idx
            call("ensvs_copy_cols", dn.data_ptr(), nin, dxr.data_ptr(), Din, M, p0, stream())
            call("ensvs_copy_cols", dn.data_ptr() + 4 * p0, nin, dxr.data_ptr() + 4 * p1, Din,
                 M, Din - p1, stream())
        else:
            dxr = dh
        r = self.reduction_factor
        if r == 1:
            return dxr
        T = st["T"]
        dx = empty(B * T, Din, device=dev)
        if self.conv_downsample is not None:
            prod = torch.zeros(M, Din * r, device=dev)
            call("ensvs_dwdown_bwd", dxr.data_ptr(), Din, st["x_full"].data_ptr(), Din,
                 self.conv_downsample.weight.data_ptr(), dx.data_ptr(), Din, prod.data_ptr(), B,
                 T, Din, r, stream())
            K.colsum(prod, Din * r, M, Din * r, grad_of(self.conv_downsample.weight).view(-1),
                     accum=True)
            Ly.colsum_into(dxr, Din, M, Din, self.conv_downsample.bias)
        else:
            call("ensvs_stride_rows", dxr.data_ptr(), Din, dx.data_ptr(), Din, B, T, Din, r,
                 r - 1, 1, stream())
        return dx

    # ---- reference API -------------------------------------------------------------
    def forward(self, x, lengths=None, y=None):
        return torch_ops.transformer_call(self, x, lengths)

