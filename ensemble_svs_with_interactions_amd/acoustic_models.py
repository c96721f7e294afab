"""Multi-track acoustic models on MI355X kernels.

* ``ResF0NonAttentiveDecoder`` / ``MultiTrackBiLSTMResF0NonAttentiveDecoder``:
  the cross-singer log-F0 model (nnsvs/acoustic_models/tacotron_f0.py:19-243,
  757-991): main+sub feature fusion, FF + Conv/BN + bi-LSTM encoder and the
  free-running autoregressive residual-F0 decoder (persistent ardec kernels).
* ``MultiTrackNPSSMDNMultistreamParametricModel``: the pairwise ensemble
  diffusion model (nnsvs/acoustic_models/multistream.py:1482-1778).

Same constructor arguments, forward/inference signatures, prediction types
and state_dict keys as the reference; ``_target_`` strings are the only change
a recipe needs (configs.py).
"""

import torch
from torch import nn

from . import _lib
from . import torch_ops
from . import kernels as K
from . import layers as Ly
from ._lib import call, ptr, query
from .base import BaseModel, PredictionType
from .engine import Branches, ModulePacks, _sig, empty, gemm_dtype, grad_of, lengths_pair
from .model import init_weights

# SeparateF0: the decoders' [encoder out, rest flag, lf0] input in rows of a multiple of 8
# columns (zero pad) with a bf16 copy, so its GEMMs run on bf16 operands (A/B switch)
DEC_PAD = {"on": True}
# SeparateF0: the decoders' weight / bias gradients issued after their input gradients, on
# their streams beside the encoder's backward (which waits for those input gradients only)
DEC_LATER = {"on": True}
# SeparateF0: the V/UV and bap decoders start once the mgc decoder's FF + conv stack is issued
# (their stacks then run beside its recurrences instead of beside its stack; A/B switch)
DEC_ORDER = {"on": True}


# Step schedule of the fused branches (0 lf0, 1 mgc, 2 bap, 3 vuv; profiles/r2_schedule_ab.txt,
# tools/schedule_ab.py).  BRANCH_AFTER {branch: earlier-issued branch whose forward must finish
# first}: the bap and V/UV branches start when the mgc forward ends, so mgc -- the critical
# branch -- runs its forward beside the lf0 chain only (round 2, bap alone: 20.9 vs 21.2
# ms/step all at once; round 3, V/UV too: 15.63 vs 15.80 ms/step, all at once 16.14).
# Round 4: V/UV after the bap forward instead (14.06 / 14.06 vs 14.34 / 14.29 ms/step; after
# the lf0 forward: 18.1, bap after lf0: 19.1-19.8; profiles/r4_branch_order_ab.txt).
# EXCL_BRANCHES: branches whose recurrence workgroups reserve their CU's LDS (the lf0 and mgc
# chains; bap / vuv LSTM workgroups share CUs with GEMMs: 20.8 vs 21.0 ms/step).  Not kept:
# the V/UV backward after the mgc DiffNet backward (24.9 vs 22.2 ms/step: the V/UV
# recurrences then lengthen the tail instead of filling it).
BRANCH_AFTER = {2: 1, 3: 2}
EXCL_BRANCHES = {0, 1}
# PREPACK_ON: the branch whose stream issues the mgc denoiser's weight repack at its head
# (None: the mgc branch itself, when its denoiser runs)
PREPACK_ON = 0


def _ar_work(H, B, device):
    """Workspace of one cooperative AR-decoder launch (per 32-sequence tile: counters +
    exchange slabs); registers the process's coop error word first."""
    from .engine import coop_error_word
    coop_error_word(device)
    n = query("ensvs_ardec_coop_work_bytes", H, B)
    return empty(n, device=device, dtype=torch.uint8), n

class ZoneOutCell(nn.Module):
    """nnsvs/tacotron/decoder.py:20-48 (container).  The recipe uses zoneout 0, for which
    the cell output is exactly the LSTMCell output in train and eval modes."""

    def __init__(self, cell, zoneout=0.1):
        super().__init__()
        self.cell = cell
        self.hidden_size = cell.hidden_size
        self.zoneout = zoneout


class ResF0NonAttentiveDecoder(BaseModel):
    """tacotron_f0.py:19-243 (parameter container; run by the ardec kernels)."""

    def __init__(self, in_dim=512, out_dim=1, layers=2, hidden_dim=1024, prenet_layers=2,
                 prenet_hidden_dim=256, prenet_dropout=0.5, zoneout=0.1, reduction_factor=1,
                 downsample_by_conv=False, scaled_tanh=True, in_lf0_idx=300, in_lf0_min=5.3936276,
                 in_lf0_max=6.491111, out_lf0_idx=180, out_lf0_mean=5.953093881972361,
                 out_lf0_scale=0.23435173188961034, init_type="none", eval_dropout=True):
        super().__init__()
        if prenet_layers != 0 or layers != 1 or out_dim != 1 or zoneout != 0.0 \
                or reduction_factor != 4 or not downsample_by_conv or not scaled_tanh:
            raise NotImplementedError(
                "the MI355X AR decoder implements the multi-track recipe configuration "
                "(prenet_layers 0, 1 LSTM layer, out_dim 1, zoneout 0, r 4, conv downsample, "
                "scaled tanh)")
        self.out_dim = out_dim
        self.reduction_factor = reduction_factor
        self.prenet_dropout = prenet_dropout
        self.scaled_tanh = scaled_tanh
        self.in_lf0_idx = in_lf0_idx
        self.in_lf0_min = in_lf0_min
        self.in_lf0_max = in_lf0_max
        self.out_lf0_idx = out_lf0_idx
        self.out_lf0_mean = out_lf0_mean
        self.out_lf0_scale = out_lf0_scale
        self.prenet = None
        lstm_in_dim = in_dim + out_dim
        self.lstm = nn.ModuleList([ZoneOutCell(nn.LSTMCell(lstm_in_dim, hidden_dim), zoneout)])
        self.feat_out = nn.Linear(in_dim + hidden_dim, out_dim * reduction_factor, bias=False)
        self.conv_downsample = nn.Conv1d(in_dim, in_dim, kernel_size=reduction_factor,
                                         stride=reduction_factor, groups=in_dim)
        init_weights(self, init_type)

    def is_autoregressive(self):
        return True

    def has_residual_lf0_prediction(self):
        return True


class BiLSTMResF0NonAttentiveDecoder(BaseModel):
    """tacotron_f0.py:528-756: FF + Conv/BN + bi-LSTM encoder and the residual-F0
    autoregressive decoder, single track (BASELINE config 2's log-F0 model).

    The decoder is teacher-forced when targets are given (the single-track model in
    training, multistream.py:1158; tacotron_f0.py:156-159, 226-228) and free-running
    otherwise; both run in the persistent ardec kernels.  The multi-track subclass adds
    the second track (additive main + sub fusion)."""

    _NTRACKS = 1

    def __init__(self, in_dim=512, ff_hidden_dim=2048, conv_hidden_dim=1024, lstm_hidden_dim=256,
                 num_lstm_layers=2, dropout=0.0, out_dim=80, decoder_layers=2,
                 decoder_hidden_dim=1024, prenet_layers=2, prenet_hidden_dim=256,
                 prenet_dropout=0.5, zoneout=0.1, reduction_factor=1, downsample_by_conv=False,
                 scaled_tanh=True, in_lf0_idx=300, in_lf0_min=5.3936276, in_lf0_max=6.491111,
                 out_lf0_idx=180, out_lf0_mean=5.953093881972361,
                 out_lf0_scale=0.23435173188961034, use_mdn=False, num_gaussians=4,
                 sampling_mode="mean", in_ph_start_idx: int = 1, in_ph_end_idx: int = 50,
                 embed_dim=None, init_type="none"):
        super().__init__()
        self._build(in_dim, ff_hidden_dim, conv_hidden_dim, lstm_hidden_dim, num_lstm_layers,
                    dropout, out_dim, decoder_layers, decoder_hidden_dim, prenet_layers,
                    prenet_hidden_dim, prenet_dropout, zoneout, reduction_factor,
                    downsample_by_conv, scaled_tanh, in_lf0_idx, in_lf0_min, in_lf0_max,
                    out_lf0_idx, out_lf0_mean, out_lf0_scale, use_mdn, in_ph_start_idx,
                    in_ph_end_idx, embed_dim, init_type)

    def _build(self, in_dim, ff_hidden_dim, conv_hidden_dim, lstm_hidden_dim, num_lstm_layers,
               dropout, out_dim, decoder_layers, decoder_hidden_dim, prenet_layers,
               prenet_hidden_dim, prenet_dropout, zoneout, reduction_factor, downsample_by_conv,
               scaled_tanh, in_lf0_idx, in_lf0_min, in_lf0_max, out_lf0_idx, out_lf0_mean,
               out_lf0_scale, use_mdn, in_ph_start_idx, in_ph_end_idx, embed_dim, init_type):
        if use_mdn or embed_dim is None:
            raise NotImplementedError("use_mdn / no phoneme embedding are not on the path")
        nt = self._NTRACKS
        self.reduction_factor = reduction_factor
        self.in_lf0_idx = in_lf0_idx
        self.in_lf0_min = in_lf0_min
        self.in_lf0_max = in_lf0_max
        self.out_lf0_idx = out_lf0_idx
        self.out_lf0_mean = out_lf0_mean
        self.out_lf0_scale = out_lf0_scale
        self.use_mdn = use_mdn
        self.in_dim = in_dim
        self.in_ph_start_idx = in_ph_start_idx
        self.in_ph_end_idx = in_ph_end_idx
        self.num_vocab = in_ph_end_idx - in_ph_start_idx
        self.embed_dim = embed_dim
        self.emb = nn.Embedding(self.num_vocab, embed_dim)
        self.fc_in = nn.Linear(in_dim - self.num_vocab, embed_dim)
        self.ff = nn.Sequential(
            nn.Linear(embed_dim, ff_hidden_dim), nn.ReLU(),
            nn.Linear(ff_hidden_dim, ff_hidden_dim), nn.ReLU(),
            nn.Linear(ff_hidden_dim, ff_hidden_dim), nn.ReLU())
        # the score log-F0 column of every track joins the conv input (ff + 1 or ff + 2)
        self.conv = nn.Sequential(
            nn.ReflectionPad1d(3), nn.Conv1d(ff_hidden_dim + nt, conv_hidden_dim, 7, padding=0),
            nn.BatchNorm1d(conv_hidden_dim), nn.ReLU(),
            nn.ReflectionPad1d(3), nn.Conv1d(conv_hidden_dim, conv_hidden_dim, 7, padding=0),
            nn.BatchNorm1d(conv_hidden_dim), nn.ReLU(),
            nn.ReflectionPad1d(3), nn.Conv1d(conv_hidden_dim, conv_hidden_dim, 7, padding=0),
            nn.BatchNorm1d(conv_hidden_dim), nn.ReLU())
        self.lstm = nn.LSTM(conv_hidden_dim, lstm_hidden_dim, num_lstm_layers, bidirectional=True,
                            batch_first=True, dropout=dropout)
        # decoder input = [bi-LSTM out, score lf0 of every track]; the residual is added to
        # the main track's score (in_lf0_idx -1 / -2: tacotron_f0.py:674, 896)
        decoder_in_dim = 2 * lstm_hidden_dim + nt
        self.decoder = ResF0NonAttentiveDecoder(
            in_dim=decoder_in_dim, out_dim=out_dim, layers=decoder_layers,
            hidden_dim=decoder_hidden_dim, prenet_layers=prenet_layers,
            prenet_hidden_dim=prenet_hidden_dim, prenet_dropout=prenet_dropout, zoneout=zoneout,
            reduction_factor=reduction_factor, downsample_by_conv=downsample_by_conv,
            scaled_tanh=scaled_tanh, in_lf0_idx=-nt, in_lf0_min=in_lf0_min,
            in_lf0_max=in_lf0_max, out_lf0_idx=out_lf0_idx, out_lf0_mean=out_lf0_mean,
            out_lf0_scale=out_lf0_scale)
        init_weights(self, init_type)
        self._packs = ModulePacks()
        self._ar = None

    def is_autoregressive(self):
        return True

    def prediction_type(self):
        return PredictionType.DETERMINISTIC

    def has_residual_lf0_prediction(self):
        return True

    def _set_lf0_params(self):
        self.decoder.in_lf0_min = self.in_lf0_min
        self.decoder.in_lf0_max = self.in_lf0_max
        self.decoder.out_lf0_mean = self.out_lf0_mean
        self.decoder.out_lf0_scale = self.out_lf0_scale

    # ------------------------------------------------------------------ packs
    def _register(self, pk):
        Ly.phoneme_input_register(pk, self.emb, self.fc_in)
        Ly.ff_register(pk, self.ff)
        F = self.ff[4].weight.shape[0]
        cols = [("ff", (0, F)), ("s0", (F, F + 1))]
        if self._NTRACKS == 2:
            cols.append(("s1", (F + 1, F + 2)))
        # the score log-F0 column(s) as one forward operand (_conv_in)
        cols.append(("lf0", (F, F + self._NTRACKS)))
        Ly.conv_register(pk, self.conv, first_cols=cols, first_bwd_cols=["ff"])
        Ly.lstm_register(pk, self.lstm)
        cell = self.decoder.lstm[0].cell
        Ce = self.decoder.conv_downsample.weight.shape[0]
        H = cell.hidden_size
        pk.linear("dec_ih_e", cell.weight_ih, cols=(0, Ce))
        pk.bias_vec("dec_b", cell.bias_ih, b2=cell.bias_hh)
        pk.linear("dec_fo_e", self.decoder.feat_out.weight, cols=(H, H + Ce))

    def _ar_prepare(self):
        """Packed W_hh layouts and the contiguous prenet column of W_ih for the ardec kernels:
        (wpf, wpb, wih_p), plus the cooperative kernels' fp16 / bf16 MFMA fragments (coop_f,
        coop_b) when the decoder runs them (_ar_coop)."""
        cell = self.decoder.lstm[0].cell
        params = [cell.weight_hh, cell.weight_ih]
        sig = _sig(params)
        if self._ar is not None and self._ar[0] == sig:
            return self._ar[1]
        H = cell.hidden_size
        dev = cell.weight_hh.device
        wpf = empty(4 * H * H, device=dev)
        wpb = empty(4 * H * H, device=dev)
        call("ensvs_ardec_pack", cell.weight_hh.data_ptr(), H, wpf.data_ptr(), wpb.data_ptr(),
             Ly.stream())
        Ce1 = cell.weight_ih.shape[1]
        wih_p = empty(4 * H, device=dev)
        call("ensvs_copy_cols", cell.weight_ih.data_ptr() + 4 * (Ce1 - 1), Ce1, wih_p.data_ptr(), 1,
             4 * H, 1, Ly.stream())
        coop = None
        if query("ensvs_ardec_coop_supported", 1, H) == 1:
            coop = (torch.empty(4 * H * H, dtype=torch.float16, device=dev),
                    torch.empty(4 * H * H, dtype=torch.bfloat16, device=dev))
            for bwd, buf in enumerate(coop):
                call("ensvs_ardec_coop_pack", cell.weight_hh.data_ptr(), H, bwd, buf.data_ptr(),
                     Ly.stream())
        self._ar = (sig, (wpf, wpb, wih_p, coop))
        return self._ar[1]

    def _ar_coop(self, B):
        """Whether the AR decoder runs the cooperative kernels (ardec.hip: H = 128 / 256,
        any B in tiles of 32 sequences (8 tiles per launch), production bf16 precision; fp16 / bf16 recurrent products with fp32
        accumulation, gates, cell state and feat_out).  The fp32 parity mode keeps the exact
        per-sequence kernels."""
        H = self.decoder.lstm[0].cell.hidden_size
        return Ly.gemm_dtype() == _lib.DT_BF16 and query("ensvs_ardec_coop_supported", B, H) == 1

    # ------------------------------------------------------------------ kernels
    def _embed(self, pk, xs, ld, B, T, spks, spk_ld, dev):
        """x = sum over tracks of (emb + fc_in + spk)   (tacotron_f0.py:710-726, 929-965)."""
        M = B * T
        ph0, ph1 = self.in_ph_start_idx, self.in_ph_end_idx
        E = self.embed_dim
        Y = empty(M, E, device=dev)
        saved = []
        ids = []
        for k, x in enumerate(xs):
            ph_src, X, Kin, ldx = Ly.gather_input([(x, ld, 0, ld)], ph0, ph1, M, dev)
            idv = torch.empty(M, dtype=torch.int32, device=dev)
            t, lds, off = ph_src
            call("ensvs_phoneme_ids", t.data_ptr() + 4 * off, lds, M, 0, ph1 - ph0, idv.data_ptr(),
                 Ly.stream())
            K.gemm([Ly.fc_in_seg(pk, X, ldx, Kin, M, T)], B, T, E, pk.fwd, Y, E, accum=k > 0,
                   **pk.bias_ptr_args("fc_in.b"))
            saved.append(dict(ids=idv, X=X, Kin=Kin, ldx=ldx))
            ids.append(idv)
        two = len(xs) == 2
        call("ensvs_embed_add", Y.data_ptr(), E, M, E, T, self.emb.weight.data_ptr(),
             ids[0].data_ptr(), ids[1].data_ptr() if two else None, ptr(spks[0]),
             ptr(spks[1]) if two else None, spk_ld, Ly.stream())
        return Y, saved

    def _conv_in(self, pk, h, xs, ld, B, T, dev, hb=None):
        """conv.1's input columns [FF output, score log-F0 of each track]: the fp32 segments
        (weight gradients) and, with bf16 operands, the forward's bf16 copies -- the FF
        output (hb: the FF GEMM's own copy), and the 1-2 log-F0 columns gathered into one
        zero-padded 8-wide operand, so
        the k7 conv runs on the LDS-DMA kernel (K = 256 + 1 + 1 fails its K % 8 contract
        as three segments: 182 us on the register-staged fp32 path at 30 x 1024 frames)."""
        F, li, M = h.shape[1], self.in_lf0_idx, B * T
        segs = [("ff", h, F, F, 0)] + [(f"s{k}", x, ld, 1, li) for k, x in enumerate(xs)]
        if not K.bf16_operands(pk.fwd, M) or F % 8:
            return segs, None
        if hb is None:
            hb = K.cast_bf16(h, F, F, M)
        cols = empty(M, len(xs), device=dev)
        for k, x in enumerate(xs):
            call("ensvs_copy_cols", x.data_ptr() + 4 * li, ld, cols.data_ptr() + 4 * k,
                 len(xs), M, 1, Ly.stream())
        lb = K.cast_bf16(cols, len(xs), len(xs), M,
                         out=torch.empty(M, 8, dtype=torch.bfloat16, device=dev), out_ld=8)
        return segs, [("ff", hb, F, F), ("lf0", lb, 8, len(xs))]

    def _fwd(self, xs, ld, B, T, lens_dev, spks=(None, None), spk_ld=0, masks=None,
             training=None, save=True, teacher=None):
        """xs: [x_main] or [x_main, x_sub] (B*T rows of ld floats); spks: per-sequence speaker
        vectors (or None); teacher: (targets, ld, col) of the normalised log-F0 target for
        teacher forcing, None = free-running.  Returns (lf0 (B*T,), res (B*T,), state)."""
        self._set_lf0_params()
        training = self.training if training is None else training
        pk = self._packs.ensure(self, self._register)
        dev = self.fc_in.weight.device
        M = B * T
        li = self.in_lf0_idx
        X0, esv = self._embed(pk, xs, ld, B, T, spks, spk_ld, dev)
        hs, hs16 = Ly.ff_fwd(pk, self.ff, X0, B, T, dev)
        segs, b16 = self._conv_in(pk, hs[2], xs, ld, B, T, dev, hs16[2])
        a, csv = Ly.conv_fwd(pk, self.conv, segs, B, T, dev, training, save=save,
                             first_b16=b16)
        C = a.shape[1]
        y, lsv = Ly.lstm_fwd(pk, self.lstm, a, C, B, T, lens_dev, dev, None, save=save,
                             x16=csv[-1]["out16"] if csv else None)
        dec = self.decoder
        cell = dec.lstm[0].cell
        H = cell.hidden_size
        Hl2 = y.shape[1]
        Ce = Hl2 + len(xs)
        Tr = T // 4
        e = empty(B * Tr, Ce, device=dev)
        x1 = xs[1].data_ptr() + 4 * li if len(xs) == 2 else None
        call("ensvs_downsample_fwd", y.data_ptr(), Hl2, Hl2, xs[0].data_ptr() + 4 * li, ld, 1,
             x1, ld, 1, dec.conv_downsample.weight.data_ptr(),
             dec.conv_downsample.bias.data_ptr(), B, T, e.data_ptr(), Ce, Ly.stream())
        gx = empty(B * Tr, 4 * H, device=dev)
        K.gemm([K.Seg(e, Ce, Ce, pk["dec_ih_e"], Tr)], B, Tr, 4 * H, pk.fwd, gx, 4 * H,
               **pk.bias_ptr_args("dec_b"))
        ofx = empty(B * Tr, 4, device=dev)
        K.gemm([K.Seg(e, Ce, Ce, pk["dec_fo_e"], Tr)], B, Tr, 4, pk.fwd, ofx, 4)
        wpf, wpb, wih_p, coop = self._ar_prepare()
        if masks is None:
            masks = Ly.dropout_mask(B * Tr, dec.prenet_dropout, dev)
        lf0 = empty(M, device=dev)
        res = empty(M, device=dev)
        sg = empty(B * Tr, 4 * H, device=dev)
        sc = empty(B * Tr, H, device=dev)
        sh = empty(B * Tr, H, device=dev)
        so = empty(B * Tr, 4, device=dev)
        sp = empty(B * Tr, device=dev)
        tptr, tld = (None, 0) if teacher is None else \
            (teacher[0].data_ptr() + 4 * teacher[2], teacher[1])
        consts = (float(dec.in_lf0_min), float(dec.in_lf0_max), float(dec.out_lf0_mean),
                  float(dec.out_lf0_scale))
        outs = (lf0.data_ptr(), res.data_ptr(), sg.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                so.data_ptr(), sp.data_ptr())
        ins = (wih_p.data_ptr(), dec.feat_out.weight.data_ptr(), dec.feat_out.weight.shape[1],
               xs[0].data_ptr() + 4 * li, ld, masks.data_ptr(), tptr, tld, B, T, H)
        if coop is not None and self._ar_coop(B):
            work, nbytes = _ar_work(H, B, dev)
            call("ensvs_ardec_coop_fwd", gx.data_ptr(), 4 * H, ofx.data_ptr(), 4,
                 coop[0].data_ptr(), *ins, *consts, *outs, work.data_ptr(), nbytes, Ly.stream())
        else:
            call("ensvs_ardec_fwd", gx.data_ptr(), 4 * H, ofx.data_ptr(), 4, wpf.data_ptr(),
                 *ins, *consts, *outs, Ly.stream())
        st = None
        if save:
            st = dict(X0=X0, esv=esv, hs=hs, hs16=hs16, csv=csv, lsv=lsv, y=y, e=e, masks=masks, sg=sg,
                      sc=sc, sh=sh, so=so, sp=sp, B=B, T=T, lens=lens_dev, xs=xs, ld=ld,
                      teacher=teacher is not None)
        return lf0, res, st

    def _bwd(self, st, dlf0, dres=None, want_spk=True):
        """dlf0 / dres: (B*T,) grads of the lf0 / residual outputs.  Returns (per-sequence
        speaker-vector grads of the main and sub track (B, E) -- the same tensor: the
        fused input holds both -- or None, the input grad dX0 (B*T, E))."""
        pk = self._packs
        dev = dlf0.device
        B, T = st["B"], st["T"]
        M, Tr = B * T, T // 4
        dec = self.decoder
        cell = dec.lstm[0].cell
        H = cell.hidden_size
        Ce = st["e"].shape[1]
        xs = st["xs"]
        wpf, wpb, wih_p, coop = self._ar_prepare()
        dg = empty(B * Tr, 4 * H, device=dev)
        do4 = empty(B * Tr, 4, device=dev)
        args = (wih_p.data_ptr(), dec.feat_out.weight.data_ptr(), dec.feat_out.weight.shape[1],
                st["masks"].data_ptr(), int(st["teacher"]), B, T, H, float(dec.in_lf0_min),
                float(dec.in_lf0_max), float(dec.out_lf0_mean), float(dec.out_lf0_scale),
                st["sg"].data_ptr(), st["sc"].data_ptr(), st["so"].data_ptr(), dg.data_ptr(),
                do4.data_ptr())
        if coop is not None and self._ar_coop(B):
            work, nbytes = _ar_work(H, B, dev)
            call("ensvs_ardec_coop_bwd", dlf0.data_ptr(), ptr(dres), coop[1].data_ptr(), *args,
                 work.data_ptr(), nbytes, Ly.stream())
        else:
            call("ensvs_ardec_bwd", dlf0.data_ptr(), ptr(dres), wpb.data_ptr(), *args,
                 Ly.stream())
        wg = Ly.wgrad_into
        # decoder weights
        wg(cell.weight_hh, dg, 4 * H, st["sh"], H, B, Tr, Tr, 4 * H, H, shift0=-1)
        wg(cell.weight_ih, dg, 4 * H, st["e"], Ce, B, Tr, Tr, 4 * H, Ce, col0=0)
        wg(cell.weight_ih, dg, 4 * H, st["sp"], 1, B, Tr, Tr, 4 * H, 1, col0=Ce)
        bsum = empty(4 * H, device=dg.device)
        K.colsum(dg, 4 * H, B * Tr, 4 * H, bsum)
        Ly.add_into_pair(bsum.data_ptr(), 4 * H, cell.bias_ih, cell.bias_hh)
        wg(dec.feat_out.weight, do4, 4, st["sh"], H, B, Tr, Tr, 4, H, col0=0)
        wg(dec.feat_out.weight, do4, 4, st["e"], Ce, B, Tr, Tr, 4, Ce, col0=H)
        de = empty(B * Tr, Ce, device=dev)
        K.gemm([K.Seg(dg, 4 * H, 4 * H, pk["dec_ih_e^T"], Tr),
                K.Seg(do4, 4, 4, pk["dec_fo_e^T"], Tr)], B, Tr, Ce, pk.bwd, de, Ce)
        Hl2 = st["y"].shape[1]
        dy = empty(M, Hl2, device=dev)
        li = self.in_lf0_idx
        x1 = xs[1].data_ptr() + 4 * li if len(xs) == 2 else None
        call("ensvs_downsample_bwd", de.data_ptr(), Ce, st["y"].data_ptr(), Hl2, Hl2,
             xs[0].data_ptr() + 4 * li, st["ld"], 1, x1, st["ld"], 1,
             dec.conv_downsample.weight.data_ptr(), B, T, dy.data_ptr(), Hl2,
             grad_of(dec.conv_downsample.weight).data_ptr(),
             grad_of(dec.conv_downsample.bias).data_ptr(), Ly.stream())
        # encoder
        da = Ly.lstm_bwd(pk, self.lstm, st["lsv"], dy, B, T, st["lens"], dev)
        F = st["hs"][2].shape[1]
        (dh3,) = Ly.conv_bwd(pk, self.conv, st["csv"], da, B, T, dev, first_dx=[("ff", F)])
        dX0 = Ly.ff_bwd(pk, self.ff, st["X0"], st["hs"], st["hs16"], dh3, B, T, dev)
        E = self.embed_dim
        dspk = torch.zeros(B, E, device=dev) if want_spk else None
        for k, sv in enumerate(st["esv"]):
            Ly.embed_bwd(self.emb, self.fc_in, sv, dX0, B, T, dspk if k == 0 else None)
        return dspk, dspk, dX0

    def _pad_infer(self, xs, ld, B, T, lens_host, masks=None):
        """pad_inference (acoustic_models/util.py:60-151) of the lf0 model alone, as the
        single-track model's inference calls it (multistream.py:1152): replicate-pad r frames
        (r - max(L) % r, never 0), free-running forward in eval mode, trim.  Returns
        lf0 (B*T,) of the unpadded frames."""
        r = self.reduction_factor
        pad = r - max(lens_host) % r
        dev = xs[0].device
        D = ld
        xps = [_replicate_pad(x, B, T, D, pad) for x in xs]
        _, lens_dev = lengths_pair([v + pad for v in lens_host], B, T + pad, dev)
        lf0, _, _ = self._fwd(xps, D, B, T + pad, lens_dev, masks=masks, training=False,
                              save=False)
        out = empty(B * T, device=dev)
        call("ensvs_copy_cols", lf0.data_ptr(), T + pad, out.data_ptr(), T, B, T, Ly.stream())
        return out

    # ---------------------------------------------------------------- reference API
    def forward(self, x, lengths=None, y=None, spk_embs=None):
        return torch_ops.lf0_call(self, x, None, spk_embs, None, lengths, y)

    def inference(self, x, lengths=None, spk_embs=None):
        if spk_embs is not None:
            raise NotImplementedError("speaker embeddings at lf0 inference are not on the path")
        B, T, D = x.shape
        lens = [int(v) for v in (lengths if lengths is not None else [T] * B)]
        x = x.contiguous().float()
        return self._pad_infer([x], D, B, T, lens).view(B, T, 1)


def _replicate_pad(x, B, T, D, pad):
    """F.pad(x, (0, 0, 0, pad), mode="replicate") of a (B, T, D) fp32 tensor."""
    xp = empty(B, T + pad, D, device=x.device)
    call("ensvs_copy_cols", x.data_ptr(), T * D, xp.data_ptr(), (T + pad) * D, B, T * D,
         Ly.stream())
    for k in range(pad):  # replicate the last frame
        call("ensvs_copy_cols", x.data_ptr() + 4 * (T - 1) * D, T * D,
             xp.data_ptr() + 4 * (T + k) * D, (T + pad) * D, B, D, Ly.stream())
    return xp


class MultiTrackBiLSTMResF0NonAttentiveDecoder(BiLSTMResF0NonAttentiveDecoder):
    """tacotron_f0.py:757-991: cross-singer log-F0 model (additive main+sub fusion)."""

    _NTRACKS = 2

    def __init__(self, in_dim=512, ff_hidden_dim=2048, conv_hidden_dim=1024, lstm_hidden_dim=256,
                 num_lstm_layers=2, dropout=0.0, out_dim=80, num_speaker=15, decoder_layers=2,
                 decoder_hidden_dim=1024, prenet_layers=2, prenet_hidden_dim=256,
                 prenet_dropout=0.5, zoneout=0.1, reduction_factor=1, downsample_by_conv=False,
                 scaled_tanh=True, in_lf0_idx=300, in_lf0_min=5.3936276, in_lf0_max=6.491111,
                 out_lf0_idx=180, out_lf0_mean=5.953093881972361,
                 out_lf0_scale=0.23435173188961034, use_mdn=False, num_gaussians=4,
                 sampling_mode="mean", in_ph_start_idx: int = 1, in_ph_end_idx: int = 50,
                 embed_dim=None, init_type="none"):
        BaseModel.__init__(self)
        self._build(in_dim, ff_hidden_dim, conv_hidden_dim, lstm_hidden_dim, num_lstm_layers,
                    dropout, out_dim, decoder_layers, decoder_hidden_dim, prenet_layers,
                    prenet_hidden_dim, prenet_dropout, zoneout, reduction_factor,
                    downsample_by_conv, scaled_tanh, in_lf0_idx, in_lf0_min, in_lf0_max,
                    out_lf0_idx, out_lf0_mean, out_lf0_scale, use_mdn, in_ph_start_idx,
                    in_ph_end_idx, embed_dim, init_type)

    def _bn_only(self, x_main, x_sub, ld, B, T, s_main, s_sub, spk_ld):
        """Forward of a call whose outputs are unused in training (the sub-track call with
        output_subtrack=False, multistream.py:1649-1651): only its BatchNorm running-statistic
        updates are observable, so only embed + FF + the conv/BN stack run."""
        pk = self._packs.ensure(self, self._register)
        dev = self.fc_in.weight.device
        li = self.in_lf0_idx
        X0, _ = self._embed(pk, [x_main, x_sub], ld, B, T, [s_main, s_sub], spk_ld, dev)
        hs, hs16 = Ly.ff_fwd(pk, self.ff, X0, B, T, dev)
        segs, b16 = self._conv_in(pk, hs[2], [x_main, x_sub], ld, B, T, dev, hs16[2])
        Ly.conv_fwd(pk, self.conv, segs, B, T, dev, True, save=False, first_b16=b16)

    # ---------------------------------------------------------------- reference API
    def forward(self, x_main, x_sub, spk_emb_main, spk_emb_sub, lengths=None, y=None):
        return torch_ops.lf0_call(self, x_main, x_sub, spk_emb_main, spk_emb_sub, lengths, y)

    def inference(self, *args, **kwargs):
        raise NotImplementedError("the multi-track model calls the lf0 model's forward "
                                  "(multistream.py:1646-1651)")




class _MultistreamHybrid(BaseModel):
    """Kernel orchestration shared by the single-track and the pairwise multi-track NPSS
    multistream models: four branches (lf0, mgc, bap, V/UV) on concurrent HIP streams,
    their backward, and the reverse-diffusion inference.  ``_MULTI`` selects the
    multi-track variant (second track, speaker embeddings, free-running lf0 decoder in
    training) or the single-track one (no speaker, teacher-forced lf0 decoder)."""

    _MULTI = True
    output_subtrack = False

    def _set_lf0_params(self):
        if hasattr(self.lf0_model, "out_lf0_mean"):
            self.lf0_model.in_lf0_min = self.in_lf0_min
            self.lf0_model.in_lf0_max = self.in_lf0_max
            self.lf0_model.out_lf0_mean = self.out_lf0_mean
            self.lf0_model.out_lf0_scale = self.out_lf0_scale

    def prediction_type(self):
        return PredictionType.MULTISTREAM_HYBRID

    def has_residual_lf0_prediction(self):
        return True

    # ------------------------------------------------------------------ helpers
    def _stream_cols(self):
        s = self.stream_sizes
        o = [0]
        for n in s:
            o.append(o[-1] + n)
        return o  # mgc [o0,o1) lf0 [o1,o2) vuv [o2,o3) bap [o3,o4)

    def _vuv_sources(self, x, ldx, y, ldy):
        o = self._stream_cols()
        src = [(x, ldx, 0, ldx)]
        if self.vuv_model_mgc_conditioning:
            src.append((y, ldy, o[0], o[1] - o[0]))
        if self.vuv_model_lf0_conditioning:
            src.append((y, ldy, o[1], o[2] - o[1]))
        if self.vuv_model_bap_conditioning:
            n = 1 if self.vuv_model_bap0_conditioning else o[4] - o[3]
            src.append((y, ldy, o[3], n))
        # merge adjacent column ranges of the same tensor
        merged = [src[0]]
        for s in src[1:]:
            p = merged[-1]
            if s[0] is p[0] and p[2] + p[3] == s[2]:
                merged[-1] = (p[0], p[1], p[2], p[3] + s[3])
            else:
                merged.append(s)
        return merged

    def _spk_vectors(self, spk0, spk1, B):
        table = self.speaker_embedding.emb.weight
        E = table.shape[1]
        out = []
        for s in (spk0, spk1):
            idx = s.reshape(-1).to(device=table.device, dtype=torch.int64).contiguous()
            v = empty(B, E, device=table.device)
            call("ensvs_gather_rows", table.data_ptr(), idx.data_ptr(), B, E, v.data_ptr(),
                 Ly.stream())
            out.append((v, idx))
        return out

    # ------------------------------------------------------------------ training
    def _fwd_prologue(self, x_main, x_sub, y_main, spk0, spk1, lengths, draws):
        self._set_lf0_params()
        B, T, D = x_main.shape
        Dy = y_main.shape[2]
        dev = x_main.device
        lens_host, lens_dev = lengths_pair(lengths, B, T, dev)
        if self._MULTI:
            (s0, i0), (s1, i1) = self._spk_vectors(spk0, spk1, B)
            E = s0.shape[1]
        else:  # single track: no speaker embedding
            s0 = i0 = s1 = i1 = None
            E = 0
        o = self._stream_cols()
        st = dict(i0=i0, i1=i1, B=B, T=T, E=E, lens_host=lens_host, lens_dev=lens_dev)
        c = dict(x_main=x_main, x_sub=x_sub, y_main=y_main, D=D, Dy=Dy, o=o, s0=s0, s1=s1,
                 draws=draws or {}, enc_src=[(x_main, D, 0, D), (y_main, Dy, o[1], o[2] - o[1])])
        return c, st

    def _fwd_branch(self, i, c, outs, st):
        """Forward of branch i (0 lf0, 1 mgc, 2 bap, 3 V/UV) into outs / st."""
        B, T, E, lens_dev = st["B"], st["T"], st["E"], st["lens_dev"]
        x_main, x_sub, y_main, D, Dy, o = c["x_main"], c["x_sub"], c["y_main"], c["D"], c["Dy"], c["o"]
        s0, s1, draws = c["s0"], c["s1"], c["draws"]
        if i == 0 and not self._MULTI:
            # single track: lf0 model with the lf0 target stream (multistream.py:1158)
            lf0, res, st["lf0"] = self.lf0_model._fwd([x_main], D, B, T, lens_dev,
                                                      masks=draws.get("lf0_main"),
                                                      teacher=(y_main, Dy, o[1]))
            outs.update(lf0=lf0, lf0_residual=res)
        elif i == 0:
            lf0, res, st["lf0"] = self.lf0_model._fwd([x_main, x_sub], D, B, T, lens_dev,
                                                      (s0, s1), E, masks=draws.get("lf0_main"))
            outs.update(lf0=lf0, lf0_residual=res)
            if self.output_subtrack:
                # sub-track call with its outputs (multistream.py:1649-1651, 1759-1768):
                # the lf0 prediction the interaction loss compares with the main one.
                # Same stream as the main call: BatchNorm running statistics are
                # updated main-then-sub, as in the reference.
                lf0_s, res_s, st["lf0_sub"] = self.lf0_model._fwd(
                    [x_sub, x_main], D, B, T, lens_dev, (s1, s0), E, masks=draws.get("lf0_sub"))
                outs.update(lf0_sub=lf0_s, lf0_residual_sub=res_s)
            elif self.training:
                # sub-track call (outputs unused without output_subtrack): BN statistics
                self.lf0_model._bn_only(x_sub, x_main, D, B, T, s1, s0, E)
        elif i == 1:
            nm, rm, st["mgc"] = self.mgc_model._fwd(c["enc_src"], B, T, lens_dev, (y_main, Dy, o[0]),
                                                    s0, E, t=draws.get("mgc_t"),
                                                    noise=draws.get("mgc_noise"),
                                                    **({"pack_ev": c["mgc_pack_ev"]}
                                                       if c.get("mgc_pack_ev") else {}))
            outs.update(mgc_noise=nm, mgc_recon=rm)
        elif i == 2:
            nb, rb, st["bap"] = self.bap_model._fwd(c["enc_src"], B, T, lens_dev, (y_main, Dy, o[3]),
                                                    s0, E, t=draws.get("bap_t"),
                                                    noise=draws.get("bap_noise"))
            outs.update(bap_noise=nb, bap_recon=rb)
        else:
            outs["vuv"], st["vuv"] = self.vuv_model._fwd(self._vuv_sources(x_main, D, y_main, Dy),
                                                         B, T, lens_dev, s0, E,
                                                         lstm_masks=draws.get("vuv_lstm"))

    def _train_fwd(self, x_main, x_sub, y_main, spk0, spk1, lengths, draws=None):
        """One training forward.  x_* (B, T, in_dim), y_main (B, T, out_dim) contiguous fp32
        device tensors.  Returns (outputs dict of (B*T, .) tensors, state)."""
        c, st = self._fwd_prologue(x_main, x_sub, y_main, spk0, spk1, lengths, draws)
        outs = {}
        # The four branches are independent until the loss: concurrent HIP streams
        # (the recurrences alone occupy only 2*B workgroups each).
        with Branches(x_main.device) as br:
            for i in range(4):
                with br.on(i):
                    self._fwd_branch(i, c, outs, st)
        return outs, st

    def _bwd_branch(self, i, st, g, dsp):
        """Backward of branch i from its output grads g; its speaker-vector grads -> dsp."""
        spk = self._MULTI
        if i == 0 and not spk:
            self.lf0_model._bwd(st["lf0"], g["lf0"], g.get("lf0_residual"), want_spk=False)
        elif i == 0:
            dmain, dsub, _ = self.lf0_model._bwd(st["lf0"], g["lf0"], g.get("lf0_residual"))
            dsp["lf0"], dsp["lf0_sub_in"] = dmain, dsub
            if st.get("lf0_sub") is not None and (g.get("lf0_sub") is not None or
                                                  g.get("lf0_residual_sub") is not None):
                gs = g.get("lf0_sub")
                if gs is None:
                    gs = torch.zeros(st["B"] * st["T"], device=st["lens_dev"].device)
                dsp["lf0_sub"], _, _ = self.lf0_model._bwd(st["lf0_sub"], gs,
                                                           g.get("lf0_residual_sub"))
        elif i == 1:
            hooks = []
            if dsp.get("_reduce") is not None:
                red = dsp["_reduce"]
                hooks.append(lambda: red("mgc_denoiser"))
            hook = (lambda: [h() for h in hooks]) if hooks else None  # noqa: E731
            dsp["mgc"] = self.mgc_model._bwd(st["mgc"], g["mgc_recon"], after_denoiser=hook,
                                             want_spk=spk)
        elif i == 2:
            dsp["bap"] = self.bap_model._bwd(st["bap"], g["bap_recon"], want_spk=spk)
        else:
            _, dsp["vuv"] = self.vuv_model._bwd(st["vuv"], g["vuv"], want_spk=spk)

    def _l1_terms(self, outs, y_main):
        """The masked-L1 terms of the multistream-hybrid loss (train_acoustic_multitrack.py:
        120-173): diffusion noise vs its prediction for mgc / bap, lf0 and V/UV vs the
        targets.  Returns (preds, targets, grad keys) for train.masked_l1."""
        Dy = y_main.shape[2]
        o = self._stream_cols()
        nm, nb = self.stream_sizes[0], self.stream_sizes[3]
        preds = [(outs["mgc_recon"], nm, 0, nm), (outs["lf0"], 1, 0, 1), (outs["vuv"], 1, 0, 1),
                 (outs["bap_recon"], nb, 0, nb)]
        targets = [(outs["mgc_noise"], nm, 0), (y_main, Dy, o[1]), (y_main, Dy, o[2]),
                   (outs["bap_noise"], nb, 0)]
        return preds, targets, ["mgc_recon", "lf0", "vuv", "bap_recon"]

    def _bwd_epilogue(self, st, dsp):
        """Speaker-embedding gradient: the branch contributions, summed after the join."""
        if not self._MULTI:
            return
        B, E = st["B"], st["E"]
        dev = st["lens_dev"].device
        dsc, dsub = dsp.get("lf0_sub"), dsp["lf0_sub_in"]
        ds0 = torch.zeros(B, E, device=dev)
        for k in ("mgc", "bap", "vuv", "lf0") + (("lf0_sub",) if dsc is not None else ()):
            call("ensvs_axpy", ds0.data_ptr(), dsp[k].data_ptr(), 1.0, B * E, Ly.stream())
        if dsc is not None:  # the sub call's fused input holds both speaker vectors too
            call("ensvs_axpy", dsub.data_ptr(), dsc.data_ptr(), 1.0, B * E, Ly.stream())
        table = grad_of(self.speaker_embedding.emb.weight)
        call("ensvs_spk_scatter", ds0.data_ptr(), B, E, st["i0"].data_ptr(), table.data_ptr(),
             Ly.stream())
        call("ensvs_spk_scatter", dsub.data_ptr(), B, E, st["i1"].data_ptr(), table.data_ptr(),
             Ly.stream())

    def _train_bwd(self, st, g):
        """g: dict of grads (B*T, .) for mgc_recon, lf0, vuv, bap_recon [, lf0_residual]
        [, lf0_sub, lf0_residual_sub (output_subtrack)]."""
        dsp = {}
        with Branches(st["lens_dev"].device) as br:  # same branch -> stream assignment as _train_fwd
            for i in range(4):
                with br.on(i):
                    self._bwd_branch(i, st, g, dsp)
        self._bwd_epilogue(st, dsp)

    def _train_fused(self, x_main, x_sub, y_main, spk0, spk1, lengths, draws, branch_loss,
                     reduce_hook=None):
        """Training forward + loss gradient + backward with each branch end to end on its
        own stream: a branch's loss gradient needs only its own outputs (the masked L1
        normaliser is known on the host), so its backward starts when its forward ends,
        not when the slowest forward does.  branch_loss(i, outs, st) -> (partial loss
        (1,) tensor, grads dict of branch i); the partial losses are summed after the
        join.  reduce_hook(tag): called on the branch's stream where a parameter group's
        gradients are final ("lf0", "mgc_denoiser", "mgc", "bap", "vuv";
        train.BucketedAllReduce).  Returns (loss, outs)."""
        c, st = self._fwd_prologue(x_main, x_sub, y_main, spk0, spk1, lengths, draws)
        outs, dsp, parts = {}, {}, {}
        if reduce_hook is not None:
            dsp["_reduce"] = reduce_hook
        tags = ("lf0", "mgc", "bap", "vuv")
        fwd_done = {}
        with Branches(x_main.device) as br:
            for i in range(4):
                with br.on(i):
                    if len(EXCL_BRANCHES) < 4:
                        call("ensvs_set_recurrence_exclusive", int(i in EXCL_BRANCHES))
                    # schedule knob: branch i starts after branch a's forward (BRANCH_AFTER)
                    a = BRANCH_AFTER.get(i)
                    if a is not None and a in fwd_done:
                        torch.cuda.current_stream().wait_event(fwd_done[a])
                    if i == PREPACK_ON and hasattr(self.mgc_model, "prepack"):
                        # the mgc denoiser's weight repack at the head of this branch
                        c["mgc_pack_ev"] = self.mgc_model.prepack()
                    self._fwd_branch(i, c, outs, st)
                    if i in BRANCH_AFTER.values():
                        fwd_done[i] = torch.cuda.current_stream().record_event()
                    parts[i], g = branch_loss(i, outs, st)
                    self._bwd_branch(i, st, g, dsp)
                    if reduce_hook is not None:
                        reduce_hook(tags[i])
        if len(EXCL_BRANCHES) < 4:
            call("ensvs_set_recurrence_exclusive", 1)
        loss = parts[0]
        for i in (1, 2, 3):
            call("ensvs_axpy", loss.data_ptr(), parts[i].data_ptr(), 1.0, 1, Ly.stream())
        self._bwd_epilogue(st, dsp)
        return loss, outs

    # ------------------------------------------------------------------ inference
    def _infer(self, x_main, x_sub, spk0, spk1, lengths, noises=None, masks=None, graph=None):
        """noises: {"mgc"/"bap": (K+1, B*T, M) replayed draws}; masks: (B*T/4,) AR-decoder
        dropout keep-masks of the main-track call; graph: captured reverse diffusion."""
        self._set_lf0_params()
        B, T, D = x_main.shape
        dev = x_main.device
        lens_host, lens_dev = lengths_pair(lengths, B, T, dev)
        if self._MULTI:
            (s0, _), (s1, _) = self._spk_vectors(spk0, spk1, B)
            E = s0.shape[1]
            lf0, _, _ = self.lf0_model._fwd([x_main, x_sub], D, B, T, lens_dev, (s0, s1), E,
                                            masks=masks, training=False, save=False)
        else:
            # single track: lf0_model.inference, itself pad_inference (multistream.py:1152),
            # i.e. r more replicated frames on the already padded input, then trimmed
            s0, E = None, 0
            lf0 = self.lf0_model._pad_infer([x_main], D, B, T, lens_host, masks=masks)
        o = self._stream_cols()
        Dy = self.out_dim
        out = empty(B * T, Dy, device=dev)
        call("ensvs_copy_cols", lf0.data_ptr(), 1, out.data_ptr() + 4 * o[1], Dy, B * T, 1,
             Ly.stream())
        enc_src = [(x_main, D, 0, D), (out, Dy, o[1], 1)]
        nz = noises or {}
        # the two reverse diffusions are independent: concurrent HIP streams
        with Branches(dev) as br:
            with br.on(1):
                mgc = self.mgc_model._inference(enc_src, B, T, lens_dev, s0, E, nz.get("mgc"),
                                                graph=graph)
            with br.on(2):
                bap = self.bap_model._inference(enc_src, B, T, lens_dev, s0, E, nz.get("bap"),
                                                graph=graph)
        if br.on_side:  # consumed on the main stream: keep the blocks alive for it
            main = torch.cuda.current_stream(dev)
            mgc.record_stream(main)
            bap.record_stream(main)
        call("ensvs_copy_cols", mgc.data_ptr(), o[1] - o[0], out.data_ptr() + 4 * o[0], Dy, B * T,
             o[1] - o[0], Ly.stream())
        call("ensvs_copy_cols", bap.data_ptr(), o[4] - o[3], out.data_ptr() + 4 * o[3], Dy, B * T,
             o[4] - o[3], Ly.stream())
        vuv, _ = self.vuv_model._fwd(self._vuv_sources(x_main, D, out, Dy), B, T, lens_dev, s0, E,
                                     training=False, save=False)
        call("ensvs_copy_cols", vuv.data_ptr(), 1, out.data_ptr() + 4 * o[2], Dy, B * T, 1,
             Ly.stream())
        return out.view(B, T, Dy)


class MultiTrackNPSSMDNMultistreamParametricModel(_MultistreamHybrid):
    """multistream.py:1482-1778: pairwise (main, sub) ensemble diffusion model."""

    def __init__(self, in_dim: int, out_dim: int, stream_sizes: list, reduction_factor: int,
                 lf0_model: nn.Module, mgc_model: nn.Module, bap_model: nn.Module,
                 vuv_model: nn.Module, speaker_embedding: nn.Module, in_rest_idx=0, in_lf0_idx=51,
                 in_lf0_min=5.3936276, in_lf0_max=6.491111, out_lf0_idx=60,
                 out_lf0_mean=5.953093881972361, out_lf0_scale=0.23435173188961034,
                 vuv_model_bap_conditioning=True, vuv_model_bap0_conditioning=False,
                 vuv_model_lf0_conditioning=True, vuv_model_mgc_conditioning=False,
                 output_subtrack=False):
        super().__init__()
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.stream_sizes = stream_sizes
        self.reduction_factor = reduction_factor
        self.vuv_model_bap_conditioning = vuv_model_bap_conditioning
        self.vuv_model_bap0_conditioning = vuv_model_bap0_conditioning
        self.vuv_model_lf0_conditioning = vuv_model_lf0_conditioning
        self.vuv_model_mgc_conditioning = vuv_model_mgc_conditioning
        self.output_subtrack = output_subtrack
        assert len(stream_sizes) in [4]
        self.lf0_model = lf0_model
        self.mgc_model = mgc_model
        self.bap_model = bap_model
        self.vuv_model = vuv_model
        self.speaker_embedding = speaker_embedding
        self.in_rest_idx = in_rest_idx
        self.in_lf0_idx = in_lf0_idx
        self.in_lf0_min = in_lf0_min
        self.in_lf0_max = in_lf0_max
        self.out_lf0_idx = out_lf0_idx
        self.out_lf0_mean = out_lf0_mean
        self.out_lf0_scale = out_lf0_scale

    def is_autoregressive(self):
        return True  # the lf0 model is autoregressive

    # ---------------------------------------------------------------- reference API
    def forward(self, x_main, x_sub, spks_list, lengths=None, ys=None):
        assert x_main.shape[-1] == self.in_dim
        if ys is None:
            out = self._infer(x_main.contiguous().float(), x_sub.contiguous().float(),
                              spks_list[0], spks_list[1], lengths)
            return out, out
        outs = torch_ops.multitrack_call(self, x_main, x_sub, ys[0], spks_list[0], spks_list[1],
                                         lengths)
        nm, rm, lf0, vuv, nb, rb, res = outs[:7]
        main = (((nm, rm), lf0, vuv, (nb, rb)), res)
        if not self.output_subtrack:
            return main, (None, None)
        # sub track: ground truth except lf0 (multistream.py:1759-1764)
        o = self._stream_cols()
        y1 = ys[1]
        sub = (y1[..., o[0]:o[1]], outs[7], y1[..., o[2]:o[3]], y1[..., o[3]:o[4]])
        return main, (sub, outs[8])

    def inference(self, x_main, x_sub, spks=None, lengths=None, draws=None):
        """pad_inference_multitrack (acoustic_models/util.py:154-188): replicate-pad to a
        multiple of r (r frames when already divisible), run, trim.  ``draws`` (tests only)
        replays random draws: dict(noises=..., masks=..., graph=...) of ``_infer``."""
        r = self.reduction_factor
        B, T, D = x_main.shape
        lens = [int(v) for v in (lengths if lengths is not None else [T] * B)]
        pad = r - max(lens) % r
        dev = x_main.device
        xs = []
        for x in (x_main, x_sub):
            x = x.contiguous().float()
            xp = empty(B, T + pad, D, device=dev)
            call("ensvs_copy_cols", x.data_ptr(), T * D, xp.data_ptr(), (T + pad) * D, B, T * D,
                 Ly.stream())
            for k in range(pad):  # replicate the last frame
                call("ensvs_copy_cols", x.data_ptr() + 4 * (T - 1) * D, T * D,
                     xp.data_ptr() + 4 * (T + k) * D, (T + pad) * D, B, D, Ly.stream())
            xs.append(xp)
        out = self._infer(xs[0], xs[1], spks[0], spks[1], [v + pad for v in lens], **(draws or {}))
        return out[:, :-pad]


class NPSSMDNMultistreamParametricModel(_MultistreamHybrid):
    """multistream.py:1025-1243: single-track NPSS multistream model (BASELINE config 2 with
    the recipe's diffusion config acoustic_nnsvs_world_multi_ar_f0_diff_mgcbap.yaml):
    teacher-forced residual-F0 model, mgc / bap GaussianDiffusion conditioned on
    [x, lf0] (ground truth in training), V/UV conditioned per the vuv_model_* flags."""

    _MULTI = False

    def __init__(self, in_dim: int, out_dim: int, stream_sizes: list, reduction_factor: int,
                 lf0_model: nn.Module, mgc_model: nn.Module, bap_model: nn.Module,
                 vuv_model: nn.Module, in_rest_idx=0, in_lf0_idx=51, in_lf0_min=5.3936276,
                 in_lf0_max=6.491111, out_lf0_idx=60, out_lf0_mean=5.953093881972361,
                 out_lf0_scale=0.23435173188961034, vuv_model_bap_conditioning=True,
                 vuv_model_bap0_conditioning=False, vuv_model_lf0_conditioning=True,
                 vuv_model_mgc_conditioning=False):
        super().__init__()
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.stream_sizes = stream_sizes
        self.reduction_factor = reduction_factor
        self.vuv_model_bap_conditioning = vuv_model_bap_conditioning
        self.vuv_model_bap0_conditioning = vuv_model_bap0_conditioning
        self.vuv_model_lf0_conditioning = vuv_model_lf0_conditioning
        self.vuv_model_mgc_conditioning = vuv_model_mgc_conditioning
        assert len(stream_sizes) in [4]
        if not isinstance(lf0_model, BiLSTMResF0NonAttentiveDecoder) or \
                isinstance(lf0_model, MultiTrackBiLSTMResF0NonAttentiveDecoder):
            raise NotImplementedError("lf0_model: BiLSTMResF0NonAttentiveDecoder (recipe)")
        self.lf0_model = lf0_model
        self.mgc_model = mgc_model
        self.bap_model = bap_model
        self.vuv_model = vuv_model
        self.in_rest_idx = in_rest_idx
        self.in_lf0_idx = in_lf0_idx
        self.in_lf0_min = in_lf0_min
        self.in_lf0_max = in_lf0_max
        self.out_lf0_idx = out_lf0_idx
        self.out_lf0_mean = out_lf0_mean
        self.out_lf0_scale = out_lf0_scale

    def is_autoregressive(self):
        return (self.mgc_model.is_autoregressive() or self.lf0_model.is_autoregressive()
                or self.vuv_model.is_autoregressive() or self.bap_model.is_autoregressive())

    # ---------------------------------------------------------------- reference API
    def forward(self, x, lengths=None, y=None):
        """multistream.py:1133-1233: training (teacher forcing) when y is given, else the
        inference cascade on x as is; returns ((mgc, lf0, vuv, bap), lf0_residual) /
        (out, out)."""
        assert x.shape[-1] == self.in_dim
        if y is None:
            out = self._infer(x.contiguous().float(), None, None, None, lengths)
            return out, out
        outs = torch_ops.multitrack_call(self, x, None, y, None, None, lengths)
        nm, rm, lf0, vuv, nb, rb, res = outs[:7]
        return ((nm, rm), lf0, vuv, (nb, rb)), res

    def inference(self, x, lengths=None, draws=None):
        """pad_inference(mdn=True) (acoustic_models/util.py:60-141): replicate-pad
        r - max(L) % r frames (never 0), forward(y=None), trim; returns (mu, sigma) = (out,
        out).  ``draws`` (tests only): dict(noises=..., masks=...) replayed draws."""
        r = self.reduction_factor
        B, T, D = x.shape
        lens = [int(v) for v in (lengths if lengths is not None else [T] * B)]
        pad = r - max(lens) % r
        xp = _replicate_pad(x.contiguous().float(), B, T, D, pad)
        out = self._infer(xp, None, None, None, [v + pad for v in lens], **(draws or {}))
        mu = out[:, :-pad]
        return mu, mu


class MultiTrackMultistreamSeparateF0ParametricModel(_MultistreamHybrid):
    """multistream.py:348-577: the recipe's default pairwise model (config.yaml:93-95,
    multitrack_acoustic_nnsvs_world_multi_ar_f0.yaml).  The cross-singer log-F0 model (main
    and sub call), the concatenation-fusion MultiTrackLSTMEncoder, and FFConvLSTM mgc / V/UV
    / bap decoders on [encoder out, rest flag, lf0] (ground-truth lf0 under
    lf0_teacher_forcing in training, the predicted one otherwise).

    Reference quirks kept: the sub-track decoders read the MAIN track's decoder input
    (multistream.py:519-521), so the sub outputs differ from the main ones only by the LSTM
    dropout draws and the log-F0 stream; the sub track's encoder output is never read
    (multistream.py:490-492, 507-510) and is not computed here.  The fused train step
    (train.train_step; loss on the main outputs) runs the unobservable sub calls only for
    their BatchNorm running-statistic updates: the lf0 model's conv stack on the sub input,
    and for the decoders a second update with the main call's batch statistics (same input)."""

    _MULTI = True
    _train_fused = None  # the per-branch fused schedule is the diffusion model's

    def __init__(self, in_dim: int, out_dim: int, stream_sizes: list, reduction_factor: int,
                 encoder: nn.Module, mgc_model: nn.Module, lf0_model: nn.Module,
                 vuv_model: nn.Module, bap_model: nn.Module, speaker_embedding: nn.Module,
                 vib_model: nn.Module = None, vib_flags_model: nn.Module = None, in_rest_idx=1,
                 in_lf0_idx=300, in_lf0_min=5.3936276, in_lf0_max=6.491111, out_lf0_idx=180,
                 out_lf0_mean=5.953093881972361, out_lf0_scale=0.23435173188961034,
                 lf0_teacher_forcing=True):
        super().__init__()
        from .model import FFConvLSTM, MultiTrackLSTMEncoder
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.stream_sizes = stream_sizes
        self.reduction_factor = reduction_factor
        self.lf0_teacher_forcing = lf0_teacher_forcing
        assert len(stream_sizes) in [4]
        if vib_model is not None or vib_flags_model is not None:
            raise NotImplementedError("vib_model / vib_flags_model (deprecated in the reference)")
        if not isinstance(lf0_model, MultiTrackBiLSTMResF0NonAttentiveDecoder):
            raise NotImplementedError("lf0_model: MultiTrackBiLSTMResF0NonAttentiveDecoder")
        if encoder is not None and not isinstance(encoder, MultiTrackLSTMEncoder):
            raise NotImplementedError("encoder: MultiTrackLSTMEncoder (recipe) or None")
        for m in (mgc_model, vuv_model, bap_model):
            if not isinstance(m, FFConvLSTM):
                raise NotImplementedError("mgc / vuv / bap models: FFConvLSTM (recipe)")
        self.encoder = encoder
        if self.encoder is not None:
            assert not encoder.is_autoregressive()
        self.mgc_model = mgc_model
        self.lf0_model = lf0_model
        self.vuv_model = vuv_model
        self.bap_model = bap_model
        self.speaker_embedding = speaker_embedding
        self.in_rest_idx = in_rest_idx
        self.in_lf0_idx = in_lf0_idx
        self.in_lf0_min = in_lf0_min
        self.in_lf0_max = in_lf0_max
        self.out_lf0_idx = out_lf0_idx
        self.out_lf0_mean = out_lf0_mean
        self.out_lf0_scale = out_lf0_scale

    def prediction_type(self):
        return PredictionType.DETERMINISTIC  # BaseModel's default (nnsvs/base.py:128-136)

    def is_autoregressive(self):
        return (self.mgc_model.is_autoregressive() or self.lf0_model.is_autoregressive()
                or self.vuv_model.is_autoregressive() or self.bap_model.is_autoregressive())

    def _decoders(self):
        return (("mgc", self.mgc_model), ("vuv", self.vuv_model), ("bap", self.bap_model))

    # ------------------------------------------------------------------ core
    def _fwd_core(self, x_main, x_sub, y_main, y_sub, spk0, spk1, lengths, training,
                  want_sub, draws=None, save=True, sub_decoders=None):
        """x_*: (B, T, in_dim) fp32 contiguous; y_*: (B, T, out_dim) targets or None;
        want_sub: the sub-track lf0 call with outputs; sub_decoders (default want_sub): the
        sub-track decoder calls.  Returns (outputs dict of (B*T, .) tensors, state)."""
        sub_decoders = want_sub if sub_decoders is None else sub_decoders
        self._set_lf0_params()
        B, T, D = x_main.shape
        dev = x_main.device
        lens_host, lens_dev = lengths_pair(lengths, B, T, dev)
        if max(lens_host) != T:
            raise ValueError("max(lengths) must equal the frame count (multistream.py:495-510 "
                             "concatenates T-frame rest flags with the packed outputs)")
        (s0, i0), (s1, i1) = self._spk_vectors(spk0, spk1, B)
        E = s0.shape[1]
        o = self._stream_cols()
        Dy = self.out_dim
        dr = draws or {}
        teach = self.lf0_teacher_forcing and y_main is not None
        M = B * T
        outs = {}
        st = dict(i0=i0, i1=i1, B=B, T=T, E=E, lens_host=lens_host, lens_dev=lens_dev,
                  teach=teach, want_sub=want_sub)
        if self.encoder is not None:
            N = self.encoder.out_dim
            Din = N + 2
            # rows padded to a multiple of 8 columns (zeros): the decoders' first GEMM and its
            # weight gradient then take a bf16 copy, and their input gradients come back in
            # rows the encoder's bf16 GEMMs can read (DEC_PAD off: the fp32 form)
            ldX = (Din + 7) // 8 * 8 if DEC_PAD["on"] else (Din + 3) // 4 * 4
            X = empty(M, ldX, device=dev)
        # phase 1: the lf0 model (main and sub calls) beside the encoder
        with Branches(dev) as br:
            with br.on(0):
                tm = None if y_main is None else (y_main, Dy, o[1])
                outs["lf0"], outs["lf0_residual"], st["lf0"] = self.lf0_model._fwd(
                    [x_main, x_sub], D, B, T, lens_dev, (s0, s1), E,
                    masks=dr.get("lf0_main"), training=training, save=save, teacher=tm)
                if want_sub:
                    ts = None if y_sub is None else (y_sub, Dy, o[1])
                    outs["lf0_sub"], outs["lf0_residual_sub"], st["lf0_sub"] = \
                        self.lf0_model._fwd([x_sub, x_main], D, B, T, lens_dev, (s1, s0), E,
                                            masks=dr.get("lf0_sub"), training=training,
                                            save=save, teacher=ts)
                elif training:
                    self.lf0_model._bn_only(x_sub, x_main, D, B, T, s1, s0, E)
            if self.encoder is not None:
                _, st["enc"] = self.encoder._fwd(x_main, x_sub, D, B, T, lens_dev, (s0, s1), E,
                                                 training=training, save=save,
                                                 lstm_masks=dr.get("enc_lstm"),
                                                 out=(X, X.shape[1]))
        if self.encoder is not None:
            # [encoder out, rest flag, lf0] (multistream.py:495-510)
            call("ensvs_copy_cols", x_main.data_ptr() + 4 * self.in_rest_idx, D,
                 X.data_ptr() + 4 * N, X.shape[1], M, 1, Ly.stream())
            lsrc, lld = (y_main.data_ptr() + 4 * o[1], Dy) if teach else \
                (outs["lf0"].data_ptr(), 1)
            call("ensvs_copy_cols", lsrc, lld, X.data_ptr() + 4 * (N + 1), X.shape[1], M, 1,
                 Ly.stream())
            src = [(X, X.shape[1], 0, Din)]
            X16 = None
            if DEC_PAD["on"] and ldX > Din and gemm_dtype() == _lib.DT_BF16:
                X.narrow(1, Din, ldX - Din).zero_()
                X16 = K.cast_bf16(X, ldX, ldX, M)
            st["dx_ld"] = ldX if DEC_PAD["on"] else None
        else:
            src = [(x_main, D, 0, D)]
            X16 = None
            st["dx_ld"] = None
        st["X"] = src
        # phase 2: the three decoders (sub calls on the same input: multistream.py:519-521)
        conv_ev = []
        order = DEC_ORDER["on"] and not sub_decoders

        def mark():
            conv_ev.append(torch.cuda.current_stream().record_event())
        with Branches(dev) as br:
            for bi, (name, m) in enumerate(self._decoders()):
                with br.on(bi):
                    if order and bi > 0 and conv_ev and br.on_side:
                        torch.cuda.current_stream().wait_event(conv_ev[0])
                    outs[name], st[name] = m._fwd(
                        src, B, T, lens_dev, training=training, save=save,
                        lstm_masks=dr.get(f"{name}_lstm"),
                        bn_updates=1 if sub_decoders or not training else 2, x16=X16,
                        after_conv=mark if order and bi == 0 else None)
                    if sub_decoders:
                        outs[name + "_sub"], st[name + "_sub"] = m._fwd(
                            src, B, T, lens_dev, training=training, save=save,
                            lstm_masks=dr.get(f"{name}_sub_lstm"), x16=X16)
        return outs, st

    def _bwd_core(self, st, g):
        """g: grads (B*T, .) keyed like the outputs (missing = zero)."""
        B, T, E = st["B"], st["T"], st["E"]
        M = B * T
        dev = st["lens_dev"].device
        dX = {}
        later = {}
        with Branches(dev) as br:
            for bi, (name, m) in enumerate(self._decoders()):
                with br.on(bi):
                    acc = None
                    for key in (name, name + "_sub"):
                        if key not in st or g.get(key) is None:
                            continue
                        d, _ = m._bwd(st[key], g[key].contiguous(), dx_ld=st.get("dx_ld"),
                                      later=later.setdefault(bi, []) if DEC_LATER["on"]
                                      else None)
                        if acc is None:
                            acc = d
                        else:
                            call("ensvs_axpy", acc.data_ptr(), d.data_ptr(), 1.0, d.numel(),
                                 Ly.stream())
                    dX[name] = acc
        parts = [d for d in dX.values() if d is not None]
        dsum = None
        if parts:
            dsum = parts[0]
            for d in parts[1:]:
                call("ensvs_axpy", dsum.data_ptr(), d.data_ptr(), 1.0, d.numel(), Ly.stream())
        enc = self.encoder is not None
        glf0 = g.get("lf0")
        if glf0 is None:
            glf0 = torch.zeros(M, device=dev)
        if enc and dsum is not None and not st["teach"]:
            # predicted lf0 fed the decoders: its column of the decoder-input gradient
            N = self.encoder.out_dim
            gl = empty(M, device=dev)
            call("ensvs_copy_cols", dsum.data_ptr() + 4 * (N + 1), dsum.shape[1], gl.data_ptr(),
                 1, M, 1, Ly.stream())
            call("ensvs_axpy", gl.data_ptr(), glf0.contiguous().data_ptr(), 1.0, M, Ly.stream())
            glf0 = gl
        dsp = {}
        with Branches(dev) as br:
            with br.on(0):
                dsp["lf0"], _, _ = self.lf0_model._bwd(st["lf0"], glf0.contiguous().view(-1),
                                                       g.get("lf0_residual"))
                if "lf0_sub" in st and (g.get("lf0_sub") is not None or
                                        g.get("lf0_residual_sub") is not None):
                    gs = g.get("lf0_sub")
                    if gs is None:
                        gs = torch.zeros(M, device=dev)
                    dsp["lf0_sub"], _, _ = self.lf0_model._bwd(
                        st["lf0_sub"], gs.contiguous().view(-1), g.get("lf0_residual_sub"))
            # the decoders' parameter gradients, each on its forward's stream
            for bi, fns in later.items():
                with br.on(bi):
                    for f in fns:
                        f()
            if enc and dsum is not None:
                dsp["enc0"], dsp["enc1"], _ = self.encoder._bwd(
                    st["enc"], dsum, ld=dsum.shape[1], want_spk=True)
        # speaker vectors: the lf0 calls' fused input holds both tracks' vectors
        ds = [torch.zeros(B, E, device=dev) for _ in range(2)]
        for k in range(2):
            for key in ("lf0", "lf0_sub", "enc0" if k == 0 else "enc1"):
                if dsp.get(key) is not None:
                    call("ensvs_axpy", ds[k].data_ptr(), dsp[key].data_ptr(), 1.0, B * E,
                         Ly.stream())
        table = grad_of(self.speaker_embedding.emb.weight)
        call("ensvs_spk_scatter", ds[0].data_ptr(), B, E, st["i0"].data_ptr(), table.data_ptr(),
             Ly.stream())
        call("ensvs_spk_scatter", ds[1].data_ptr(), B, E, st["i1"].data_ptr(), table.data_ptr(),
             Ly.stream())

    def _assemble(self, outs, sfx=""):
        """cat([mgc, lf0, vuv, bap], -1) (multistream.py:559-560) as (B*T, out_dim)."""
        o = self._stream_cols()
        Dy = self.out_dim
        M = outs["mgc" + sfx].shape[0]
        out = empty(M, Dy, device=outs["mgc" + sfx].device)
        for k, name in enumerate(("mgc", "lf0", "vuv", "bap")):
            n = o[k + 1] - o[k]
            call("ensvs_copy_cols", outs[name + sfx].data_ptr(), n, out.data_ptr() + 4 * o[k], Dy,
                 M, n, Ly.stream())
        return out

    def _split(self, g, sfx, into):
        """Per-stream contiguous grads of a (B*T, out_dim) output grad."""
        o = self._stream_cols()
        Dy = self.out_dim
        M = g.shape[0]
        for k, name in enumerate(("mgc", "lf0", "vuv", "bap")):
            n = o[k + 1] - o[k]
            d = empty(M, n, device=g.device)
            call("ensvs_copy_cols", g.data_ptr() + 4 * o[k], Dy, d.data_ptr(), n, M, n,
                 Ly.stream())
            into[name + sfx] = d.view(-1) if name == "lf0" else d

    # ------------------------------------------------------------------ fused train step
    def _train_fwd(self, x_main, x_sub, y_main, spk0, spk1, lengths, draws=None):
        return self._fwd_core(x_main, x_sub, y_main, None, spk0, spk1, lengths, True, False,
                              draws)

    def _train_bwd(self, st, g):
        self._bwd_core(st, g)

    def _l1_terms(self, outs, y_main):
        """The reference's deterministic loss (train_acoustic_multitrack.py:197-238,
        stream_wise_loss false): L1 of the whole main output against the main targets,
        mean over valid frames x out_dim."""
        o = self._stream_cols()
        Dy = y_main.shape[2]
        preds, targets, keys = [], [], []
        for k, name in enumerate(("mgc", "lf0", "vuv", "bap")):
            n = o[k + 1] - o[k]
            preds.append((outs[name], n, 0, n))
            targets.append((y_main, Dy, o[k]))
            keys.append(name)
        return preds, targets, keys

    # ------------------------------------------------------------------ inference
    def _infer(self, x_main, x_sub, spk0, spk1, lengths, masks=None):
        """multistream.py:447-567 with ys=None: (out_main, out_sub) (B, T, out_dim); the
        sub output's mgc / V/UV / bap equal the main ones (same input, no dropout).
        masks (tests only): dict(lf0_main=..., lf0_sub=...) AR prenet keep-masks to replay."""
        B, T, _ = x_main.shape
        outs, _ = self._fwd_core(x_main, x_sub, None, None, spk0, spk1, lengths, False, True,
                                 masks, save=False, sub_decoders=False)
        for name, _m in self._decoders():
            outs[name + "_sub"] = outs[name]
        return self._assemble(outs).view(B, T, -1), self._assemble(outs, "_sub").view(B, T, -1)

    # ---------------------------------------------------------------- reference API
    def forward(self, x_main, x_sub, spks_list, lengths=None, ys=None):
        assert x_main.shape[-1] == self.in_dim
        if ys is None:
            return self._infer(x_main.contiguous().float(), x_sub.contiguous().float(),
                               spks_list[0], spks_list[1], lengths)
        om, rm, os_, rs = torch_ops.separate_f0_call(self, x_main, x_sub, ys[0], ys[1],
                                                     spks_list[0], spks_list[1], lengths)
        return (om, rm), (os_, rs)

    def inference(self, x_main, x_sub, spks=None, lengths=None, draws=None):
        """pad_inference_multitrack (acoustic_models/util.py:154-188): replicate-pad r -
        max(L) % r frames (r when divisible), forward, main output, trim.  draws (tests
        only): dict(lf0_main=..., lf0_sub=...) AR prenet keep-masks to replay."""
        r = self.reduction_factor
        B, T, D = x_main.shape
        lens = [int(v) for v in (lengths if lengths is not None else [T] * B)]
        pad = r - max(lens) % r
        xm = _replicate_pad(x_main.contiguous().float(), B, T, D, pad)
        xs = _replicate_pad(x_sub.contiguous().float(), B, T, D, pad)
        out, _ = self._infer(xm, xs, spks[0], spks[1], [v + pad for v in lens], masks=draws)
        return out[:, :-pad]

