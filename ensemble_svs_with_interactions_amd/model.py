"""Encoders of the multi-track path: ``FFConvLSTM`` and ``SpeakerEmbedding``.

Drop-in for nnsvs.model.FFConvLSTM (nnsvs/model.py:779-927) and
nnsvs.model.SpeakerEmbedding (nnsvs/model.py:35-53): same constructor
arguments, ``forward``/``inference`` signatures and ``state_dict`` keys.  The
nn.Linear / nn.Conv1d / nn.BatchNorm1d / nn.LSTM members are parameter
containers only; their forward methods are never called — every op runs in
libensvs.so.
"""
import torch
from torch import nn

from . import layers as Ly
from .base import BaseModel, PredictionType
from . import torch_ops
from .engine import ModulePacks, empty


def init_weights(net, init_type="normal", init_gain=0.02):
    """nnsvs/util.py:31-67 (initialisation only; plumbing)."""
    if init_type == "none" or init_type is None:
        return

    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, "weight") and (classname.find("Conv") != -1 or classname.find("Linear") != -1):
            if init_type == "normal":
                nn.init.normal_(m.weight.data, 0.0, init_gain)
            elif init_type == "xavier_normal":
                nn.init.xavier_normal_(m.weight.data, gain=init_gain)
            elif init_type == "kaiming_normal":
                nn.init.kaiming_normal_(m.weight.data, a=0, mode="fan_in")
            elif init_type == "orthogonal":
                nn.init.orthogonal_(m.weight.data, gain=init_gain)
            else:
                raise NotImplementedError(init_type)
            if hasattr(m, "bias") and m.bias is not None:
                nn.init.constant_(m.bias.data, 0.0)
        elif classname.find("BatchNorm2d") != -1:
            nn.init.normal_(m.weight.data, 1.0, init_gain)
            nn.init.constant_(m.bias.data, 0.0)

    net.apply(init_func)


class SpeakerEmbedding(BaseModel):
    """nnsvs/model.py:35-53."""

    def __init__(self, num_embeddings, embedding_dim, padding_idx, std=0.01):
        super().__init__()
        self.emb = nn.Embedding(num_embeddings, embedding_dim, padding_idx=padding_idx)
        self.std = std

    def forward(self, x, lengths=None, y=None):
        return torch.ops.ensvs.embedding_gather(self.emb.weight, x)

    def embedding_dim(self):
        return self.emb.embedding_dim





class FFConvLSTM(BaseModel):
    """FFN + Conv1d + LSTM (nnsvs/model.py:779-927), MI355X kernels."""

    def __init__(self, in_dim, ff_hidden_dim=2048, conv_hidden_dim=1024, lstm_hidden_dim=256,
                 out_dim=67, dropout=0.0, num_lstm_layers=2, bidirectional=True, init_type="none",
                 use_mdn=False, dim_wise=True, num_gaussians=4, in_ph_start_idx: int = 1,
                 in_ph_end_idx: int = 50, embed_dim=None):
        super().__init__()
        if use_mdn:
            raise NotImplementedError("FFConvLSTM(use_mdn=True) is not on the multi-track path")
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.in_ph_start_idx = in_ph_start_idx
        self.in_ph_end_idx = in_ph_end_idx
        self.num_vocab = in_ph_end_idx - in_ph_start_idx
        self.embed_dim = embed_dim
        self.use_mdn = use_mdn
        if embed_dim is not None:
            assert in_dim > self.num_vocab
            self.emb = nn.Embedding(self.num_vocab, embed_dim)
            self.fc_in = nn.Linear(in_dim - self.num_vocab, embed_dim)
            ff_in_dim = embed_dim
        else:
            # the SeparateF0 recipe model's decoders read [encoder out, rest flag, lf0]
            ff_in_dim = in_dim
        self.ff = nn.Sequential(
            nn.Linear(ff_in_dim, ff_hidden_dim), nn.ReLU(),
            nn.Linear(ff_hidden_dim, ff_hidden_dim), nn.ReLU(),
            nn.Linear(ff_hidden_dim, ff_hidden_dim), nn.ReLU(),
        )
        self.conv = nn.Sequential(
            nn.ReflectionPad1d(3), nn.Conv1d(ff_hidden_dim, conv_hidden_dim, 7, padding=0),
            nn.BatchNorm1d(conv_hidden_dim), nn.ReLU(),
            nn.ReflectionPad1d(3), nn.Conv1d(conv_hidden_dim, conv_hidden_dim, 7, padding=0),
            nn.BatchNorm1d(conv_hidden_dim), nn.ReLU(),
            nn.ReflectionPad1d(3), nn.Conv1d(conv_hidden_dim, conv_hidden_dim, 7, padding=0),
            nn.BatchNorm1d(conv_hidden_dim), nn.ReLU(),
        )
        num_direction = 2 if bidirectional else 1
        # like the reference (model.py:862-869) the LSTM is always bidirectional
        self.lstm = nn.LSTM(conv_hidden_dim, lstm_hidden_dim, num_lstm_layers, bidirectional=True,
                            batch_first=True, dropout=dropout)
        self.fc = nn.Linear(num_direction * lstm_hidden_dim, out_dim)
        init_weights(self, init_type)
        self._packs = ModulePacks()

    def prediction_type(self):
        return PredictionType.DETERMINISTIC

    # ---- kernels -----------------------------------------------------------------
    def _register(self, pk):
        if self.embed_dim is not None:
            Ly.phoneme_input_register(pk, self.emb, self.fc_in)
        Ly.ff_register(pk, self.ff)
        Ly.conv_register(pk, self.conv)
        Ly.lstm_register(pk, self.lstm)
        pk.linear("fc", self.fc.weight)
        pk.bias_vec("fc.b", self.fc.bias)

    def _fwd(self, sources, B, T, lens_dev, spk_seq=None, spk_ld=0, training=None,
             lstm_masks=None, save=True, bn_updates=1, x16=None, after_conv=None):
        """sources: [(tensor, ld, col_offset, ncols)] of the logical input columns (without
        phoneme embedding: one (X, ldx, 0, in_dim) source is read in place); x16: an optional
        bf16 copy of that single source (rows zero-padded to a multiple of 8 columns), the
        first FF GEMM's operand and its weight gradient's; after_conv: called once the FF +
        conv stack is issued (before the recurrence; a schedule hook).
        Returns (out (B*T, out_dim), saved state)."""
        training = self.training if training is None else training
        pk = self._packs.ensure(self, self._register)
        dev = self.fc.weight.device
        if self.embed_dim is not None:
            X0, esv = Ly.embed_fwd(pk, self.emb.weight, sources, self.in_ph_start_idx,
                                   self.in_ph_end_idx, B, T, spk_seq, spk_ld, dev)
        else:
            if spk_seq is not None:
                raise NotImplementedError("FFConvLSTM(embed_dim=None) with spk_embs")
            X0, esv = _plain_input(sources, self.in_dim, B * T, dev), None
        if x16 is not None and (self.embed_dim is not None or
                                not Ly.K.bf16_operands(pk.fwd, B * T)):
            x16 = None
        hs, hs16 = Ly.ff_fwd(pk, self.ff, X0, B, T, dev, x16=x16)
        F = hs[2].shape[1]
        a, csv = Ly.conv_fwd(pk, self.conv, [("", hs[2], F, F, 0)], B, T, dev, training,
                             save=save, running_updates=bn_updates,
                             first_b16=None if hs16[2] is None else [("", hs16[2], F, F)])
        if after_conv is not None:
            after_conv()
        if training and self.lstm.dropout > 0 and lstm_masks is None:
            lstm_masks = [Ly.dropout_mask(B * T * 2 * self.lstm.hidden_size, self.lstm.dropout,
                                          dev)
                          for _ in range(self.lstm.num_layers - 1)]
        C = a.shape[1]
        y, lsv = Ly.lstm_fwd(pk, self.lstm, a, C, B, T, lens_dev, dev,
                             lstm_masks if training else None, save=save,
                             x16=csv[-1]["out16"] if csv else None)
        out = empty(B * T, self.out_dim, device=dev)
        H2 = 2 * self.lstm.hidden_size
        Ly.K.gemm([Ly.K.Seg(y, H2, H2, pk["fc"], T)], B, T, self.out_dim, pk.fwd, out,
                  self.out_dim, **pk.bias_ptr_args("fc.b"))
        st = dict(X0=X0, X16=x16, esv=esv, hs=hs, hs16=hs16, csv=csv, lsv=lsv, y=y, B=B, T=T,
                  lens=lens_dev) \
            if save else None
        return out, st

    def _bwd(self, st, dout, want_spk=False, dx_ld=None, later=None):
        """dout (B*T, out_dim).  Accumulates parameter grads; returns (dX0 per-frame input
        grad (B*T, E) -- rows of stride dx_ld when given --, dspk per-sequence (B, E) or
        None).  later (a list): the weight and bias gradients are appended to it as closures
        instead of being issued between the input-gradient launches -- the caller issues
        them once dX0 is out (the SeparateF0 decoders: the encoder's backward waits for dX0
        only)."""
        pk = self._packs
        dev = dout.device
        B, T = st["B"], st["T"]
        M = B * T
        H2 = 2 * self.lstm.hidden_size
        D = self.out_dim
        Ly.issue(later, lambda: (
            Ly.wgrad_into(self.fc.weight, dout, D, st["y"], H2, B, T, T, D, H2),
            Ly.colsum_into(dout, D, M, D, self.fc.bias, defer=True)))
        dy = empty(M, H2, device=dev)
        Ly.K.gemm([Ly.K.Seg(dout, self.out_dim, self.out_dim, pk["fc^T"], T)], B, T, H2, pk.bwd,
                  dy, H2)
        da = Ly.lstm_bwd(pk, self.lstm, st["lsv"], dy, B, T, st["lens"], dev, later=later)
        F = st["hs"][2].shape[1]
        (dh3,) = Ly.conv_bwd(pk, self.conv, st["csv"], da, B, T, dev, first_dx=[("", F)],
                             later=later)
        dX0 = Ly.ff_bwd(pk, self.ff, st["X0"], st["hs"], st["hs16"], dh3, B, T, dev,
                        x16=st.get("X16"), dx_ld=dx_ld, later=later)
        dspk = None
        if self.embed_dim is None:
            return dX0, None
        if want_spk:
            dspk = torch.zeros(B, self.embed_dim, device=dev)
        Ly.embed_bwd(self.emb, self.fc_in, st["esv"], dX0, B, T, dspk)
        return dX0, dspk

    # ---- reference API -----------------------------------------------------------
    def forward(self, x, lengths=None, y=None, spk_embs=None):
        B, T, _ = x.shape
        x = x.contiguous().float()
        return torch_ops.ffconvlstm_call(self, x, spk_embs, lengths)

    def inference(self, x, lengths=None, spk_embs=None):
        return self(x, lengths, spk_embs=spk_embs)


def _plain_input(sources, D, M, device):
    """The logical input columns as one (M, ldx) buffer (ldx = D rounded up to 4): the
    single source itself when it is already such a buffer, else a gathered copy."""
    if len(sources) == 1:
        t, ld, off, n = sources[0]
        if off == 0 and n == D and t.dim() == 2 and t.shape[1] == ld and ld % 4 == 0:
            return t
    _, X, _, _ = Ly.gather_input(sources, D, D, M, device)
    return X


def _spk_args(spk_embs, B, T):
    """Per-sequence pointer view of an (expanded) (B, T, E) speaker-embedding tensor."""
    if spk_embs is None:
        return None, 0, None
    if spk_embs.dim() == 3 and spk_embs.stride(1) == 0 and spk_embs.stride(2) == 1:
        return spk_embs, spk_embs.stride(0), None
    full = spk_embs.reshape(B * T, -1).contiguous()
    return full, full.shape[1], full




class MultiTrackLSTMEncoder(BaseModel):
    """nnsvs/model.py:1435-1537: the concatenation-fusion encoder of the SeparateF0 recipe
    model.  Each track's input becomes emb(argmax one-hot phoneme) + fc_in(other columns)
    + its speaker vector, written side by side into one (M, 2E) buffer (the reference's
    torch.concat, model.py:1527-1529), then the packed bidirectional LSTM (H = 512 in the
    recipe: the per-step recurrence kernels) and hidden2out."""

    def __init__(self, in_dim: int, hidden_dim: int, out_dim: int, num_layers: int = 1,
                 bidirectional: bool = True, dropout: float = 0.0, init_type: str = "none",
                 in_ph_start_idx: int = 1, in_ph_end_idx: int = 50, embed_dim=None):
        super().__init__()
        self.in_dim = in_dim
        self.in_ph_start_idx = in_ph_start_idx
        self.in_ph_end_idx = in_ph_end_idx
        self.num_vocab = in_ph_end_idx - in_ph_start_idx
        self.embed_dim = embed_dim
        if embed_dim is None:
            # the reference adds the speaker vectors to its caller's inputs in place
            # (model.py:1527-1528); the recipe always embeds (embed_dim 256)
            raise NotImplementedError("MultiTrackLSTMEncoder(embed_dim=None)")
        if not bidirectional:
            raise NotImplementedError("MultiTrackLSTMEncoder(bidirectional=False)")
        assert in_dim > self.num_vocab
        self.emb = nn.Embedding(self.num_vocab, embed_dim)
        self.fc_in = nn.Linear(in_dim - self.num_vocab, embed_dim)
        self.num_layers = num_layers
        self.lstm = nn.LSTM(embed_dim * 2, hidden_dim, num_layers, bidirectional=True,
                            batch_first=True, dropout=dropout)
        self.hidden2out = nn.Linear(2 * hidden_dim, out_dim)
        init_weights(self, init_type)
        self._packs = ModulePacks()

    @property
    def out_dim(self):
        return self.hidden2out.out_features

    def _register(self, pk):
        Ly.phoneme_input_register(pk, self.emb, self.fc_in)
        Ly.lstm_register(pk, self.lstm)
        pk.linear("h2o", self.hidden2out.weight)
        pk.bias_vec("h2o.b", self.hidden2out.bias)

    def _fwd(self, x_main, x_sub, D, B, T, lens_dev, spks=(None, None), spk_ld=0,
             training=None, lstm_masks=None, save=True, out=None):
        """x_main / x_sub: (B*T, D) rows (ld D); spks: per-sequence speaker vectors (B rows of
        stride spk_ld) or None; out: (buffer, ld) to write the (B*T, out_dim) output into the
        first columns of a wider buffer.  Returns (out, saved state)."""
        training = self.training if training is None else training
        pk = self._packs.ensure(self, self._register)
        dev = self.hidden2out.weight.device
        E = self.embed_dim
        X = empty(B * T, 2 * E, device=dev)
        esv = []
        for k, x in enumerate((x_main, x_sub)):
            _, sv = Ly.embed_fwd(pk, self.emb.weight, [(x, D, 0, D)], self.in_ph_start_idx,
                                 self.in_ph_end_idx, B, T, spks[k], spk_ld, dev,
                                 out=(X, 2 * E, k * E))
            esv.append(sv)
        H = self.lstm.hidden_size
        if training and self.lstm.dropout > 0 and lstm_masks is None:
            lstm_masks = [Ly.dropout_mask(B * T * 2 * H, self.lstm.dropout, dev)
                          for _ in range(self.num_layers - 1)]
        y, lsv = Ly.lstm_fwd(pk, self.lstm, X, 2 * E, B, T, lens_dev, dev,
                             lstm_masks if training else None, save=save)
        N = self.out_dim
        out, ldo = (empty(B * T, N, device=dev), N) if out is None else out
        Ly.K.gemm([Ly.K.Seg(y, 2 * H, 2 * H, pk["h2o"], T)], B, T, N, pk.fwd, out, ldo,
                  **pk.bias_ptr_args("h2o.b"))
        st = dict(X=X, esv=esv, lsv=lsv, y=y, B=B, T=T, lens=lens_dev) if save else None
        return out, st

    def _bwd(self, st, dout, ld=None, want_spk=True):
        """dout: (B*T, out_dim) rows of stride ld.  Accumulates parameter grads; returns the
        per-sequence speaker-vector grads (dspk_main, dspk_sub) (B, E) (or None) and the
        grad of the fused (B*T, 2E) LSTM input."""
        pk = self._packs
        dev = dout.device
        B, T = st["B"], st["T"]
        M = B * T
        N = self.out_dim
        ld = N if ld is None else ld
        H2 = 2 * self.lstm.hidden_size
        E = self.embed_dim
        # the output gradient rounded to bf16 once, for the weight gradient (against the last
        # recurrence's bf16 output copy) and the input-gradient GEMM, when both can take it
        y16 = st["lsv"][-1].get("y16") if st["lsv"] else None
        d16 = None
        if (y16 is not None and N % 8 == 0 and Ly.K.bf16_operands(pk.bwd, M)
                and Ly.K._castable(Ly.K.Seg(dout, ld, N, None, T))):
            d16 = Ly.K.cast_bf16(dout, ld, N, M)
        if d16 is not None:
            Ly.wgrad_into(self.hidden2out.weight, d16, N, y16, H2, B, T, T, N, H2)
        else:
            Ly.wgrad_into(self.hidden2out.weight, dout, ld, st["y"], H2, B, T, T, N, H2)
        Ly.colsum_into(dout, ld, M, N, self.hidden2out.bias, defer=True)
        dy = empty(M, H2, device=dev)
        seg = Ly.K.Seg(dout, ld, N, pk["h2o^T"], T) if d16 is None else \
            Ly.K.Seg(d16, N, N, pk["h2o^T"], T)
        Ly.K.gemm([seg], B, T, H2, pk.bwd, dy, H2)
        dX = Ly.lstm_bwd(pk, self.lstm, st["lsv"], dy, B, T, st["lens"], dev)
        dspk = [torch.zeros(B, E, device=dev) if want_spk else None for _ in range(2)]
        for k in range(2):
            Ly.embed_bwd(self.emb, self.fc_in, st["esv"][k], dX, B, T, dspk[k], ld=2 * E,
                         col=k * E)
        return dspk[0], dspk[1], dX

    # ---- reference API -----------------------------------------------------------
    def forward(self, x_main, x_sub, spk_embs, lengths, y=None):
        return torch_ops.lstm_encoder_call(self, x_main, x_sub, spk_embs[0], spk_embs[1], lengths)

