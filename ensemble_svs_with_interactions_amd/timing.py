"""Multi-track timing models on MI355X kernels.

Drop-in for nnsvs.mdn (``MDNLayer``, ``mdn_loss``, ``mdn_get_most_probable_sigma_and_mu``,
nnsvs/mdn.py:6-212), nnsvs.model.MDN (model.py:538-618; BASELINE config 1) and
nnsvs.model.MultiTrackVariancePredictor (model.py:1180-1346; the recipe's duration and
time-lag models, recipes/jaCappella_ritsu/dev-48k-world-multitrack/conf/train/
{duration,timelag}/model/multitrack_*_vp_mdn.yaml): same constructor arguments, forward /
inference signatures and state_dict keys.  Autograd runs through custom Functions whose
backward launches the HIP kernels.

  * Linear / Conv1d layers: the MFMA implicit-GEMM engine (ReLU fused in the epilogue).
  * MDN head: three GEMMs into [log_pi | log_sigma | mu], the log-softmax / loss /
    most-probable arithmetic with the mixture axis held in lane groups of one wavefront
    (xor-shuffle max and log-sum-exp, timing.hip).
  * VariancePredictor conv stack: Conv1d(k, zero pad) + ReLU (GEMM epilogue) -> channel
    LayerNorm (one wavefront per frame) -> dropout keep-mask.
"""
import torch
from torch import nn

from . import kernels as K
from . import layers as Ly
from ._lib import call
from .base import BaseModel, PredictionType
from .engine import ModulePacks, empty, grad_of
from .model import init_weights


def stream():
    return torch.cuda.current_stream().cuda_stream


def _rows(t, n):
    return t.contiguous().float().view(-1, n)


# ------------------------------------------------------------------ mdn_loss

class _MdnLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_pi, log_sigma, mu, target, log_pi_min, log_sigma_min):
        B, T, G, D = log_sigma.shape
        dw = log_pi.dim() == 4
        M = B * T
        lp = _rows(log_pi, G * D if dw else G)
        ls, m_ = _rows(log_sigma, G * D), _rows(mu, G * D)
        tg = _rows(target, D)
        loss = empty(M * D if dw else M, device=lp.device)
        call("ensvs_mdn_loss", lp.data_ptr(), ls.data_ptr(), m_.data_ptr(), tg.data_ptr(), D, M, G,
             D, int(dw), float(log_pi_min), float(log_sigma_min), loss.data_ptr(), None, None, None,
             None, stream())
        ctx.save_for_backward(lp, ls, m_, tg)
        ctx.cfg = (B, T, G, D, dw, float(log_pi_min), float(log_sigma_min), log_pi.shape)
        return loss.view(B, T, D) if dw else loss.view(B, T)

    @staticmethod
    def backward(ctx, gloss):
        lp, ls, m_, tg = ctx.saved_tensors
        B, T, G, D, dw, lpm, lsm, lp_shape = ctx.cfg
        g = gloss.contiguous().float()
        dlp, dls, dmu = torch.empty_like(lp), torch.empty_like(ls), torch.empty_like(m_)
        call("ensvs_mdn_loss", lp.data_ptr(), ls.data_ptr(), m_.data_ptr(), tg.data_ptr(), D,
             B * T, G, D, int(dw), lpm, lsm, None, g.data_ptr(), dlp.data_ptr(), dls.data_ptr(),
             dmu.data_ptr(), stream())
        return (dlp.view(lp_shape), dls.view(B, T, G, D), dmu.view(B, T, G, D), None, None, None)


class _MeanTFn(torch.autograd.Function):
    """loss.mean(dim=1) of (B, T[, D]) on the device (column sums per sequence)."""

    @staticmethod
    def forward(ctx, loss):
        B, T = loss.shape[:2]
        D = loss.shape[2] if loss.dim() == 3 else 1
        out = empty(B, D, device=loss.device)
        K.colsum(loss.contiguous(), D, T, D, out, groups=B, scale=1.0 / T)
        ctx.shape = loss.shape
        return out.view(B, D) if loss.dim() == 3 else out.view(B)

    @staticmethod
    def backward(ctx, g):
        shape = ctx.shape
        B, T = shape[:2]
        D = shape[2] if len(shape) == 3 else 1
        gs = empty(B, D, device=g.device)
        call("ensvs_axpby", gs.data_ptr(), 0.0, g.contiguous().data_ptr(), 1.0 / T, B * D,
             stream())
        out = torch.zeros(B * T, D, device=g.device)
        call("ensvs_embed_add", out.data_ptr(), D, B * T, D, T, None, None, None, gs.data_ptr(),
             None, D, stream())
        return out.view(shape)


def mdn_loss(log_pi, log_sigma, mu, target, log_pi_min=-7.0, log_sigma_min=-7.0, reduce=True):
    """nnsvs/mdn.py:78-154: negative log-likelihood of the target under the mixture
    ((B,) when reduce, else (B, T) or, dim-wise, (B, T, D))."""
    loss = _MdnLossFn.apply(log_pi, log_sigma, mu, target, log_pi_min, log_sigma_min)
    return _MeanTFn.apply(loss) if reduce else loss



class _MaskedMeanFn(torch.autograd.Function):
    """loss.masked_select(mask).mean() on the device (ensvs_masked_mean); mask broadcasts
    to the loss shape as masked_select does."""

    @staticmethod
    def forward(ctx, x, mask):
        xc = x.contiguous().float()
        m = mask.expand(x.shape).contiguous().to(torch.uint8)
        out = empty(2, device=x.device)
        part = empty(1024, device=x.device)
        call("ensvs_masked_mean", xc.data_ptr(), m.data_ptr(), xc.numel(), part.data_ptr(),
             out.data_ptr(), stream())
        ctx.save_for_backward(m, out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        m, out = ctx.saved_tensors
        dx = empty(*m.shape, device=m.device)
        call("ensvs_masked_mean_bwd", m.data_ptr(), m.numel(), g.contiguous().data_ptr(),
             out.data_ptr(), dx.data_ptr(), stream())
        return dx, None


def masked_mean(x, mask):
    return _MaskedMeanFn.apply(x, mask)


@torch.no_grad()
def mdn_get_most_probable_sigma_and_mu(log_pi, log_sigma, mu):
    """nnsvs/mdn.py:167-212 -> (sigma, mu) of the component with the largest weight."""
    B, T, G, D = log_sigma.shape
    dw = log_pi.dim() == 4
    lp = _rows(log_pi, G * D if dw else G)
    sig = empty(B, T, D, device=lp.device)
    m_ = empty(B, T, D, device=lp.device)
    call("ensvs_mdn_most_probable", lp.data_ptr(), _rows(log_sigma, G * D).data_ptr(),
         _rows(mu, G * D).data_ptr(), B * T, G, D, int(dw), sig.data_ptr(), m_.data_ptr(),
         stream())
    return sig, m_


# ------------------------------------------------------------------ MDN head

class MDNLayer(nn.Module):
    """nnsvs/mdn.py:6-75."""

    def __init__(self, in_dim, out_dim, num_gaussians=30, dim_wise=False):
        super().__init__()
        if num_gaussians > 64:
            raise ValueError("num_gaussians <= 64 (one wavefront lane group per item)")
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.num_gaussians = num_gaussians
        self.dim_wise = dim_wise
        odim_log_pi = out_dim * num_gaussians if dim_wise else num_gaussians
        self.log_pi = nn.Linear(in_dim, odim_log_pi)
        self.log_sigma = nn.Linear(in_dim, out_dim * num_gaussians)
        self.mu = nn.Linear(in_dim, out_dim * num_gaussians)
        self._packs = ModulePacks()

    @property
    def n_pi(self):
        return self.out_dim * self.num_gaussians if self.dim_wise else self.num_gaussians

    def _register(self, pk, pre=""):
        for n in ("log_pi", "log_sigma", "mu"):
            lin = getattr(self, n)
            pk.linear(pre + n, lin.weight)
            pk.bias_vec(pre + n + ".b", lin.bias)

    def _fwd(self, pk, X, ldx, Kin, B, T, pre=""):
        """Head on frame rows X (B*T, ldx) -> (log_pi, log_sigma, mu) row tensors."""
        dev = X.device
        M, G, D = B * T, self.num_gaussians, self.out_dim
        outs = []
        for n, w in (("log_pi", self.n_pi), ("log_sigma", G * D), ("mu", G * D)):
            y = empty(M, w, device=dev)
            K.gemm([K.Seg(X, ldx, Kin, pk[pre + n], T)], B, T, w, pk.fwd, y, w,
                   **pk.bias_ptr_args(pre + n + ".b"))
            outs.append(y)
        call("ensvs_mdn_log_softmax", outs[0].data_ptr(), M, G, D, int(self.dim_wise), stream())
        return outs

    def _bwd(self, pk, X, ldx, Kin, B, T, lp, grads, need_dx=True, pre=""):
        """grads: (d log_pi, d log_sigma, d mu) row tensors (None -> 0).  Returns dX."""
        dev = X.device
        M, G, D = B * T, self.num_gaussians, self.out_dim
        widths = (self.n_pi, G * D, G * D)
        gs = [torch.zeros(M, w, device=dev) if g is None else g.contiguous().float().view(M, w)
              .clone() for g, w in zip(grads, widths)]
        call("ensvs_mdn_log_softmax_bwd", lp.data_ptr(), gs[0].data_ptr(), M, G, D,
             int(self.dim_wise), stream())
        segs = []
        for n, g, w in zip(("log_pi", "log_sigma", "mu"), gs, widths):
            lin = getattr(self, n)
            Ly.wgrad_into(lin.weight, g, w, X, ldx, B, T, T, w, Kin)
            Ly.colsum_into(g, w, M, w, lin.bias)
            segs.append(K.Seg(g, w, w, pk[pre + n + "^T"], T))
        if not need_dx:
            return None
        dX = empty(M, Kin, device=dev)
        K.gemm(segs, B, T, Kin, pk.bwd, dX, Kin)
        return dX

    def _views(self, outs, B, T):
        G, D = self.num_gaussians, self.out_dim
        lp = outs[0].view(B, T, G, D) if self.dim_wise else outs[0].view(B, T, G)
        return lp, outs[1].view(B, T, G, D), outs[2].view(B, T, G, D)

    def forward(self, minibatch):
        return _MdnLayerFn.apply(self, minibatch, self.mu.weight)


class _MdnLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, anchor):
        B, T, H = x.shape
        X = x.contiguous().float().view(B * T, H)
        pk = mod._packs.ensure(mod, mod._register)
        outs = mod._fwd(pk, X, H, H, B, T)
        ctx.mod, ctx.st = mod, (X, H, B, T, outs[0])
        return mod._views(outs, B, T)

    @staticmethod
    def backward(ctx, glp, gls, gmu):
        X, H, B, T, lp = ctx.st
        mod = ctx.mod
        dX = mod._bwd(mod._packs, X, H, H, B, T, lp, (glp, gls, gmu))
        ctx.st = None
        return None, dX.view(B, T, H), None


# ------------------------------------------------------------------ MDN (config 1)

class MDN(BaseModel):
    """nnsvs/model.py:538-618: (Linear + ReLU) x num_layers + MDNLayer."""

    def __init__(self, in_dim, hidden_dim, out_dim, num_layers=1, num_gaussians=8,
                 dim_wise=False, init_type="none", **kwargs):
        super().__init__()
        model = [nn.Linear(in_dim, hidden_dim), nn.ReLU()]
        for _ in range(num_layers - 1):
            model += [nn.Linear(hidden_dim, hidden_dim), nn.ReLU()]
        model += [MDNLayer(in_dim=hidden_dim, out_dim=out_dim, num_gaussians=num_gaussians,
                           dim_wise=dim_wise)]
        self.model = nn.Sequential(*model)
        init_weights(self, init_type)
        self._packs = ModulePacks()

    def prediction_type(self):
        return PredictionType.PROBABILISTIC

    def _register(self, pk):
        for i, m in enumerate(self.model):
            if isinstance(m, nn.Linear):
                pk.linear(f"l{i}", m.weight)
                pk.bias_vec(f"l{i}.b", m.bias)
        self.model[-1]._register(pk, pre="head.")

    def forward(self, x, lengths=None, y=None):
        return _MdnModelFn.apply(self, x, self.model[0].weight)

    def inference(self, x, lengths=None):
        log_pi, log_sigma, mu = self.forward(x, lengths)
        sigma, mu = mdn_get_most_probable_sigma_and_mu(log_pi, log_sigma, mu)
        return mu, sigma


class _MdnModelFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, anchor):
        B, T, Din = x.shape
        M = B * T
        dev = x.device
        pk = mod._packs.ensure(mod, mod._register)
        h = x.contiguous().float().view(M, Din)
        hs = [h]
        for i, m in enumerate(mod.model[:-1]):
            if isinstance(m, nn.Linear):
                out = empty(M, m.out_features, device=dev)
                K.gemm([K.Seg(h, h.shape[1], h.shape[1], pk[f"l{i}"], T)], B, T, m.out_features,
                       pk.fwd, out, m.out_features, relu=True, **pk.bias_ptr_args(f"l{i}.b"))
                h = out
                hs.append(h)
        head = mod.model[-1]
        H = h.shape[1]
        outs = head._fwd(pk, h, H, H, B, T, pre="head.")
        ctx.mod, ctx.st = mod, (hs, B, T, outs[0])
        return head._views(outs, B, T)

    @staticmethod
    def backward(ctx, glp, gls, gmu):
        hs, B, T, lp = ctx.st
        mod = ctx.mod
        pk = mod._packs
        M = B * T
        head = mod.model[-1]
        H = hs[-1].shape[1]
        d = head._bwd(pk, hs[-1], H, H, B, T, lp, (glp, gls, gmu), pre="head.")
        lins = [(i, m) for i, m in enumerate(mod.model[:-1]) if isinstance(m, nn.Linear)]
        for li in reversed(range(len(lins))):
            i, m = lins[li]
            out, inp = hs[li + 1], hs[li]
            call("ensvs_relu_mask", d.data_ptr(), None, d.data_ptr(), out.data_ptr(), d.numel(), stream())
            Ly.wgrad_into(m.weight, d, m.out_features, inp, inp.shape[1], B, T, T, m.out_features,
                          m.in_features)
            Ly.colsum_into(d, m.out_features, M, m.out_features, m.bias)
            nd = empty(M, m.in_features, device=d.device)
            K.gemm([K.Seg(d, m.out_features, m.out_features, pk[f"l{i}^T"], T)], B, T,
                   m.in_features, pk.bwd, nd, m.in_features)
            d = nd
        ctx.st = None
        return None, d.view(B, T, -1), None


# ------------------------------------------------------------ VariancePredictor

class LayerNorm(nn.LayerNorm):
    """nnsvs/layers/layer_norm.py:10-35 (eps 1e-12; container, run by ensvs_layer_norm_*)."""

    def __init__(self, nout, dim=-1):
        super().__init__(nout, eps=1e-12)
        self.dim = dim


class MultiTrackVariancePredictor(BaseModel):
    """nnsvs/model.py:1180-1346: concat(x0, x1) + both speaker embeddings -> (Conv1d + ReLU +
    LayerNorm + Dropout) x num_layers -> MDN head (or Linear)."""

    def __init__(self, in_dim, out_dim, num_speaker, spk_embed_dim, num_layers=5,
                 hidden_dim=256, kernel_size=5, dropout=0.5, init_type="none", use_mdn=False,
                 num_gaussians=1, dim_wise=False, in_ph_start_idx: int = 1,
                 in_ph_end_idx: int = 50, embed_dim=None, mask_indices=None):
        super().__init__()
        if embed_dim is not None:
            raise NotImplementedError("phoneme embedding in the timing models is not in the "
                                      "multi-track recipe (embed_dim None)")
        if kernel_size % 2 != 1:
            raise NotImplementedError("odd kernel_size ('same' zero padding)")
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.use_mdn = use_mdn
        self.in_ph_start_idx = in_ph_start_idx
        self.in_ph_end_idx = in_ph_end_idx
        self.num_vocab = in_ph_end_idx - in_ph_start_idx
        self.embed_dim = embed_dim
        self.mask_indices = mask_indices
        self.kernel_size = kernel_size
        self.speaker_emb = nn.Embedding(num_speaker, spk_embed_dim)
        conv = []
        for idx in range(num_layers):
            in_channels = (in_dim + spk_embed_dim) * 2 if idx == 0 else hidden_dim
            conv += [nn.Sequential(
                nn.Conv1d(in_channels, hidden_dim, kernel_size, stride=1,
                          padding=(kernel_size - 1) // 2),
                nn.ReLU(), LayerNorm(hidden_dim, dim=1), nn.Dropout(dropout))]
        self.conv = nn.Sequential(*conv)
        if use_mdn:
            self.mdn_layer = MDNLayer(hidden_dim, out_dim, num_gaussians=num_gaussians,
                                      dim_wise=dim_wise)
        else:
            self.fc = nn.Linear(hidden_dim, out_dim)
        init_weights(self, init_type)
        self._packs = ModulePacks()

    def prediction_type(self):
        return PredictionType.PROBABILISTIC if self.use_mdn else PredictionType.DETERMINISTIC

    def _register(self, pk):
        E = self.speaker_emb.embedding_dim
        for i, blk in enumerate(self.conv):
            pk.conv(f"c{i}", blk[0].weight, bwd=i > 0)
            pk.bias_vec(f"c{i}.b", blk[0].bias)
        # input gradient of the first conv restricted to the speaker-embedding columns
        Din = 2 * self.in_dim
        pk.conv("c0@spk", self.conv[0][0].weight, cols=(Din, Din + 2 * E))
        if self.use_mdn:
            self.mdn_layer._register(pk, pre="head.")
        else:
            pk.linear("fc", self.fc.weight)
            pk.bias_vec("fc.b", self.fc.bias)

    def forward(self, x, spks, lengths=None, y=None):
        outs = _VPFn.apply(self, x, spks[0], spks[1], self.conv[0][0].weight)
        out = list(outs)
        if lengths is not None:
            out = [t[:, :lengths, ...] for t in out]
        return tuple(out)

    def inference(self, x, spks, lengths=None):
        if self.use_mdn:
            log_pi, log_sigma, mu = self(x, spks, lengths)
            sigma, mu = mdn_get_most_probable_sigma_and_mu(log_pi, log_sigma, mu)
            return mu, sigma
        # the reference calls self(x, lengths) here (model.py:1346), passing lengths as spks
        return self(x, spks, lengths)


class _VPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, s0, s1, anchor):
        B, T, Din = x.shape
        M = B * T
        dev = x.device
        pk = mod._packs.ensure(mod, mod._register)
        E = mod.speaker_emb.embedding_dim
        Cin = Din + 2 * E
        ldx = (Cin + 3) // 4 * 4
        X = torch.zeros(M, ldx, device=dev)
        xin = x.contiguous().float()
        call("ensvs_copy_cols", xin.data_ptr(), Din, X.data_ptr(), ldx, M, Din, stream())
        zcol = torch.zeros(M, device=dev)
        for idx in (mod.mask_indices or []):  # x[:, :, idx] *= 0 (model.py:1291-1293)
            call("ensvs_copy_cols", zcol.data_ptr(), 1, X.data_ptr() + 4 * idx, ldx, M, 1,
                 stream())
        table = mod.speaker_emb.weight
        ids = []
        for k, s in enumerate((s0, s1)):
            idx = s.reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
            v = empty(B, E, device=dev)
            call("ensvs_gather_rows", table.data_ptr(), idx.data_ptr(), B, E, v.data_ptr(),
                 stream())
            call("ensvs_embed_add", X.data_ptr() + 4 * (Din + k * E), ldx, M, E, T, None, None,
                 None, v.data_ptr(), None, E, stream())
            ids.append(idx)
        k_ = mod.kernel_size
        sh = -(k_ - 1) // 2
        training = mod.training
        replay = getattr(mod, "_replay_masks", None)
        h, ldh, Kin = X, ldx, Cin
        sv = []
        for i, blk in enumerate(mod.conv):
            conv, ln, drop = blk[0], blk[2], blk[3]
            H = conv.out_channels
            yc = empty(M, H, device=dev)
            K.gemm([K.Seg(h, ldh, Kin, pk[f"c{i}"], T, taps=k_, shift0=sh)], B, T, H, pk.fwd,
                   yc, H, relu=True, **pk.bias_ptr_args(f"c{i}.b"))
            yl = empty(M, H, device=dev)
            mean, rstd = empty(M, device=dev), empty(M, device=dev)
            call("ensvs_layer_norm_fwd", yc.data_ptr(), H, M, H, ln.weight.data_ptr(),
                 ln.bias.data_ptr(), float(ln.eps), yl.data_ptr(), H, mean.data_ptr(),
                 rstd.data_ptr(), stream())
            mask = None
            out = yl
            if training and drop.p > 0:
                mask = replay[i] if replay is not None else Ly.dropout_mask(M * H, drop.p, dev)
                out = empty(M, H, device=dev)
                call("ensvs_mul_out", out.data_ptr(), yl.data_ptr(), mask.data_ptr(), M * H,
                     stream())
            sv.append((h, ldh, Kin, yc, mean, rstd, mask))
            h, ldh, Kin = out, H, H
        if mod.use_mdn:
            head = mod.mdn_layer
            outs = head._fwd(pk, h, ldh, Kin, B, T, pre="head.")
            res = head._views(outs, B, T)
            lp = outs[0]
        else:
            o = empty(M, mod.out_dim, device=dev)
            K.gemm([K.Seg(h, ldh, Kin, pk["fc"], T)], B, T, mod.out_dim, pk.fwd, o, mod.out_dim,
                   **pk.bias_ptr_args("fc.b"))
            res, lp = (o.view(B, T, -1),), None
        ctx.mod = mod
        ctx.st = dict(sv=sv, h=h, B=B, T=T, ids=ids, Din=Din, E=E, lp=lp)
        return res

    @staticmethod
    def backward(ctx, *grads):
        mod, st = ctx.mod, ctx.st
        pk = mod._packs
        B, T, E, Din = st["B"], st["T"], st["E"], st["Din"]
        M = B * T
        h = st["h"]
        H = h.shape[1]
        dev = h.device
        if mod.use_mdn:
            d = mod.mdn_layer._bwd(pk, h, H, H, B, T, st["lp"], grads, pre="head.")
        else:
            g = grads[0].contiguous().float().view(M, mod.out_dim)
            Ly.wgrad_into(mod.fc.weight, g, mod.out_dim, h, H, B, T, T, mod.out_dim, H)
            Ly.colsum_into(g, mod.out_dim, M, mod.out_dim, mod.fc.bias)
            d = empty(M, H, device=dev)
            K.gemm([K.Seg(g, mod.out_dim, mod.out_dim, pk["fc^T"], T)], B, T, H, pk.bwd, d, H)
        k_ = mod.kernel_size
        sh = -(k_ - 1) // 2
        for i in reversed(range(len(mod.conv))):
            conv, ln = mod.conv[i][0], mod.conv[i][2]
            hin, ldh, Kin, yc, mean, rstd, mask = st["sv"][i]
            if mask is not None:
                call("ensvs_mul", d.data_ptr(), mask.data_ptr(), M * H, stream())
            dyc = empty(M, H, device=dev)
            dyx = empty(M, H, device=dev)
            call("ensvs_layer_norm_bwd", d.data_ptr(), H, yc.data_ptr(), H, M, H,
                 ln.weight.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dyc.data_ptr(), H,
                 dyx.data_ptr(), stream())
            Ly.colsum_into(dyx, H, M, H, ln.weight)
            Ly.colsum_into(d, H, M, H, ln.bias)
            call("ensvs_relu_mask", dyc.data_ptr(), None, dyc.data_ptr(), yc.data_ptr(), M * H, stream())
            Ly.colsum_into(dyc, H, M, H, conv.bias)
            Ly.wgrad_into(conv.weight, dyc, H, hin, ldh, B, T, T, H, Kin, taps=k_, shift0=sh)
            if i > 0:
                nd = empty(M, Kin, device=dev)
                K.gemm([K.Seg(dyc, H, H, pk[f"c{i}^T"], T, taps=k_, shift0=sh)], B, T, Kin,
                       pk.bwd, nd, Kin)
                d = nd
            else:  # speaker-embedding columns only: per-sequence sums -> table rows
                dsp = empty(M, 2 * E, device=dev)
                K.gemm([K.Seg(dyc, H, H, pk["c0@spk^T"], T, taps=k_, shift0=sh)], B, T, 2 * E,
                       pk.bwd, dsp, 2 * E)
                dseq = empty(B, 2 * E, device=dev)
                K.colsum(dsp, 2 * E, T, 2 * E, dseq, groups=B)
                table = grad_of(mod.speaker_emb.weight)
                dk = empty(B, E, device=dev)
                for k, idx in enumerate(st["ids"]):
                    call("ensvs_copy_cols", dseq.data_ptr() + 4 * k * E, 2 * E, dk.data_ptr(), E,
                         B, E, stream())
                    call("ensvs_spk_scatter", dk.data_ptr(), B, E, idx.data_ptr(),
                         table.data_ptr(), stream())
        ctx.st = None
        return None, None, None, None, None


def timing_train_step(model, optimizer, x0, x1, y, spk0, spk1, mask, train=True):
    """train_step of bin/train_multitrack.py:46-154 for the recipe's MDN timing models
    (MultiTrackVariancePredictor with use_mdn; duration or time-lag): forward on
    concat(x0, x1) with both tracks' speakers, mdn_loss(reduce=False) masked by the collate's
    note mask (mask_list[0], (B, T, 1) bool; squeezed unless the MDN is dim-wise) and
    averaged, backward and one Adam step.  The reference's live pdb.set_trace()
    (App. A-11) is not reproduced; its AMP grad scaler is not used (fp32); it clips
    nothing, so pass an optimizer built with clip_norm=float("inf").  FusedAdam skips a
    non-finite step where torch.optim.Adam would apply it.  Returns the loss (device)."""
    if not getattr(model, "use_mdn", True):
        raise NotImplementedError("timing_train_step: the recipe's timing models are MDN models")
    model.train() if train else model.eval()
    optimizer.zero_grad()
    x = torch.cat((x0, x1), dim=2)
    lp, ls, mu = model(x, (spk0, spk1))
    mask_ = mask if lp.dim() == 4 else mask.squeeze(-1)
    loss = masked_mean(mdn_loss(lp, ls, mu, y, reduce=False), mask_)
    if train:
        loss.backward()
        optimizer.step()
    return loss.detach()
