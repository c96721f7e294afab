"""uSFGAN vocoder generator on MI355X kernels (synthesis path).

Drop-in for nnsvs.usfgan.models.ParallelHnUSFGANGenerator
(nnsvs/usfgan/models/generator.py:359-544) and nnsvs.usfgan.USFGANWrapper
(nnsvs/usfgan/__init__.py:7-65): same constructor arguments and ``state_dict`` keys
(``weight_g``/``weight_v`` while weight norm is on), ``forward(x, c, d) -> (x, s, h, n, a)``,
``remove_weight_norm()`` and ``USFGANWrapper(config, generator).inference(f0, aux)``.

Every convolution is one launch of the MFMA implicit-GEMM engine (gemm.hip):
  * AdaptiveBlock (residual_block.py:198-234): ONE GEMM whose first K-segment is a 3-tap
    "convolution" over [x(past) | x | x(future)] -- the pitch-dependent taps are gathered in
    the operand staging with the reference's float32 index arithmetic (usfgan/utils/index.py
    :27-54, nothing materialised) -- and whose second K-segment is the 1x1 aux conditioning;
    tanh(xa) * sigmoid(xb) in the epilogue (EPI_GATE_TS).  Then the 1x1 output conv with
    (out + x) * sqrt(1/2) fused and written in place (EPI_ADDSCALE).
  * FixedBlock (:123-157): the same two GEMMs with a reflect-padded dilated 3-tap segment.
  * The skip convolutions are never run: ResidualBlocks discards them (:323-336).
Weight norm is folded on the device (ensvs_weight_norm) into GEMM operands once per
parameter version.  The nn.Conv modules are parameter containers; their forward is never
called.
"""
import math

import numpy as np
import torch
from torch import nn

from . import _lib
from . import kernels as K
from ._lib import call
from .engine import _sig, empty, gemm_dtype, next_seed
from .kernels import PackedBuffer

SQRT1_2 = math.sqrt(0.5)
_PAD = {"zeros": _lib.PAD_ZERO, "reflect": _lib.PAD_REFLECT, "replicate": _lib.PAD_REPLICATE}


def stream():
    return torch.cuda.current_stream().cuda_stream


# ------------------------------------------------------------ parameter containers

class Conv1d(nn.Conv1d):
    """usfgan/layers/residual_block.py:27-38 (kaiming-normal weights, zero bias)."""

    def reset_parameters(self):
        nn.init.kaiming_normal_(self.weight, nonlinearity="relu")
        if self.bias is not None:
            nn.init.constant_(self.bias, 0.0)


class Conv1d1x1(Conv1d):
    def __init__(self, in_channels, out_channels, bias=True):
        super().__init__(in_channels, out_channels, kernel_size=1, padding=0, dilation=1,
                         bias=bias)


class Conv2d(nn.Conv2d):
    """usfgan/layers/upsample.py:47-58 (weights 1 / prod(kernel_size))."""

    def reset_parameters(self):
        self.weight.data.fill_(1.0 / np.prod(self.kernel_size))
        if self.bias is not None:
            nn.init.constant_(self.bias, 0.0)


class Stretch2d(nn.Module):
    """upsample.py:15-44 (nearest stretch along time; no parameters)."""

    def __init__(self, x_scale, y_scale, mode="nearest"):
        super().__init__()
        self.x_scale, self.y_scale, self.mode = x_scale, y_scale, mode


class UpsampleNetwork(nn.Module):
    """upsample.py:61-128: per scale, Stretch2d(s, 1) + Conv2d(1, 1, (1, 2s+1))."""

    def __init__(self, upsample_scales, nonlinear_activation=None,
                 nonlinear_activation_params={}, interpolate_mode="nearest",
                 freq_axis_kernel_size=1, use_causal_conv=False):
        super().__init__()
        if nonlinear_activation is not None or interpolate_mode != "nearest" or \
                freq_axis_kernel_size != 1 or use_causal_conv:
            raise NotImplementedError("the recipe upsampler: nearest, no activation, "
                                      "freq kernel 1, non-causal")
        self.upsample_scales = list(upsample_scales)
        self.up_layers = nn.ModuleList()
        for s in upsample_scales:
            self.up_layers += [Stretch2d(s, 1),
                               Conv2d(1, 1, kernel_size=(1, 2 * s + 1), padding=(0, s),
                                      bias=False)]


class ConvInUpsampleNetwork(nn.Module):
    """upsample.py:131-194."""

    def __init__(self, upsample_scales, nonlinear_activation=None,
                 nonlinear_activation_params={}, interpolate_mode="nearest",
                 freq_axis_kernel_size=1, aux_channels=80, aux_context_window=0,
                 use_causal_conv=False):
        super().__init__()
        if use_causal_conv:
            raise NotImplementedError("causal upsampling is not in the recipe")
        self.aux_context_window = aux_context_window
        self.conv_in = Conv1d(aux_channels, aux_channels, kernel_size=2 * aux_context_window + 1,
                              bias=False)
        self.upsample = UpsampleNetwork(upsample_scales, nonlinear_activation,
                                        nonlinear_activation_params, interpolate_mode,
                                        freq_axis_kernel_size, use_causal_conv)


class FixedBlock(nn.Module):
    """residual_block.py:75-157."""

    def __init__(self, residual_channels=64, gate_channels=128, skip_channels=64,
                 aux_channels=80, kernel_size=3, dilation=1, bias=True):
        super().__init__()
        if kernel_size != 3:
            raise NotImplementedError("FixedBlock kernel_size 3 (recipe)")
        self.dilation = dilation
        self.conv = Conv1d(residual_channels, gate_channels, kernel_size,
                           padding=(kernel_size - 1) // 2 * dilation, padding_mode="reflect",
                           dilation=dilation, bias=bias)
        self.conv1x1_aux = Conv1d1x1(aux_channels, gate_channels, bias=False) \
            if aux_channels > 0 else None
        self.conv1x1_out = Conv1d1x1(gate_channels // 2, residual_channels, bias=bias)
        self.conv1x1_skip = Conv1d1x1(gate_channels // 2, skip_channels, bias=bias)


class AdaptiveBlock(nn.Module):
    """residual_block.py:160-234."""

    def __init__(self, residual_channels=64, gate_channels=128, skip_channels=64,
                 aux_channels=80, bias=True):
        super().__init__()
        self.convP = Conv1d1x1(residual_channels, gate_channels, bias=bias)
        self.convC = Conv1d1x1(residual_channels, gate_channels, bias=bias)
        self.convF = Conv1d1x1(residual_channels, gate_channels, bias=bias)
        self.conv1x1_aux = Conv1d1x1(aux_channels, gate_channels, bias=False) \
            if aux_channels > 0 else None
        self.conv1x1_out = Conv1d1x1(gate_channels // 2, residual_channels, bias=bias)
        self.conv1x1_skip = Conv1d1x1(gate_channels // 2, skip_channels, bias=bias)


class ResidualBlocks(nn.Module):
    """residual_block.py:237-336 (cascade_mode 0: adaptive -> fixed, 1: fixed -> adaptive)."""

    def __init__(self, blockA, cycleA, blockF, cycleF, cascade_mode=0, residual_channels=64,
                 gate_channels=128, skip_channels=64, aux_channels=80):
        super().__init__()
        cycleA, cycleF = max(cycleA, 1), max(cycleF, 1)
        assert blockA % cycleA == 0 and blockF % cycleF == 0
        self.blockA_per_cycle = blockA // cycleA
        fpc = blockF // cycleF
        kw = dict(residual_channels=residual_channels, gate_channels=gate_channels,
                  skip_channels=skip_channels, aux_channels=aux_channels)
        adaptive = [AdaptiveBlock(**kw) for _ in range(blockA)]
        fixed = [FixedBlock(dilation=2 ** (b % fpc), **kw) for b in range(blockF)]
        if cascade_mode == 0:
            blocks, modes = adaptive + fixed, [True] * blockA + [False] * blockF
        elif cascade_mode == 1:
            blocks, modes = fixed + adaptive, [False] * blockF + [True] * blockA
        else:
            raise ValueError(f"Cascaded mode {cascade_mode} is not supported!")
        self.conv_dilated = nn.ModuleList(blocks)
        self.block_modes = modes
        # per block: pitch-dependent dilation (adaptive, :327) or fixed dilation
        dil, ia = [], 0
        for blk, mode in zip(blocks, modes):
            if mode:
                dil.append(2 ** (ia % self.blockA_per_cycle))
                ia += 1
            else:
                dil.append(blk.dilation)
        self.dilations = dil


class PeriodicityEstimator(nn.Module):
    """residual_block.py:339-399: convs with ReLU between and a sigmoid last."""

    def __init__(self, in_channels, residual_channels=64, conv_layers=3, kernel_size=5,
                 dilation=1, padding_mode="replicate"):
        super().__init__()
        self.padding_mode = padding_mode
        mods = []
        for idx in range(conv_layers):
            conv = Conv1d(in_channels, residual_channels, kernel_size=kernel_size,
                          dilation=dilation, padding=kernel_size // 2 * dilation,
                          padding_mode=padding_mode)
            if idx != conv_layers - 1:
                act = nn.ReLU(inplace=True)
            else:
                nn.init.normal_(conv.weight, std=1e-4)
                act = nn.Sigmoid()
            mods += [conv, act]
            in_channels = residual_channels
        self.layers = nn.Sequential(*mods)


# ------------------------------------------------------------ effective weights

def _wv(m):
    """(g or None, v) of a conv module: weight-normed (weight_g, weight_v) or plain weight."""
    p = m._parameters
    if "weight_g" in p:
        return p["weight_g"], p["weight_v"]
    return None, p["weight"]


class _Prepared:
    """Weight-norm-folded weights of every conv (one flat fp32 buffer written by
    ensvs_weight_norm) and their packed GEMM operands (one pack launch)."""

    def __init__(self, gen, dev):
        self.jobs, self.size = [], 0
        self.fwd = PackedBuffer(gemm_dtype())
        self.bias_buf = PackedBuffer(_lib.DT_F32)
        self.ref, self.bref = {}, {}
        self.fir = []
        plan = []  # deferred pack registrations (need the flat buffer)
        Gh = gen.gate_channels // 2

        def weight(m, off=None, sn=None, sk=None):
            g, v = _wv(m)
            N, Kf = v.shape[0], v[0].numel()
            if off is None:
                off = self._alloc(v.numel())
                sn, sk = Kf, 1
            self.jobs.append(("w", g, v, N, Kf, off, sn, sk))
            return off

        def bias(bs, scale=1.0):
            off = self._alloc(bs[0].numel())
            self.jobs.append(("b", bs, off))
            return off

        def conv(name, m, perm_c=0, scale=1.0, with_bias=True):
            N, Kc, taps = m.weight_shape
            off = weight(m)
            plan.append(("w", name, off, N, Kc, taps, perm_c, scale))
            if with_bias and m.bias is not None:
                plan.append(("b", name, bias([m.bias]), N, perm_c, scale))

        for mod in gen.modules():  # shapes of weight-normed convs (weight is derived)
            if isinstance(mod, (nn.Conv1d, nn.Conv2d)):
                _, v = _wv(mod)
                mod.weight_shape = (v.shape[0], v.shape[1], int(np.prod(v.shape[2:])))

        conv("first_sine", gen.conv_first_sine)
        conv("first_noise", gen.conv_first_noise)
        conv("conv_in", gen.upsample_net.conv_in)
        for m in gen.upsample_net.upsample.up_layers:
            if isinstance(m, nn.Conv2d):
                self.fir.append(weight(m))
        for i, m in enumerate(gen._pe_convs()):
            conv(f"pe{i}", m)
        for net in ("harmonic_network", "noise_network", "filter_network"):
            for i, (blk, mode) in enumerate(zip(getattr(gen, net).conv_dilated,
                                                getattr(gen, net).block_modes)):
                key = f"{net}.{i}"
                R = blk.conv1x1_out.weight_shape[0]
                if mode:  # [past | current | future] as the 3 taps of one weight
                    off = self._alloc(2 * Gh * R * 3)
                    for j, m in enumerate((blk.convP, blk.convC, blk.convF)):
                        weight(m, off + j, 3 * R, 3)
                    plan.append(("w", key + ".g", off, 2 * Gh, R, 3, Gh, 1.0))
                    plan.append(("b", key + ".g", bias([blk.convP.bias, blk.convC.bias,
                                                        blk.convF.bias]), 2 * Gh, Gh, 1.0))
                else:
                    conv(key + ".g", blk.conv, perm_c=Gh)
                conv(key + ".aux", blk.conv1x1_aux, perm_c=Gh)
                conv(key + ".out", blk.conv1x1_out, scale=SQRT1_2)
        conv("last1", gen.conv_last[1])
        conv("last3", gen.conv_last[3])

        self.buf = torch.empty(max(self.size, 64), device=dev)
        for item in plan:
            if item[0] == "w":
                _, name, off, N, Kc, taps, perm_c, scale = item
                src = self.buf[off:off + N * Kc * taps].view(N, Kc, taps)
                self.ref[name] = self.fwd.add(src, N, Kc, taps, Kc * taps, taps, 1,
                                              perm_c=perm_c, scale=scale)
            else:
                _, name, off, N, perm_c, scale = item
                src = self.buf[off:off + N].view(N, 1, 1)
                self.bref[name] = self.bias_buf.add(src, N, 1, 1, 1, 1, 1, perm_c=perm_c,
                                                    scale=scale, kpad_to=1)
        for pb in (self.fwd, self.bias_buf):
            pb.finalize(dev)
        self.refresh()

    def _alloc(self, n):
        off = self.size
        self.size += (n + 63) // 64 * 64
        return off

    def refresh(self):
        """Re-fold the weights and repack (after the parameters changed)."""
        base = self.buf.data_ptr()
        for j in self.jobs:
            if j[0] == "w":
                _, g, v, N, Kf, off, sn, sk = j
                call("ensvs_weight_norm", None if g is None else g.data_ptr(), v.data_ptr(), N,
                     Kf, base + 4 * off, sn, sk, stream())
            else:
                _, bs, off = j
                N = bs[0].numel()
                call("ensvs_weight_norm", None, bs[0].data_ptr(), N, 1, base + 4 * off, 1, 0,
                     stream())
                for b in bs[1:]:
                    call("ensvs_axpy", base + 4 * off, b.data_ptr(), 1.0, N, stream())
        for pb in (self.fwd, self.bias_buf):
            pb.repack()

    def bias(self, name):
        r = self.bref.get(name)
        if r is None:
            return {}
        return dict(bias=self.bias_buf.buf, bias_off=r.offset)

    def fir_taps(self, i):
        return self.buf[self.fir[i]:]


# ------------------------------------------------------------------ generator

# inference blocks as one launch each (ensvs_usf_block; off: two GEMMs, the bitwise tests)
FUSED_BLOCK = {"on": True}


class ParallelHnUSFGANGenerator(nn.Module):
    """usfgan/models/generator.py:359-544."""

    def __init__(self, harmonic_network_params={"blockA": 20, "cycleA": 4, "blockF": 0,
                                                 "cycleF": 0, "cascade_mode": 0},
                 noise_network_params={"blockA": 0, "cycleA": 0, "blockF": 5, "cycleF": 5,
                                       "cascade_mode": 0},
                 filter_network_params={"blockA": 0, "cycleA": 0, "blockF": 30, "cycleF": 3,
                                        "cascade_mode": 0},
                 periodicity_estimator_params={"conv_blocks": 3, "kernel_size": 5,
                                               "dilation": 1, "padding_mode": "replicate"},
                 in_channels=1, out_channels=1, residual_channels=64, gate_channels=128,
                 skip_channels=64, aux_channels=80, aux_context_window=2, use_weight_norm=True,
                 upsample_params={"upsample_scales": [5, 4, 3, 2]}):
        super().__init__()
        if in_channels != 1 or out_channels != 1:
            raise NotImplementedError("in_channels / out_channels 1 (recipe)")
        if (gate_channels // 2) % 16 != 0:
            raise ValueError("gate_channels / 2 must be a multiple of 16 (MFMA gate interleave)")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.aux_channels = aux_channels
        self.n_ch = residual_channels
        self.gate_channels = gate_channels
        self.aux_context_window = aux_context_window
        self.conv_first_sine = Conv1d1x1(in_channels, residual_channels)
        self.conv_first_noise = Conv1d1x1(in_channels, residual_channels)
        self.upsample_net = ConvInUpsampleNetwork(**upsample_params, aux_channels=aux_channels,
                                                  aux_context_window=aux_context_window)
        nets = []
        for params in (harmonic_network_params, noise_network_params, filter_network_params):
            p = dict(params)
            p.update(residual_channels=residual_channels, gate_channels=gate_channels,
                     skip_channels=skip_channels, aux_channels=aux_channels)
            nets.append(ResidualBlocks(**p))
        self.harmonic_network, self.noise_network, self.filter_network = nets
        pe = dict(periodicity_estimator_params)
        pe.pop("conv_blocks", None)  # the reference default dict names an unused key
        self.periodicity_estimator = PeriodicityEstimator(**pe, in_channels=aux_channels)
        self.conv_last = nn.Sequential(nn.ReLU(), Conv1d1x1(skip_channels, skip_channels),
                                       nn.ReLU(), Conv1d1x1(skip_channels, out_channels))
        if use_weight_norm:
            self.apply_weight_norm()
        self._prep = None

    def _pe_convs(self):
        return [m for m in self.periodicity_estimator.layers if isinstance(m, nn.Conv1d)]

    # ---- weight norm (parameter registration as the reference) ---------------------
    def apply_weight_norm(self):
        """generator.py:536-544: weight_g / weight_v parameters on every Conv1d/Conv2d."""
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for m in self.modules():
                if isinstance(m, (nn.Conv1d, nn.Conv2d)):
                    nn.utils.weight_norm(m)

    def remove_weight_norm(self):
        """generator.py:524-534: fold g * v / ||v|| into a plain ``weight`` (on the device,
        ensvs_weight_norm) and drop the weight-norm parametrisation."""
        from torch.nn.utils.weight_norm import WeightNorm
        for m in self.modules():
            if not isinstance(m, (nn.Conv1d, nn.Conv2d)) or "weight_g" not in m._parameters:
                continue
            g, v = m.weight_g, m.weight_v
            if not v.is_cuda:
                raise RuntimeError("ensvs: remove_weight_norm folds on the GPU (no CPU "
                                   "fallback); move the generator to the device first")
            w = torch.empty_like(v)
            call("ensvs_weight_norm", g.data_ptr(), v.data_ptr(), v.shape[0], v[0].numel(),
                 w.data_ptr(), v[0].numel(), 1, stream())
            for k, hook in list(m._forward_pre_hooks.items()):
                if isinstance(hook, WeightNorm) and hook.name == "weight":
                    del m._forward_pre_hooks[k]
            del m._parameters["weight_g"]
            del m._parameters["weight_v"]
            if "weight" in m.__dict__:
                del m.__dict__["weight"]
            m.weight = nn.Parameter(w)
        self._prep = None

    def _prepare(self):
        params = list(self.parameters())
        sig = _sig(params)
        if self._prep is not None and self._prep[0] == sig:
            return self._prep[1]
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError("ensvs: the uSFGAN kernels need the generator on a GPU "
                               "(no CPU fallback)")
        layout = (sig[1], tuple(p.data_ptr() for p in params))
        if self._prep is not None and self._prep[2] == layout:
            prep = self._prep[1]  # same storage and precision: re-fold + repack only
            prep.refresh()
        else:
            prep = _Prepared(self, dev)
        self._prep = (sig, prep, layout)
        return prep

    # ---- kernels ------------------------------------------------------------------
    def _blocks(self, P, name, x, c, ldc, d, B, L, z, relu_last=False, xb=None, cb=None,
                zb=None):
        """The network's residual blocks on x in place.  bf16 operands (xb, cb, zb given): the
        blocks read x's bf16 copy xb (kept current by each output GEMM's epilogue), the
        auxiliary features' zero-padded bf16 copy cb and z's bf16 copy zb -- the rounding
        the register-staged kernel applies while staging, so the same bits, without an fp32
        z round trip or an fp32 re-read of the features per block."""
        net = getattr(self, name)
        R, Gh, Ca = self.n_ch, self.gate_channels // 2, self.aux_channels
        nb = len(net.conv_dilated)
        xs = x if xb is None else xb
        for i, (mode, dil) in enumerate(zip(net.block_modes, net.dilations)):
            key = f"{name}.{i}"
            if mode:
                seg0 = K.Seg(xs, R, R, P.ref[key + ".g"], L, taps=3, pd=d, pd_dil=dil)
            else:
                if dil >= L:
                    raise ValueError(f"reflect padding {dil} needs more than {dil} samples")
                seg0 = K.Seg(xs, R, R, P.ref[key + ".g"], L, taps=3, dil=dil, shift0=-dil,
                             pad=_lib.PAD_REFLECT)
            seg1 = (K.Seg(c, ldc, ldc, P.ref[key + ".aux"], L) if cb is None else
                    K.Seg(cb, cb.shape[1], Ca, P.ref[key + ".aux"], L))
            r2 = P.ref[key + ".out"]
            if zb is not None and FUSED_BLOCK["on"] and Gh == 64 and R == 64 and r2.Kp == 64:
                # the whole block in one launch, z kept on chip (ensvs_usf_block)
                b1, b2 = P.bias(key + ".g"), P.bias(key + ".out")
                K.usf_block([seg0, seg1], B, L, P.fwd, Gh, r2, x, R, SQRT1_2,
                            relu=relu_last and i == nb - 1, xb=xb,
                            bias=b1.get("bias"), bias_off=b1.get("bias_off", 0),
                            bias2=b2.get("bias"), bias2_off=b2.get("bias_off", 0))
                continue
            K.gemm([seg0, seg1], B, L, 2 * Gh, P.fwd, z, Gh, epi=_lib.EPI_GATE_TS, C=Gh,
                   ybf=zb, ybf_ld=Gh, keep_y=zb is None, **P.bias(key + ".g"))
            K.gemm([K.Seg(z, Gh, Gh, P.ref[key + ".out"], L) if zb is None else
                    K.Seg(zb, Gh, Gh, P.ref[key + ".out"], L)], B, L, R, P.fwd, x, R,
                   epi=_lib.EPI_ADDSCALE, aux1=x, ld1=R, alpha=SQRT1_2,
                   relu=relu_last and i == nb - 1, ybf=xb, ybf_ld=R, **P.bias(key + ".out"))

    def _conv_last(self, P, xr, B, L, dev):
        """conv_last on an already ReLU'd input (generator.py:461-466); xr fp32 or its bf16
        copy."""
        R = self.n_ch
        t = empty(B * L, R, device=dev)
        K.gemm([K.Seg(xr, R, R, P.ref["last1"], L)], B, L, R, P.fwd, t, R, relu=True,
               **P.bias("last1"))
        y = empty(B * L, device=dev)
        K.gemm([K.Seg(t, R, R, P.ref["last3"], L)], B, L, 1, P.fwd, y, 1, **P.bias("last3"))
        return y

    def _run(self, xsrc, csrc, c_ld, Tin, c_shift, c_pad, T, d, B, keep=False):
        """xsrc (B*L, 2) [sine, noise]; csrc (B*Tin, c_ld) aux frames, conv_in reads frame
        t + c_shift + k (k < 2w+1) under padding c_pad; d (B*L,) dilation factors.
        Returns y (B*L,), or (y, s, h, n, a) raw tensors when keep."""
        P = self._prepare()
        dev = xsrc.device
        up = self.upsample_net
        scales = up.upsample.upsample_scales
        L = T * int(np.prod(scales))
        M = B * L
        R, Gh, Ca = self.n_ch, self.gate_channels // 2, self.aux_channels
        ldc = (Ca + 3) // 4 * 4
        kw = 2 * self.aux_context_window + 1
        c = empty(B * T, ldc, device=dev)
        K.gemm([K.Seg(csrc, c_ld, Ca, P.ref["conv_in"], Tin, taps=kw, shift0=c_shift,
                      pad=c_pad)], B, T, Ca, P.fwd, c, ldc)
        Tc = T
        for i, s in enumerate(scales):
            nxt = empty(B * Tc * s, ldc, device=dev)
            call("ensvs_usf_upsample", c.data_ptr(), ldc, B, Tc, Ca, s, float(1.0 / s),
                 P.fir_taps(i).data_ptr(), nxt.data_ptr(), stream())
            c, Tc = nxt, Tc * s
        # inference with bf16 operands: the residual streams' bf16 copies ride along in the
        # epilogues, the auxiliary features are rounded once (zero K padding) for all blocks
        # and the periodicity estimator
        b16 = not keep and K.bf16_operands(P.fwd, M)
        hb = nb_ = cb = zb = None
        if b16:
            hb = empty(M, R, device=dev, dtype=torch.bfloat16)
            nb_ = empty(M, R, device=dev, dtype=torch.bfloat16)
            zb = empty(M, Gh, device=dev, dtype=torch.bfloat16)
            cb = empty(M, -(-Ca // 8) * 8, device=dev, dtype=torch.bfloat16)
            K.cast_bf16(c, ldc, Ca, M, out=cb, out_ld=cb.shape[1])
        # periodicity estimator (ReLU, ReLU, sigmoid); bf16: each conv's epilogue writes the
        # next one's operand copy
        pe = self._pe_convs()
        pad = _PAD[self.periodicity_estimator.padding_mode]
        a, lda, Kin = (c, ldc, ldc) if cb is None else (cb, cb.shape[1], Ca)
        for i, m in enumerate(pe):
            k, dl = m.kernel_size[0], m.dilation[0]
            out = empty(M, R, device=dev)
            last = i == len(pe) - 1
            ob = empty(M, R, device=dev, dtype=torch.bfloat16) if b16 and not last else None
            K.gemm([K.Seg(a, lda, Kin, P.ref[f"pe{i}"], L, taps=k, dil=dl,
                          shift0=-(k // 2) * dl, pad=pad)], B, L, R, P.fwd, out, R,
                   relu=_lib.ACT_SIGMOID if last else _lib.ACT_RELU, ybf=ob, ybf_ld=R,
                   **P.bias(f"pe{i}"))
            a, lda, Kin = (out, R, R) if ob is None else (ob, R, R)
        a = out
        h = empty(M, R, device=dev)
        n = empty(M, R, device=dev)
        K.gemm([K.Seg(xsrc, 2, 1, P.ref["first_sine"], L)], B, L, R, P.fwd, h, R,
               ybf=hb, ybf_ld=R, **P.bias("first_sine"))
        K.gemm([K.Seg(xsrc, 2, 1, P.ref["first_noise"], L, xoff=1)], B, L, R, P.fwd, n, R,
               ybf=nb_, ybf_ld=R, **P.bias("first_noise"))
        z = empty(M, Gh, device=dev)
        self._blocks(P, "harmonic_network", h, c, ldc, d, B, L, z, xb=hb, cb=cb, zb=zb)
        self._blocks(P, "noise_network", n, c, ldc, d, B, L, z, xb=nb_, cb=cb, zb=zb)
        s = empty(M, R, device=dev)
        call("ensvs_usf_mix", a.data_ptr(), h.data_ptr(), n.data_ptr(), s.data_ptr(), M * R,
             int(keep), stream())
        if not keep:
            # inference: the filter runs in place on s, its last block emits ReLU(x) for
            # conv_last
            sb = K.cast_bf16(s, R, R, M) if b16 else None
            self._blocks(P, "filter_network", s, c, ldc, d, B, L, z, relu_last=True, xb=sb,
                         cb=cb, zb=zb)
            return self._conv_last(P, s if sb is None else sb, B, L, dev)
        x = empty(M, R, device=dev)
        call("ensvs_copy_cols", s.data_ptr(), R, x.data_ptr(), R, M, R, stream())
        self._blocks(P, "filter_network", x, c, ldc, d, B, L, z, relu_last=True)
        outs = [self._conv_last(P, x, B, L, dev)]
        for t in (s, h, n):
            tr = empty(M, R, device=dev)
            call("ensvs_relu_mask", tr.data_ptr(), None, t.data_ptr(), t.data_ptr(), M * R, stream())
            outs.append(self._conv_last(P, tr, B, L, dev))
        return outs + [a]

    # ---------------------------------------------------------------- reference API
    @torch.no_grad()
    def forward(self, x, c, d):
        """x (B, 2, L) [sine, noise], c (B, C, T + 2w) aux with context, d (B, 1, L)
        -> (x, s, h, n, a) with shapes (B, 1, L) x 4 and (B, residual_channels, L)."""
        B, _, L = x.shape
        Tin = c.shape[2]
        T = Tin - 2 * self.aux_context_window
        if T * int(np.prod(self.upsample_net.upsample.upsample_scales)) != L:
            raise AssertionError("c.size(-1) after upsampling must equal x.size(-1)")
        # reference layouts are (B, C, T); the kernels use sample rows (B*L, C)
        xs = x.float().transpose(1, 2).contiguous().view(B * L, 2)
        cr = c.float().transpose(1, 2).contiguous().view(B * Tin, -1)
        dd = d.float().reshape(B * L).contiguous()
        y, s, h, n, a = self._run(xs, cr, cr.shape[1], Tin, 0, _lib.PAD_ZERO, T, dd, B,
                                  keep=True)
        v = lambda t: t.view(B, 1, L)  # noqa: E731
        return v(y), v(s), v(h), v(n), a.view(B, L, -1).transpose(1, 2)


def _cfg_get(cfg, key):
    return cfg[key] if isinstance(cfg, dict) else getattr(cfg, key)


class USFGANWrapper(nn.Module):
    """nnsvs/usfgan/__init__.py:7-65 on the device: dilated factors, the sine/noise source
    and the generator, from a host f0 track and device aux features."""

    def __init__(self, config, generator):
        super().__init__()
        self.generator = generator
        self.config = config

    def _data(self):
        return _cfg_get(self.config, "data")

    def _sources(self, f0_dev, B, T, noises=None):
        data = self._data()
        fs, hop = float(_cfg_get(data, "sample_rate")), int(_cfg_get(data, "hop_size"))
        if list(_cfg_get(data, "signal_types")) != ["sine", "noise"]:
            raise NotImplementedError("signal_types ['sine', 'noise'] (recipe)")
        dev = f0_dev.device
        L = T * hop
        d = empty(B * L, device=dev)
        call("ensvs_usf_dfactor", f0_dev.data_ptr(), B, T, hop, fs,
             float(_cfg_get(data, "dense_factor")), d.data_ptr(), stream())
        if noises is None:
            noises = []
            for _ in range(2):
                z = empty(B * L, device=dev)
                call("ensvs_randn", z.data_ptr(), B * L, next_seed(), stream())
                noises.append(z)
        sine_noise, noise = [t.reshape(-1).contiguous().float() for t in noises]
        ws = torch.empty(_lib.query("ensvs_usf_source_workspace", B, T, hop),
                         dtype=torch.float64, device=dev)
        xsrc = empty(B * L, 2, device=dev)
        scale = float(np.float32(T) / np.float32(L))
        call("ensvs_usf_source", f0_dev.data_ptr(), B, T, hop, scale, fs,
             float(_cfg_get(data, "sine_amp")), float(_cfg_get(data, "noise_amp")),
             sine_noise.data_ptr(), noise.data_ptr(), ws.data_ptr(), xsrc.data_ptr(), 2,
             stream())
        return xsrc, d, L

    @torch.no_grad()
    def inference(self, f0, aux_feats, noises=None):
        """f0 (T, 1) numpy (Hz), aux_feats (T, C) -> waveform (1, 1, T*hop).  ``noises``
        optionally replays the two N(0, 1) draws (sine noise, noise) of SignalGenerator."""
        gen = self.generator
        if "aux_context_window" not in _cfg_get(self.config, "generator"):
            raise NotImplementedError("SiFi-GAN branch (no aux_context_window) is not on the "
                                      "path")
        dev = next(gen.parameters()).device
        f0_dev = torch.from_numpy(np.ascontiguousarray(np.asarray(f0, dtype=np.float32)
                                                       .reshape(-1))).to(dev)
        T = f0_dev.numel()
        xsrc, d, L = self._sources(f0_dev, 1, T, noises)
        aux = aux_feats.to(dev).float().contiguous()
        w = gen.aux_context_window
        y = gen._run(xsrc, aux, aux.shape[1], T, -w, _lib.PAD_REPLICATE, T, d, 1)
        return y.view(1, 1, L)

    @torch.no_grad()
    def inference_batch(self, f0, aux_feats, noises=None):
        """Batched synthesis of B equal-length tracks: f0 (B, T) device tensor (Hz),
        aux_feats (B, T, C) -> (B, 1, T*hop).  One launch sequence for all tracks."""
        gen = self.generator
        B, T = f0.shape
        f0 = f0.float().contiguous()
        xsrc, d, L = self._sources(f0, B, T, noises)
        aux = aux_feats.float().contiguous().view(B * T, -1)
        w = gen.aux_context_window
        y = gen._run(xsrc, aux, aux.shape[1], T, -w, _lib.PAD_REPLICATE, T, d, B)
        return y.view(B, 1, L)
