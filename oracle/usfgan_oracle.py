"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU (PyTorch fp32) restatement of the uSFGAN synthesis path of
sarulab-speech/ensemble_svs_with_interactions: the
``ParallelHnUSFGANGenerator`` forward and the ``USFGANWrapper.inference`` input
pipeline (dilated factors, sine/noise source).  It is the checker for the HIP
vocoder path; only tests/ and bench.py's cpu_baseline leg may import it.

Parity is PINNED by tests/golden/usfgan.npz and usfgan_pd_index.npz, produced by
the reference itself (tests/golden/gen_goldens.py, cases "usfgan" / "pd_index")
and checked against this file in tests/test_oracle_golden.py.

Functional style as ensvs_oracle.py: ``P`` is a dict keyed exactly like the
reference generator's ``state_dict`` (weight-normed ``weight_g``/``weight_v`` or
plain ``weight`` after ``remove_weight_norm``); random draws are arguments.
Reference line numbers cite the 2025-03-21 snapshot.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

# recipe generator config: recipes/_common/conf/jp_dev_48k_nodyn/train_usfgan/generator/
# nnsvs_world_parallel_hn_usfgan_sr48k.yaml:8-42 and data/nnsvs_world_sr48k.yaml:12-18
RECIPE = dict(
    harmonic=dict(blockA=20, cycleA=4, blockF=0, cycleF=0),
    noise=dict(blockA=0, cycleA=0, blockF=5, cycleF=5),
    filt=dict(blockA=0, cycleA=0, blockF=30, cycleF=3),
    pe_layers=3, pe_kernel=5, aux_context_window=2, upsample_scales=[5, 4, 4, 3],
    sample_rate=48000, hop_size=240, dense_factor=4, sine_amp=0.1, noise_amp=0.003)


def weight(P, name):
    """Effective conv weight: plain, or torch weight_norm (dim 0) g * v / ||v||
    (nn.utils.weight_norm, applied by generator.py:536-544)."""
    if name + ".weight" in P:
        return P[name + ".weight"]
    g, v = P[name + ".weight_g"], P[name + ".weight_v"]
    norm = v.reshape(v.shape[0], -1).norm(dim=1).reshape(-1, *([1] * (v.dim() - 1)))
    return v * (g / norm)


def conv1x1(P, name, x):
    return F.conv1d(x, weight(P, name), P.get(name + ".bias"))


# ------------------------------------------------------------ input pipeline

def dilated_factor(f0, fs, dense_factor):
    """usfgan/utils/features.py:56-75 (float64 numpy; unvoiced -> fs / dense_factor)."""
    f0 = np.array(f0, copy=True)
    f0[f0 == 0] = fs / dense_factor
    d = np.ones(f0.shape) * fs
    d /= f0
    d /= dense_factor
    return d


def signal_generator(f0, hop, fs, sine_amp, noise_amp, sine_noise, noise):
    """SignalGenerator(signal_types=["sine", "noise"]) (usfgan/utils/features.py:112-164).

    f0 (B, 1, T) float32; sine_noise / noise: the two N(0, 1) draws (B, 1, T*hop) in the
    order the reference makes them (sinusoid first, then random_noise)."""
    L = f0.shape[-1] * hop
    vuv = F.interpolate((f0 > 0) * torch.ones_like(f0), L)
    rad = (F.interpolate(f0, L) / fs) % 1
    sine = vuv * torch.sin(torch.cumsum(rad, dim=2) * 2 * np.pi) * sine_amp
    amp = vuv * noise_amp + (1.0 - vuv) * noise_amp / 3.0
    sine = sine + sine_noise * amp
    return torch.cat([sine, noise], dim=1)


# ------------------------------------------------------------------ layers

def pd_indexing(x, d, dilation):
    """usfgan/utils/index.py:12-54: pitch-dependent past/future samples.  Index math in
    float32 as the reference (round half to even); out-of-range samples read zero."""
    B, C, L = x.shape
    dil = d * dilation
    idxP = torch.add(-dil, torch.arange(-L, 0).float()).round().long()
    maxP = int(-(idxP.min() + L))
    assert maxP >= 0
    xP = F.pad(x, (maxP, 0))
    idxF = torch.add(dil, torch.arange(0, L).float()).round().long()
    maxF = int(idxF.max() - (L - 1))
    assert maxF >= 0
    xF = F.pad(x, (0, maxF))
    bi = torch.arange(B)[:, None, None]
    ci = torch.arange(C)[None, :, None]
    return xP[bi, ci, idxP], xF[bi, ci, idxF]


def _gated(h, c_proj):
    xa, xb = (h + c_proj).chunk(2, dim=1)
    return torch.tanh(xa) * torch.sigmoid(xb)


def adaptive_block(P, pre, x, xP, xF, c):
    """AdaptiveBlock.forward (usfgan/layers/residual_block.py:198-234).  Its skip output is
    discarded by ResidualBlocks (:323-336), so it is not computed."""
    h = conv1x1(P, pre + "convC", x) + conv1x1(P, pre + "convP", xP) + \
        conv1x1(P, pre + "convF", xF)
    z = _gated(h, F.conv1d(c, weight(P, pre + "conv1x1_aux")))
    return (conv1x1(P, pre + "conv1x1_out", z) + x) * math.sqrt(0.5)


def fixed_block(P, pre, x, c, dilation):
    """FixedBlock.forward (residual_block.py:123-157): reflect-padded dilated k3 conv."""
    h = F.conv1d(F.pad(x, (dilation, dilation), mode="reflect"), weight(P, pre + "conv"),
                 P.get(pre + "conv.bias"), dilation=dilation)
    z = _gated(h, F.conv1d(c, weight(P, pre + "conv1x1_aux")))
    return (conv1x1(P, pre + "conv1x1_out", z) + x) * math.sqrt(0.5)


def residual_blocks(P, pre, spec, x, c, d):
    """ResidualBlocks.forward (residual_block.py:311-336), cascade_mode 0 (adaptive first).
    Adaptive dilation 2^(i % (blockA / cycleA)), fixed 2^(i % (blockF / cycleF))."""
    nA, cA = spec["blockA"], max(spec["cycleA"], 1)
    nF, cF = spec["blockF"], max(spec["cycleF"], 1)
    for i in range(nA):
        xP, xF = pd_indexing(x, d, 2 ** (i % (nA // cA)))
        x = adaptive_block(P, f"{pre}conv_dilated.{i}.", x, xP, xF, c)
    for i in range(nF):
        x = fixed_block(P, f"{pre}conv_dilated.{nA + i}.", x, c, 2 ** (i % (nF // cF)))
    return x


def upsample_net(P, c, scales):
    """ConvInUpsampleNetwork.forward (usfgan/layers/upsample.py:178-194, 111-128):
    conv_in without padding, then per scale nearest x s along time + Conv2d(1,1,(1,2s+1))."""
    c = F.conv1d(c, weight(P, "upsample_net.conv_in")).unsqueeze(1)
    for i, s in enumerate(scales):
        c = F.interpolate(c, scale_factor=(1, s), mode="nearest")
        c = F.conv2d(c, weight(P, f"upsample_net.upsample.up_layers.{2 * i + 1}"),
                     padding=(0, s))
    return c.squeeze(1)


def periodicity_estimator(P, c, layers=3, k=5):
    """PeriodicityEstimator.forward (residual_block.py:389-399): replicate-padded convs,
    ReLU between, sigmoid last."""
    h = c
    for i in range(layers):
        name = f"periodicity_estimator.layers.{2 * i}"
        h = F.conv1d(F.pad(h, (k // 2, k // 2), mode="replicate"), weight(P, name),
                     P[name + ".bias"])
        h = torch.sigmoid(h) if i == layers - 1 else F.relu(h)
    return h


def conv_last(P, x):
    """generator.py:461-466: ReLU -> 1x1 -> ReLU -> 1x1."""
    return conv1x1(P, "conv_last.3", F.relu(conv1x1(P, "conv_last.1", F.relu(x))))


def generator_forward(P, x, c, d, cfg=RECIPE):
    """ParallelHnUSFGANGenerator.forward (usfgan/models/generator.py:472-522)
    -> (x, s, h, n, a)."""
    c = upsample_net(P, c, cfg["upsample_scales"])
    assert c.shape[-1] == x.shape[-1]
    a = periodicity_estimator(P, c, cfg["pe_layers"], cfg["pe_kernel"])
    sine, noise = torch.chunk(x, 2, 1)
    h = conv1x1(P, "conv_first_sine", sine)
    n = conv1x1(P, "conv_first_noise", noise)
    h = residual_blocks(P, "harmonic_network.", cfg["harmonic"], h, c, d)
    n = residual_blocks(P, "noise_network.", cfg["noise"], n, c, d)
    h = a * h
    n = (1.0 - a) * n
    s = h + n
    y = residual_blocks(P, "filter_network.", cfg["filt"], s, c, d)
    return conv_last(P, y), conv_last(P, s), conv_last(P, h), conv_last(P, n), a


def generator_inputs(f0, aux, sine_noise, noise, cfg=RECIPE):
    """USFGANWrapper.inference input pipeline (usfgan/__init__.py:13-62), non-SiFiGAN
    branch.  f0 (T, 1) float32 numpy (Hz), aux (T, C) float32 tensor -> (x, c, d)."""
    fs, hop = cfg["sample_rate"], cfg["hop_size"]
    df = dilated_factor(np.squeeze(f0.copy()), fs, cfg["dense_factor"]).repeat(hop, axis=0)
    w = cfg["aux_context_window"]
    c = F.pad(aux.unsqueeze(0).transpose(2, 1), (w, w), mode="replicate")
    d = torch.FloatTensor(df).view(1, 1, -1)
    f0_t = torch.FloatTensor(f0).unsqueeze(0).transpose(2, 1)
    x = signal_generator(f0_t, hop, fs, cfg["sine_amp"], cfg["noise_amp"], sine_noise, noise)
    return x, c, d


def usfgan_inference(P, f0, aux, sine_noise, noise, cfg=RECIPE):
    """USFGANWrapper.inference (usfgan/__init__.py:13-65) -> waveform (1, 1, T*hop)."""
    x, c, d = generator_inputs(f0, aux, sine_noise, noise, cfg)
    return generator_forward(P, x, c, d, cfg)[0]
