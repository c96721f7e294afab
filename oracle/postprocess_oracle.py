"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the post-acoustic feature steps of the synthesis path (SURVEY.md §8
row f4): nnsvs/gen.py postprocess_acoustic (:1314-1530) for the configuration the multi-track
recipe synthesises with (nnsvs/bin/conf/synthesis/synthesis/world_gv_usfgan.yaml:
feature_type world, post_filter_type gv, trajectory_smoothing true (cutoff 50 / f0 20),
vuv_threshold 0.3, relative_f0 false, force_fix_vuv false, no vibrato streams), plus the
WORLD aperiodicity codec round trip predict_waveform applies before uSFGAN (gen.py:1637-1670).

Pinning: tests/golden/postprocess.npz holds the reference's own postprocess_acoustic outputs
(gen_goldens.py case_postprocess).  Two dependencies of that function are absent from this
image and are restated here from their published algorithms; the goldens run the reference
with these restatements patched in, so those two pieces are parity UNPINNED:
  * nnmnkwii.preprocessing.f0.interp1d (nnmnkwii 0.1.x): `interp1d` below;
  * nnmnkwii.frontend.merlin.linguistic_features: the frame-level features are an input
    (only the score-F0 column, get_pitch_index, is read: get_note_frame_indices,
    io/hts.py:29-45);
  * pyworld (0.3.x) DecodeAperiodicity / CodeAperiodicity of WORLD d4c.cpp: `world_bap_codec`.
"""
import numpy as np
from scipy import signal
from scipy.interpolate import interp1d as _sp_interp1d


def interp1d(f0, kind="slinear"):
    """nnmnkwii.preprocessing.f0.interp1d: fill frames <= 0 of a 1-d track by interpolating
    between the voiced frames; the ends take the first / last voiced value."""
    ndim = f0.ndim
    cont = f0.flatten()  # copy
    nz = np.where(cont > 0)[0]
    if len(nz) <= 0:
        return f0
    cont[0] = cont[nz[0]]
    cont[-1] = cont[nz[-1]]
    nz = np.where(cont > 0)[0]
    fn = _sp_interp1d(nz, cont[cont > 0], kind=kind)
    zi = np.where(cont <= 0)[0]
    cont[zi] = fn(zi)
    return cont[:, None] if ndim == 2 else cont


def variance_scaling(gv, feats, offset=2, note_frame_indices=None):
    """nnsvs/postfilters.py:9-46."""
    if note_frame_indices is not None:
        if len(note_frame_indices) == 0:
            return feats
        sel = feats[note_frame_indices]
    else:
        sel = feats
    utt_gv, utt_mu = sel.var(0), sel.mean(0)
    out = feats.copy()
    rows = note_frame_indices if note_frame_indices is not None else slice(None)
    out[rows, offset:] = (np.sqrt(gv[offset:] / utt_gv[offset:])
                          * (feats[rows, offset:] - utt_mu[offset:]) + utt_mu[offset:])
    return out


def lowpass_filter(x, fs, cutoff=5, N=5):
    """nnsvs/dsp.py:10-33 (zero-phase Butterworth)."""
    b, a = signal.butter(N, [cutoff / (fs // 2)], "lowpass")
    if len(x) <= max(len(a), len(b)) * (N // 2 + 1):
        return x
    return signal.filtfilt(b, a, x)


def world_bap_codec(bap):
    """pyworld.code_aperiodicity(clip(decode_aperiodicity(bap), 0, 1)) with the unvoiced bin-0
    fill (gen.py:1649-1670), at 48 kHz (band centres on the 2048-point FFT grid): frames whose
    mean coded aperiodicity exceeds -0.5 decode to all (1 - 1e-12) (d4c.cpp CheckVUV), others
    decode to 10^(bap/20) at the band centres and code back to themselves."""
    out = bap.astype(np.float64).copy()
    unv = out.mean(1) > -0.5
    out[unv] = 20.0 * np.log10(1.0 - 1e-12)
    return out.astype(np.float32)


def postprocess_acoustic(acoustic_features, score_f0, gv_var, stream_sizes=(60, 1, 1, 5),
                         frame_period=5, trajectory_smoothing=True,
                         trajectory_smoothing_cutoff=50, trajectory_smoothing_cutoff_f0=20,
                         vuv_threshold=0.5, f0_shift_in_cent=0, post_filter_type="gv"):
    """gen.py:1314-1530 for feature_type "world", static streams, relative_f0 False.
    score_f0: the frame-level score pitch column (> 0 on note frames)."""
    feats = acoustic_features.copy()
    if post_filter_type in ("gv", "nnsvs"):
        note = np.where(score_f0 > 0)[0]
        m = stream_sizes[0]
        feats[:, :m] = variance_scaling(np.asarray(gv_var).reshape(-1)[:m], feats[:, :m],
                                        offset=2, note_frame_indices=note)
    s = np.cumsum((0,) + tuple(stream_sizes))
    mgc, f0, vuv, bap = (feats[:, s[i]:s[i + 1]].copy() for i in range(4))
    # gen_spsvs_static_features (gen.py:1988-1991, 2010-2016)
    f0[vuv < vuv_threshold] = 0
    f0[np.nonzero(f0)] = np.exp(f0[np.nonzero(f0)])
    lf0 = f0.copy()
    lf0[np.nonzero(lf0)] = np.log(f0[np.nonzero(lf0)])
    lf0 = interp1d(lf0, kind="slinear")
    lf0 = lf0[:, None] if lf0.ndim == 1 else lf0
    if f0_shift_in_cent != 0:
        lf0 = lf0 + f0_shift_in_cent * np.log(2) / 1200
    if trajectory_smoothing:
        modfs = int(1 / (frame_period * 0.001))
        lf0[:, 0] = lowpass_filter(lf0[:, 0], modfs, cutoff=trajectory_smoothing_cutoff_f0)
        for d in range(mgc.shape[1]):
            mgc[:, d] = lowpass_filter(mgc[:, d], modfs, cutoff=trajectory_smoothing_cutoff)
        for d in range(bap.shape[1]):
            bap[:, d] = lowpass_filter(bap[:, d], modfs, cutoff=trajectory_smoothing_cutoff)
    if not bap.shape[-1] > 5:
        bap = np.clip(bap, a_min=-60, a_max=0)
    return mgc, lf0, vuv, bap
