"""Multi-track synthesis driver: timing inference glue, acoustic inference and vocoding
(BASELINE config 5, the jaCappella 6-part pipeline).

Restates, over arrays instead of nnmnkwii HTSLabelFile objects:
  * predict_timelag_multitrack   nnsvs/gen.py:214-416
  * predict_duration_multitrack  nnsvs/gen.py:551-720
  * predict_timing_multitrack    nnsvs/gen.py:912-1006 (returns all four values; the
    reference's caller unpacks three of them, Appendix A-12)
  * the ordered-pair loop of     nnsvs/bin/synthesis_multitrack.py:113-288

Host work is only what the reference does on the host around its models: scaler
transforms, the onset merge of the two tracks (data.merge_tracks_by_onset, bit-exact),
rounding / clipping and the duration fitting (timing_post.postprocess_duration).  The
time-lag and duration MDN models, the acoustic model and the vocoder run in libensvs.so.

Inputs are the host feature matrices the reference derives from HTS labels with nnmnkwii
(fe.linguistic_features + log-F0 conditioning, gen.py:262-294 / 581-597): that feature
extraction is offline label processing, out of this path's scope.
"""
import numpy as np
import torch

from . import data
from .base import PredictionType
from .timing_post import get_note_indices, postprocess_duration


def _is_silence(label):
    """gen.py:43-49."""
    if "@" in label:
        return "-sil" in label or "-pau" in label
    return label in ("sil", "pau")


def _normalise(feats, in_scaler, force_clip, pitch_indices):
    x = in_scaler.transform(np.asarray(feats, dtype=np.float32))
    if force_clip and getattr(in_scaler, "kind", "") == "minmax":
        keep = [i for i in range(x.shape[1]) if i not in set(pitch_indices)]
        x[:, keep] = np.clip(x[:, keep], in_scaler.feature_range[0], in_scaler.feature_range[1])
    return x.astype(np.float32)


def _merged_input(feats, starts, in_scaler, force_clip, pitch_indices, device):
    xs = [_normalise(f, in_scaler, force_clip, pitch_indices) for f in feats]
    x0, x1, mask0, _ = data.merge_tracks_by_onset(xs[0], xs[1], starts[0], starts[1])
    x = np.concatenate([x0, x1], axis=1)[None]
    return torch.from_numpy(np.ascontiguousarray(x)).to(device), mask0


def _spk(spks, device):
    return tuple(torch.as_tensor(s).reshape(-1).to(device) for s in spks)


@torch.no_grad()
def predict_timelag_multitrack(timelag_model, note_feats, note_starts, note_contexts0, spks,
                               in_scaler, out_scaler, allowed_range=None,
                               allowed_range_rest=None, force_clip_input_features=False,
                               pitch_indices=(), frame_period=5, device="cuda"):
    """gen.py:214-416.  note_feats / note_starts: per track (main first) the note-level
    features (un-normalised) and note onset times (HTS units); note_contexts0: the main
    track's note label strings (silence test of the clipping).  Returns (time-lag in HTS
    units (N0, D), time-lag before rounding (N0, D), merged-row mask of the main track)."""
    if allowed_range is None:
        allowed_range = [-20, 20]
    if allowed_range_rest is None:
        allowed_range_rest = [-40, 40]
    shift = int(frame_period * 1e4)
    x, mask0 = _merged_input(note_feats, note_starts, in_scaler, force_clip_input_features,
                             pitch_indices, device)
    if timelag_model.prediction_type() != PredictionType.PROBABILISTIC:
        raise NotImplementedError("the recipe's time-lag model is an MDN (gen.py:389)")
    max_mu, _ = timelag_model.inference(x, spks=_spk(spks, device))
    pred = out_scaler.inverse_transform(max_mu.squeeze(0).cpu().numpy())
    pred = pred[mask0]
    eval_pred = pred
    pred = np.round(pred)
    for idx in range(len(pred)):
        lo, hi = allowed_range_rest if _is_silence(note_contexts0[idx]) else allowed_range
        pred[idx] = np.clip(pred[idx], lo, hi)
    return pred * shift, eval_pred, mask0


@torch.no_grad()
def predict_duration_multitrack(duration_model, ph_feats, ph_starts, spks, in_scaler,
                                out_scaler, force_clip_input_features=False, pitch_indices=(),
                                device="cuda"):
    """gen.py:551-720: phoneme-level features of both tracks merged by onset, the MDN
    duration model, de-normalised (mu, sigma^2) of the main track's rows."""
    x, mask0 = _merged_input(ph_feats, ph_starts, in_scaler, force_clip_input_features,
                             pitch_indices, device)
    if duration_model.prediction_type() != PredictionType.PROBABILISTIC:
        raise NotImplementedError("the recipe's duration model is an MDN (gen.py:680)")
    max_mu, max_sigma = duration_model.inference(x, spks=_spk(spks, device))
    sigma_sq = max_sigma.squeeze(0).cpu().numpy() ** 2 * out_scaler.var_
    sigma_sq = np.maximum(sigma_sq, 1e-14)
    mu = out_scaler.inverse_transform(max_mu.squeeze(0).cpu().numpy())
    return mu[mask0], sigma_sq[mask0]


def predict_timing_multitrack(timelag_model, duration_model, tracks, spks, timelag_scalers,
                              duration_scalers, allowed_range=None, allowed_range_rest=None,
                              force_clip_input_features=True, frame_period=5, device="cuda"):
    """gen.py:912-1006.  tracks: [main, sub] dicts with the phoneme labels' 'start', 'end'
    (HTS units), 'contexts' and features 'ph_feats' (phoneme level) and 'note_feats' (note
    level, one row per note of get_note_indices).  Returns (start_times, end_times of the
    duration-modified main-track labels, d_norms, time-lag before rounding, mask)."""
    note_idx = [get_note_indices(t["start"]) for t in tracks]
    note_starts = [np.asarray(t["start"])[ni] for t, ni in zip(tracks, note_idx)]
    ctx0 = [tracks[0]["contexts"][i] for i in note_idx[0]]
    lag, lag_eval, mask = predict_timelag_multitrack(
        timelag_model, [t["note_feats"] for t in tracks], note_starts, ctx0, spks,
        timelag_scalers[0], timelag_scalers[1], allowed_range, allowed_range_rest,
        force_clip_input_features, frame_period=frame_period, device=device)
    durations = predict_duration_multitrack(
        duration_model, [t["ph_feats"] for t in tracks], [t["start"] for t in tracks], spks,
        duration_scalers[0], duration_scalers[1], force_clip_input_features, device=device)
    st, en, d_norms = postprocess_duration(tracks[0]["start"], tracks[0]["end"], durations,
                                           lag, frame_period=frame_period)
    return st, en, d_norms, lag_eval, mask


def ordered_pairs(utt_ids):
    """synthesis_multitrack.py:113-118: every (utt0, utt1) of the same segment, self-pairs
    included, in list order."""
    return data.ordered_pairs(utt_ids)
