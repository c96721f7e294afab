"""Host-side timing post-processing: note-level time-lag and phoneme-duration fitting.

Restates nnsvs/gen.py:723-817 (`postprocess_duration`) and nnsvs/io/hts.py:95-112
(`get_note_indices`) over plain arrays instead of nnmnkwii's HTSLabelFile, which is absent
from this image.  The label operations it relies on are restated from nnmnkwii's published
behaviour (HTSLabelFile.set_durations: cumulative end times from the first start time in
50 000-unit frames; merlin.duration_features: (end - start) / 50 000 per label).  Parity is
UNPINNED: no reference output covers this function (nnmnkwii cannot be imported to produce
one); tests/test_timing_post.py checks hand-computed cases and the invariants of eq. (11),
(12), (16), (17) of https://arxiv.org/abs/2108.02776.

Times are HTS units (100 ns); one frame at frame_period 5 ms is 50 000 units.
"""
import numpy as np


def get_note_indices(start_times):
    """hts.py:95-112: index of the first label of every note (labels of one note share
    their score start time)."""
    st = np.asarray(start_times)
    if len(st) == 0:
        return []
    idx = [0]
    last = st[0]
    for i in range(1, len(st)):
        if st[i] != last:
            idx.append(i)
            last = st[i]
    return idx


def postprocess_duration(start_times, end_times, pred_durations, lag, frame_period=5):
    """gen.py:723-817 on arrays.

    start_times, end_times: (N,) score label times (HTS units); pred_durations: (N,) or
    (N, 1) predicted phoneme durations in frames, or the MDN pair (mu, sigma^2) of such
    arrays; lag: (num_notes,) or (num_notes, 1) predicted note time-lags (HTS units).
    Returns (start_times, end_times, d_norms): the output labels' times (int64) and the
    cumulative per-note phoneme durations in frames, as the reference returns."""
    shift = int(frame_period * 1e4)
    st0 = np.asarray(start_times, dtype=np.int64)
    en0 = np.asarray(end_times, dtype=np.int64)
    lag = np.asarray(lag, dtype=np.float64).reshape(-1)
    notes = get_note_indices(st0) + [len(st0)]
    is_mdn = isinstance(pred_durations, tuple) and len(pred_durations) == 2
    out_st, out_en, d_norms = [], [], []
    for i in range(1, len(notes)):
        a, b = notes[i - 1], notes[i]
        n = b - a
        # eq (11): note length corrected by the time-lags at its two ends
        L = int((en0[a] - st0[a]) / shift)
        if i < len(notes) - 1:
            L_hat = L - (lag[i - 1] - lag[i]) / shift
        else:
            L_hat = L - lag[i - 1] / shift
        L_hat = max(L_hat, 1)
        # shifted note start (kept inside the note, non-negative, after the previous one)
        ps = np.minimum(st0[a:b] + lag[i - 1], en0[a:b] - shift * n)
        ps = np.maximum(ps, 0)
        if out_st:
            ps = np.maximum(ps, out_st[-1] + shift)
        if is_mdn:
            mu = np.asarray(pred_durations[0])[a:b]
            var = np.asarray(pred_durations[1])[a:b]
            rho = (L_hat - mu.sum()) / var.sum()         # eq (17)
            d = mu + rho * var                           # eq (16)
            if np.any(d <= 0):
                d = L_hat * mu / mu.sum()                # eq (12) with mu as d_hat
        else:
            dh = np.asarray(pred_durations)[a:b]
            d = L_hat * dh / dh.sum()                    # eq (12)
        d = np.round(d)
        d[d <= 0] = 1
        # set_durations: end times accumulate from the (shifted) first start time
        ends = ps[0] + np.cumsum(d.reshape(-1)) * shift
        starts = np.concatenate(([ps[0]], ends[:-1]))
        d_norms += np.cumsum(d.reshape(-1)).tolist()
        if out_en:
            out_en[-1] = starts[0]
        out_st += [int(v) for v in starts]
        out_en += [int(v) for v in ends]
    return (np.asarray(out_st, dtype=np.int64), np.asarray(out_en, dtype=np.int64),
            np.array(d_norms))
