"""Multi-track batch formats: synthetic SATB batches, pairing, collation, masks.

Pairing/collation mirror nnsvs/train_util.py (get_filtered_files_multitrack
:153-177, collate_fn_syncmultitrack_acoustic :937-1019, ensure_divisible_by
:522-537) and nnsvs/util.py (pad_2d :171-188, make_pad_mask :191-238); they
are integer/byte work and must be bit-exact.
"""
import os
import re

import numpy as np


def synthetic_batch(P, T, seed, lengths=None, in_dim=86, out_dim=67, num_speakers=4,
                    ph_start=3, ph_end=50, lf0_idx=51, vuv_idx=61):
    """Synthetic (main, sub) pair batch with the feature layout of SURVEY.md §8(d).

    in_feats: col 0 rest flag ~ Bernoulli(0.1); cols [ph_start, ph_end) one-hot
    phoneme held for 20-frame runs; col lf0_idx score log-F0 ~ U[0.3, 0.7] held
    for 40-frame runs; other cols U[0, 1).  out_feats ~ N(0, 1) with the V/UV
    column set to {0, 1}.  Frames past each length are zero (collate padding).
    Returns a dict of numpy arrays; lengths are sorted descending.
    """
    rng = np.random.default_rng(seed)
    if lengths is None:
        lengths = np.full(P, T, dtype=np.int64)
    lengths = np.sort(np.asarray(lengths, dtype=np.int64))[::-1].copy()
    out = {}
    nv = ph_end - ph_start
    for track in ("main", "sub"):
        x = rng.random((P, T, in_dim), dtype=np.float32)
        x[:, :, 0] = (rng.random((P, T)) < 0.1).astype(np.float32)
        x[:, :, ph_start:ph_end] = 0.0
        ph = rng.integers(0, nv, size=(P, (T + 19) // 20))
        ph = np.repeat(ph, 20, axis=1)[:, :T]
        np.put_along_axis(x[:, :, ph_start:ph_end], ph[:, :, None], 1.0, axis=2)
        lf0 = rng.uniform(0.3, 0.7, size=(P, (T + 39) // 40)).astype(np.float32)
        x[:, :, lf0_idx] = np.repeat(lf0, 40, axis=1)[:, :T]
        y = rng.standard_normal((P, T, out_dim)).astype(np.float32)
        y[:, :, vuv_idx] = (rng.random((P, T)) < 0.6).astype(np.float32)
        for b in range(P):
            x[b, lengths[b]:] = 0.0
            y[b, lengths[b]:] = 0.0
        out["x_" + track] = x
        out["y_" + track] = y
        out["spk_" + track] = rng.integers(0, num_speakers, size=(P, 1)).astype(np.int64)
    out["lengths"] = lengths
    return out


def seg_name(path):
    """Segment key of a feature file: `_(.*?)-` on the basename (train_util.py:167)."""
    return re.search(r"_(.*?)-", os.path.basename(path)).group(1)


def pair_files(files, lengths):
    """All (i <= j) pairs of files that share a segment (train_util.py:169-177)."""
    names = [seg_name(f) for f in files]
    pairs, plens = [], []
    for i in range(len(files)):
        for j in range(i, len(files)):
            if names[i] == names[j]:
                pairs.append((files[i], files[j]))
                plens.append((lengths[i], lengths[j]))
    return pairs, plens


def ordered_pairs(utt_ids):
    """Ordered (main, sub) pairs of the same segment incl. self (synthesis_multitrack.py:113-118)."""
    out = []
    for u0 in utt_ids:
        for u1 in utt_ids:
            if seg_name(u0 + "-x") == seg_name(u1 + "-x"):
                out.append((u0, u1))
    return out


def ensure_divisible_by(feats, N):
    """train_util.py:522-537."""
    if N == 1:
        return feats
    mod = len(feats) % N
    return feats[: len(feats) - mod] if mod != 0 else feats


def pad_2d(x, max_len, constant_values=0):
    """nnsvs/util.py:171-188."""
    return np.pad(x, [(0, max_len - len(x)), (0, 0)], mode="constant",
                  constant_values=constant_values)


def collate_syncmultitrack_acoustic(batch, reduction_factor=1):
    """collate_fn_syncmultitrack_acoustic (train_util.py:937-1019) on numpy.

    batch: list of 8-tuples (x0, y0, spk0, times0, x1, y1, spk1, times1).
    Returns (x0, y0, spk0, len0, x1, y1, spk1, len1) numpy arrays; both tracks
    are padded to the max trimmed length over BOTH tracks.
    """
    max_len = 0
    for idx in (0, 4):
        max_len = max(max_len, max(len(ensure_divisible_by(b[idx], reduction_factor))
                                   for b in batch))
    data = []
    for idx in (0, 4):
        lens = [len(ensure_divisible_by(b[idx], reduction_factor)) for b in batch]
        xb = np.stack([pad_2d(ensure_divisible_by(b[idx], reduction_factor), max_len)
                       for b in batch])
        yb = np.stack([pad_2d(ensure_divisible_by(b[idx + 1], reduction_factor), max_len)
                       for b in batch])
        sb = np.array([[float(b[idx + 2])] for b in batch], dtype=np.float32)
        data += [xb, yb, sb, np.asarray(lens, dtype=np.int64)]
    return tuple(data)


def onset_merge_indices(a, b):
    """Row alignment of two tracks by note onset: the two-pointer merge of
    gen.py:321-356 (time-lag), gen.py:637-676 (duration) and train_util.py:811-852
    (collate_fn_syncmultitrack).  a, b: sorted onset times of tracks 0 / 1; the
    reference appends the sentinel inf = a[-1] + b[-1] to both and merges while either
    track has notes left, advancing the earlier one (both on a tie).  Returns int64
    arrays (i0, i1): the source note of each track per merged row, -1 where that track
    has no note there (a zero row, mask False)."""
    a = np.asarray(a)
    b = np.asarray(b)
    inf = a[-1] + b[-1]
    a = np.append(a, inf)
    b = np.append(b, inf)
    i0, i1 = [], []
    aid = bid = 0
    while aid < len(a) - 1 or bid < len(b) - 1:
        if a[aid] < b[bid]:
            i0.append(aid)
            i1.append(-1)
            aid += 1
        elif a[aid] > b[bid]:
            i0.append(-1)
            i1.append(bid)
            bid += 1
        else:
            i0.append(aid)
            i1.append(bid)
            aid += 1
            bid += 1
    return np.asarray(i0, dtype=np.int64), np.asarray(i1, dtype=np.int64)


def _take_rows(x, idx, like):
    """Rows idx of x (float32), zero rows where idx < 0 (the reference's zeros_like of
    the OTHER track's row: same width)."""
    out = np.zeros((len(idx), like.shape[1]), dtype=np.float32)
    ok = idx >= 0
    out[ok] = x[idx[ok]]
    return out


def merge_tracks_by_onset(x0, x1, a, b):
    """gen.py:637-676: (new_x0, new_x1, mask0, mask1), both tracks on the merged rows."""
    i0, i1 = onset_merge_indices(a, b)
    return _take_rows(x0, i0, x0), _take_rows(x1, i1, x0), i0 >= 0, i1 >= 0


def collate_syncmultitrack(batch, reduction_factor=1):
    """collate_fn_syncmultitrack (train_util.py:776-934, stream selection off) on numpy:
    the timing models' collate.  batch: 8-tuples (x0, y0, spk0, times0, x1, y1, spk1,
    times1); both tracks of a sample are first aligned by onset (onset_merge_indices).
    Returns (x0, y0, spk0, len0, mask0, x1, y1, spk1, len1, mask1); lengths are the
    reference's: measured BEFORE the merge (train_util.py:806-809)."""
    lengths_list = [[len(ensure_divisible_by(x[idx], reduction_factor)) for x in batch]
                    for idx in (0, 4)]
    merged = []
    for x in batch:
        i0, i1 = onset_merge_indices(x[3], x[7])
        nx0, nx1 = _take_rows(x[0], i0, x[0]), _take_rows(x[4], i1, x[0])
        ny0, ny1 = _take_rows(x[1], i0, x[1]), _take_rows(x[5], i1, x[1])
        merged.append((nx0, ny0, x[2], i0 >= 0, nx1, ny1, x[6], i1 >= 0))
    max_len = max(len(ensure_divisible_by(m[idx], reduction_factor))
                  for m in merged for idx in (0, 4))
    data = []
    for t, idx in enumerate((0, 4)):
        data.append(np.stack([pad_2d(ensure_divisible_by(m[idx], reduction_factor), max_len)
                              for m in merged]))
        data.append(np.stack([pad_2d(ensure_divisible_by(m[idx + 1], reduction_factor),
                                     max_len) for m in merged]))
        data.append(np.array([[float(m[idx + 2])] for m in merged], dtype=np.float32))
        data.append(np.asarray(lengths_list[t], dtype=np.int64))
        masks = []
        for m in merged:
            mk = ensure_divisible_by(m[idx + 3], reduction_factor)
            masks.append(np.concatenate([mk, np.zeros(max_len - len(mk), dtype=bool)]))
        data.append(np.stack(masks))
    return tuple(data)


def make_pad_mask(lengths, maxlen=None):
    lengths = np.asarray(lengths, dtype=np.int64)
    maxlen = int(lengths.max()) if maxlen is None else int(maxlen)
    return np.arange(maxlen, dtype=np.int64)[None, :] >= lengths[:, None]


def make_non_pad_mask(lengths, maxlen=None):
    return ~make_pad_mask(lengths, maxlen)


def sort_pair_batch(len0, len1):
    """train_acoustic_multitrack.py:472-483: the two tracks are sorted INDEPENDENTLY
    (descending, stable as torch.sort on CPU is for these sizes); returns the two
    permutations and lengths = max(L0, L1) elementwise (:82)."""
    i0 = np.argsort(-np.asarray(len0), kind="stable")
    i1 = np.argsort(-np.asarray(len1), kind="stable")
    l0 = np.asarray(len0)[i0]
    l1 = np.asarray(len1)[i1]
    return i0, i1, np.maximum(l0, l1)


def shard_pairs(batches, rank, world):
    """Per-rank mini-batches for data parallelism over pairs (train_util.py:1176-1182):
    each index batch is split as ``x[rank::world]`` and batches whose size is not a
    multiple of ``world`` are dropped, as the reference does."""
    if world == 1:
        return [list(x) for x in batches]
    return [list(x[rank::world]) for x in batches if len(x) % world == 0]


def synthetic_score(seed, parts, T, note_dim=82, frame_period=5):
    """Synthetic score tracks of a `parts`-part song of T frames for the timing models
    (config 5 bench): notes on a shared 100-frame onset grid (0.5 s; every part takes ~70 %
    of the grid points, so onsets tie across parts), 1-3 phoneme labels per note sharing
    the note onset (get_note_indices groups labels by onset), ~15 % silence notes.
    Per part: dict(start, end (HTS units, int64), contexts, ph_feats (N, note_dim) float32,
    note_feats (one row per note))."""
    rng = np.random.default_rng(seed)
    shift = int(frame_period * 1e4)
    grid = np.arange(0, T, 100)
    tracks = []
    for _ in range(parts):
        on = grid[rng.random(len(grid)) < 0.7]
        if len(on) == 0 or on[0] != 0:
            on = np.concatenate(([0], on))
        start, end, ctx, first = [], [], [], []
        for k, o in enumerate(on):
            nxt = on[k + 1] if k + 1 < len(on) else T
            sil = rng.random() < 0.15
            first.append(len(start))
            for _ in range(1 if sil else int(rng.integers(1, 4))):
                start.append(int(o) * shift)
                end.append(int(nxt) * shift)
                ctx.append("x-sil+y@1" if sil else "x-a+y@1")
        ph = rng.random((len(start), note_dim)).astype(np.float32)
        tracks.append(dict(start=np.asarray(start, np.int64), end=np.asarray(end, np.int64),
                           contexts=ctx, ph_feats=ph, note_feats=ph[first]))
    return tracks
