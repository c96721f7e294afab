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
