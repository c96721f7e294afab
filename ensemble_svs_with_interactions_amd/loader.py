"""On-disk multi-track training data: file discovery, the sync pair dataset, dynamic
batching and a pinned-memory, stream-overlapped host->HBM batch feeder.

Mirrors nnsvs/train_util.py:
  get_filtered_files            :103-150
  get_filtered_files_multitrack :153-177 (filters hard-coded off)
  batch_by_size                 :190-246 (with _is_batch_full :180-187)
  SyncMultiTrackDataset         :439-520 (__getitem__ :473-502, ordered_indices :507-520)
  ShuffleBatchSampler           :51-70
  setup_data_loaders (multitrack, padding "time", batch_max_frames > 0) :1053-1240
All of it is integer / byte work and bit-exact against reference-generated fixtures
(tests/test_loader.py, tests/golden/gen_goldens.py::case_loader).

On-disk format (prepare_features_multitrack_sync.py:37-40): `{spk}_{song_seg}-feats.npy`
float32 (T, D) under in_dir / out_dir, and `-times.npy` next to the *org* copy of the
input features (the path's "norm" replaced by "org", train_util.py:497-499).
"""
import os
import random
import sys
import threading
import time
import queue
from glob import glob

import numpy as np
import torch

from . import data as _data


def _num_frames(path):
    """Row count of a .npy file from its header (np.load(mmap_mode="r") reads no data);
    equals len(np.load(path)) as the reference computes it."""
    return int(np.load(path, mmap_mode="r").shape[0])


def get_filtered_files(data_root, logger=None, filter_long_segments=False,
                       filter_num_frames=6000, filter_min_num_frames=0):
    """train_util.py:103-150: sorted `*-feats.npy` under data_root and their lengths,
    optionally keeping only filter_min_num_frames < T < filter_num_frames."""
    files = sorted(glob(os.path.join(data_root, "*-feats.npy")))
    lengths = [_num_frames(f) for f in files]
    if filter_long_segments:
        keep = [i for i, n in enumerate(lengths)
                if filter_min_num_frames < n < filter_num_frames]
        if logger is not None and len(keep) < len(files):
            for i in sorted(set(range(len(files))) - set(keep)):
                logger.info(f"Filtered: {files[i]} is too long or short: {lengths[i]}")
            logger.info(f"Filtered {len(files) - len(keep)} files")
        files = [files[i] for i in keep]
        lengths = [lengths[i] for i in keep]
    return files, lengths


def get_filtered_files_multitrack(data_root, logger=None, filter_long_segments=False,
                                  filter_num_frames=6000, filter_min_num_frames=0):
    """train_util.py:153-177: every (i <= j) pair of files of the same segment.  The
    reference passes filter_long_segments=False to get_filtered_files whatever the
    caller asks (App. A-17); reproduced."""
    files, lengths = get_filtered_files(data_root, logger, filter_long_segments=False)
    return _data.pair_files(files, lengths)


def _is_batch_full(batch, num_tokens, max_tokens, max_sentences):
    if len(batch) == 0:
        return 0
    if len(batch) == max_sentences:
        return 1
    return 1 if num_tokens > max_tokens else 0


def batch_by_size(indices, num_tokens_fn, max_tokens=None, max_sentences=None,
                  required_batch_size_multiple=1):
    """train_util.py:190-246: greedy buckets of indices whose padded size
    (len(batch) * longest) stays within max_tokens; when a batch closes, its size is
    rounded down to a multiple of required_batch_size_multiple and the rest carries
    over.  Raises AssertionError on a sample longer than max_tokens (as the reference)."""
    max_tokens = sys.maxsize if max_tokens is None else max_tokens
    max_sentences = sys.maxsize if max_sentences is None else max_sentences
    mult = required_batch_size_multiple
    indices = list(indices)
    batches, batch, lens = [], [], []
    longest = 0
    for idx in indices:
        n = num_tokens_fn(idx)
        lens.append(n)
        longest = max(longest, n)
        assert longest <= max_tokens, (
            f"sentence at index {idx} of size {longest} exceeds max_tokens limit of "
            f"{max_tokens}!")
        if _is_batch_full(batch, (len(batch) + 1) * longest, max_tokens, max_sentences):
            cut = max(mult * (len(batch) // mult), len(batch) % mult)
            batches.append(batch[:cut])
            batch = batch[cut:]
            lens = lens[cut:]
            longest = max(lens) if lens else 0
        batch.append(idx)
    if batch:
        batches.append(batch)
    return batches


class ShuffleBatchSampler:
    """train_util.py:51-70: yields the precomputed batches, shuffled in place with
    Python's `random` each epoch when shuffle is on."""

    def __init__(self, batches, drop_last=False, shuffle=True):
        self.batches = batches
        self.drop_last = drop_last
        self.shuffle = shuffle

    def __iter__(self):
        if self.shuffle:
            random.shuffle(self.batches)
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


def times_path(in_path):
    """train_util.py:497-499: `<stem>-times.npy` of the *org* features."""
    return (in_path.split("-feats")[0] + "-times.npy").replace("norm", "org")


class SyncMultiTrackDataset:
    """train_util.py:439-520.  Item idx is the pair (in_paths[idx], out_paths[idx]) and
    returns the 8-tuple (x0, y0, spk0, times0, x1, y1, spk1, times1); the speaker id is
    speaker_list.index of the basename's prefix before the first "_".  The cache is a
    plain list (the loader below uses threads, not worker processes, so the
    reference's multiprocessing.Manager list is not needed)."""

    def __init__(self, in_paths, out_paths, lengths, speaker_list, shuffle=False,
                 allow_cache=True):
        self.in_paths = in_paths
        self.out_paths = out_paths
        self.lengths = lengths
        self.max_lengths = [max(p) for p in lengths]
        self.sort_by_len = True
        self.shuffle = shuffle
        self.allow_cache = allow_cache
        self.caches = [()] * len(in_paths) if allow_cache else None
        self.get_spkid = {name: i for i, name in enumerate(speaker_list)}

    def __len__(self):
        return len(self.in_paths)

    def __getitem__(self, idx):
        if self.allow_cache and len(self.caches[idx]) != 0:
            return self.caches[idx]
        out = []
        for src, dst in zip(self.in_paths[idx], self.out_paths[idx]):
            spk = self.get_spkid[os.path.basename(src).split("_")[0]]
            out += [np.load(src), np.load(dst), spk, np.load(times_path(src))]
        out = tuple(out)
        if self.allow_cache:
            self.caches[idx] = out
        return out

    def num_tokens(self, index):
        return self.max_lengths[index]

    def ordered_indices(self):
        """train_util.py:507-520: a np.random permutation, then a stable (mergesort)
        sort by the pair's longer length; arange when not shuffling."""
        if not self.shuffle:
            return np.arange(len(self))
        idx = np.random.permutation(len(self))
        if self.sort_by_len:
            idx = idx[np.argsort(np.array(self.max_lengths)[idx], kind="mergesort")]
        return idx


def setup_multitrack_batches(in_dir, out_dir, speaker_list, batch_max_frames, train=True,
                             rank=0, world=1, allow_cache=False):
    """The multitrack / padding "time" / dynamic-batch branch of setup_data_loaders
    (train_util.py:1053-1190): pair files, dataset, ordered indices, batch_by_size with
    required_batch_size_multiple = world, then the x[rank::world] split (batches whose
    size is not a multiple of world dropped).  Returns (dataset, batches)."""
    in_files, lengths = get_filtered_files_multitrack(in_dir)
    out_files, _ = get_filtered_files_multitrack(out_dir)
    ds = SyncMultiTrackDataset(in_files, out_files, lengths, speaker_list, shuffle=train,
                               allow_cache=allow_cache)
    batches = batch_by_size(ds.ordered_indices(), ds.num_tokens,
                            max_tokens=batch_max_frames, required_batch_size_multiple=world)
    return ds, _data.shard_pairs(batches, rank, world)


_FIELDS = ("x_main", "y_main", "spk_main", "len_main", "x_sub", "y_sub", "spk_sub", "len_sub")


class PairBatchFeeder:
    """Host->HBM feeder for the training loop.  A reader thread loads and collates
    (collate_fn_syncmultitrack_acoustic, train_util.py:937-1019) the next `prefetch`
    batches into pinned host buffers while the GPU runs the current step; each batch
    is copied with non-blocking DMA on a dedicated copy stream and the consumer's
    stream waits on the copy's event, so file I/O, collation and PCIe transfer all
    overlap the step.  Yields dicts of device tensors named as _FIELDS (speaker ids as
    int64 (P, 1), lengths as int64 (P,)); with sort_tracks (the training loop's order)
    also "lengths" = max(L_main, L_sub) on the device, and "host_lengths" (numpy).

    The reader thread replaces the reference's DataLoader worker processes: np.load
    and np.pad release the GIL for the byte work, and pinned buffers are produced
    directly instead of through DataLoader's pin-memory thread."""

    def __init__(self, dataset, batches, reduction_factor=4, device="cuda", prefetch=2,
                 sort_tracks=True):
        self.dataset = dataset
        self.sort_tracks = sort_tracks
        self.batches = batches
        self.rf = reduction_factor
        self.device = torch.device(device)
        self.prefetch = max(1, int(prefetch))
        self.cuda = self.device.type == "cuda"
        if self.cuda and not torch.cuda.is_available():
            raise RuntimeError("PairBatchFeeder: a CUDA device was requested but none is visible")
        self.copy_stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.wait_s = 0.0  # host time the consumer spent waiting for the reader (diagnostic)

    def _host_batch(self, batch):
        cols = _data.collate_syncmultitrack_acoustic([self.dataset[i] for i in batch],
                                                     reduction_factor=self.rf)
        if self.sort_tracks:
            # train_acoustic_multitrack.py:472-483: each track sorted by its own lengths
            # (descending), then lengths = max(L0, L1) (:82)
            i0, i1, lmax = _data.sort_pair_batch(cols[3], cols[7])
            cols = tuple(c[i0] for c in cols[:4]) + tuple(c[i1] for c in cols[4:])
            cols = cols + (lmax,)
        out = {}
        for name, a in zip(_FIELDS + ("lengths",), cols):
            t = torch.from_numpy(np.ascontiguousarray(a))
            if name.startswith("spk"):
                t = t.to(torch.int64)
            out[name] = t.pin_memory() if self.cuda else t
        return out

    def __len__(self):
        return len(self.batches)

    def _start(self):
        q = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()

        def reader():
            try:
                for b in self.batches:
                    if stop.is_set():
                        return
                    q.put(self._host_batch(b))
            except BaseException as e:  # surfaced in the consumer
                q.put(e)
            q.put(None)

        th = threading.Thread(target=reader, daemon=True)
        th.start()
        return q, stop, th

    def prestart(self):
        """Start loading the NEXT pass's first batches now (train.train_epoch calls it once the
        last step of a pass is issued): the reader collates them while that step runs, so a
        new epoch does not begin with the GPU waiting for its first batch."""
        if getattr(self, "_next", None) is None:
            self._next = self._start()

    def close(self):
        """Stop a prestarted reader that will not be consumed."""
        started, self._next = getattr(self, "_next", None), None
        if started is not None:
            q, stop, th = started
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)

    def __iter__(self):
        started, self._next = getattr(self, "_next", None), None
        q, stop, th = started if started is not None else self._start()
        try:
            while True:
                t0 = time.perf_counter()
                hb = q.get()
                self.wait_s += time.perf_counter() - t0
                if hb is None:
                    break
                if isinstance(hb, BaseException):
                    raise hb
                yield self._to_device(hb)
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)

    def _to_device(self, hb):
        host_lengths = (hb["lengths"].numpy().copy() if "lengths" in hb
                        else np.maximum(hb["len_main"].numpy(), hb["len_sub"].numpy()))
        if not self.cuda:
            out = dict(hb)
        else:
            consumer = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(self.copy_stream):
                out = {k: v.to(self.device, non_blocking=True) for k, v in hb.items()}
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            consumer.wait_event(ev)
            for v in out.values():
                v.record_stream(consumer)
        out["host_lengths"] = host_lengths
        return out
