"""Bit-exact integer/byte parity of the multi-track data path."""
import numpy as np

from ensemble_svs_with_interactions_amd import data
from golden_util import load_case


def test_pairing_matches_reference():
    _, meta = load_case("data_path")
    pairs, plens = data.pair_files(meta["files"], meta["file_lengths"])
    assert [list(p) for p in pairs] == meta["pairs"]
    assert [list(map(int, p)) for p in plens] == meta["pair_lengths"]


def test_collate_bit_exact():
    a, _ = load_case("data_path")
    batch = []
    i = 0
    while f"in{i}::x0" in a:
        s = a[f"in{i}::spk"]
        batch.append((a[f"in{i}::x0"], a[f"in{i}::y0"], int(s[0]), None,
                      a[f"in{i}::x1"], a[f"in{i}::y1"], int(s[1]), None))
        i += 1
    out = data.collate_syncmultitrack_acoustic(batch, reduction_factor=4)
    for j, o in enumerate(out):
        ref = a[f"collate{j}"]
        assert o.shape == ref.shape, j
        assert o.dtype == ref.dtype or (o.dtype == np.int64 and ref.dtype == np.int64), j
        assert np.array_equal(o, ref), j


def test_masks_and_pad_inference():
    a, meta = load_case("data_path")
    assert np.array_equal(data.make_non_pad_mask(a["mask_lengths"]), a["non_pad_mask"])
    from oracle.ensvs_oracle import pad_inference_lengths
    for T, pad in meta["pad_inference"].items():
        p, lens = pad_inference_lengths([int(T)], 4)
        assert p == pad and lens == [int(T) + pad]


def test_synthetic_batch_layout():
    b = data.synthetic_batch(4, 100, 1, lengths=[100, 96, 60, 80])
    assert list(b["lengths"]) == [100, 96, 80, 60]
    oh = b["x_main"][:, :, 3:50]
    assert set(np.unique(oh.sum(-1))) <= {0.0, 1.0}
    assert (b["x_main"][2, 80:] == 0).all() and (b["y_sub"][3, 60:] == 0).all()


def test_independent_track_sort_quirk():
    # train_acoustic_multitrack.py:472-483 sorts the two tracks independently
    i0, i1, lens = data.sort_pair_batch([10, 30, 20], [30, 10, 20])
    assert list(i0) == [1, 2, 0] and list(i1) == [0, 2, 1] and list(lens) == [30, 20, 10]


def test_onset_merge_collate_bit_exact():
    """Timing-path collate (collate_fn_syncmultitrack, train_util.py:776-934): rows of the
    two tracks aligned by note onset (ties merged), padded, masks and pre-merge lengths."""
    a, meta = load_case("onset_merge")
    for rf in meta["cases"]:
        batch, i = [], 0
        while f"rf{rf}_in{i}::x0" in a:
            g = lambda k: a[f"rf{rf}_in{i}::{k}"]  # noqa: E731
            s = g("spk")
            batch.append((g("x0"), g("y0"), int(s[0]), g("a"), g("x1"), g("y1"), int(s[1]),
                          g("b")))
            i += 1
        out = data.collate_syncmultitrack(batch, reduction_factor=rf)
        assert len(out) == 10
        for j, o in enumerate(out):
            ref = a[f"rf{rf}::out{j}"]
            assert o.shape == ref.shape, (rf, j)
            assert np.array_equal(o, ref), (rf, j)


def test_onset_merge_indices_edge_cases():
    # tie at the first note, one track exhausted first, identical tracks
    i0, i1 = data.onset_merge_indices([0, 5, 10], [0, 3, 10, 12])
    assert i0.tolist() == [0, -1, 1, 2, -1] and i1.tolist() == [0, 1, -1, 2, 3]
    i0, i1 = data.onset_merge_indices([2, 4], [2, 4])
    assert i0.tolist() == [0, 1] and i1.tolist() == [0, 1]
    x0 = np.arange(6, dtype=np.float32).reshape(3, 2)
    x1 = -np.arange(4, dtype=np.float32).reshape(2, 2) - 1
    n0, n1, m0, m1 = data.merge_tracks_by_onset(x0, x1, [0, 1, 2], [1, 3])
    assert m0.tolist() == [True, True, True, False] and m1.tolist() == [False, True, False, True]
    assert np.array_equal(n1[1], x1[0]) and np.array_equal(n0[3], np.zeros(2, np.float32))
