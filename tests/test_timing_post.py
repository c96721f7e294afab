"""timing_post.postprocess_duration (nnsvs/gen.py:723-817) on hand-computed cases.
Parity UNPINNED: the reference needs nnmnkwii's HTSLabelFile, absent from this image, so
no reference output pins it; these cases check eq. (11), (12), (16), (17) and the label
bookkeeping as the reference code states them."""
import numpy as np

from ensemble_svs_with_interactions_amd.timing_post import get_note_indices, postprocess_duration

F = 50000  # one 5-ms frame in HTS units


def _score():
    # note 0: 2 phonemes over frames [0, 40); note 1: 3 phonemes over [40, 100)
    st = np.array([0, 0, 40, 40, 40]) * F
    en = np.array([40, 40, 100, 100, 100]) * F
    return st, en


def test_note_indices():
    assert get_note_indices(_score()[0]) == [0, 2]
    assert get_note_indices([]) == []
    assert get_note_indices([5, 5, 5]) == [0]


def test_zero_lag_proportional_durations():
    st, en = _score()
    d_hat = np.array([10.0, 30.0, 1.0, 1.0, 2.0])
    s, e, d = postprocess_duration(st, en, d_hat, np.zeros(2))
    # eq (12): note 0 -> 40 * (10, 30) / 40; note 1 -> 60 * (1, 1, 2) / 4
    assert d.tolist() == [10, 40, 15, 30, 60]
    assert s.tolist() == [0, 10 * F, 40 * F, 55 * F, 70 * F]
    assert e.tolist() == [10 * F, 40 * F, 55 * F, 70 * F, 100 * F]


def test_mdn_variance_scaling_and_fallback():
    st, en = _score()
    mu = np.array([15.0, 15.0, 10.0, 10.0, 10.0])
    var = np.array([1.0, 1.0, 1.0, 1.0, 2.0])
    s, e, d = postprocess_duration(st, en, (mu, var), np.zeros(2))
    # eq (17) rho = (40 - 30) / 2 = 5 -> (20, 20); (60 - 30) / 4 = 7.5 -> (17.5, 17.5, 25)
    assert d.tolist() == [20, 40, 18, 36, 61]  # np.round: 17.5 -> 18 (half to even)
    # a negative variance-scaled duration falls back to uniform scaling (eq 12 with mu)
    mu2 = np.array([35.0, 5.0, 10.0, 10.0, 10.0])
    var2 = np.array([0.1, 10.0, 1.0, 1.0, 1.0])
    _, _, d2 = postprocess_duration(st, en, (mu2, var2), np.zeros(2))
    assert d2[:2].tolist() == [35, 40]


def test_time_lag_moves_note_boundary():
    st, en = _score()
    d_hat = np.ones(5)
    lag = np.array([0.0, -4 * F])  # the second note starts 4 frames early
    s, e, d = postprocess_duration(st, en, d_hat, lag)
    # eq (11): L_hat(note 0) = 40 - (0 - (-4)) = 36, L_hat(note 1) = 60 - (-4) = 64
    assert d[:2].tolist() == [18, 36]
    assert s[2] == 36 * F and e[1] == 36 * F  # previous note's end follows the new start
    assert d[2:].tolist() == [21, 42, 63]  # 64/3 = 21.33 -> 21, 21, 21 (cumulative)
    assert e[-1] == s[2] + 63 * F  # rounding: 3 x 21 frames


def test_lag_clamped_to_previous_start_and_zero():
    st, en = _score()
    lag = np.array([-10 * F, -100 * F])  # would start before 0 / before the previous note
    s, _, _ = postprocess_duration(st, en, np.ones(5), lag)
    assert s[0] == 0
    assert s[2] > s[1]
