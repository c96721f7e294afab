"""Post-acoustic feature processing (gen.py:1314-1530, 1637-1694).

CPU: the oracle restatement against the reference's own postprocess_acoustic outputs
(tests/golden/postprocess.npz; gen_goldens.py case_postprocess: a 1500-frame song, a track
shorter than the smoothing guard, one just above it, no voiced frame, no note frame).
GPU: the postprocess.hip kernels against the same fixtures (fp64 filtering as scipy;
tolerances: rel 1e-5 for mgc / bap / lf0 -- float32 exp/log and float32 reductions in a
different order -- and V/UV bit-exact), the scaler kernels against the numpy scalers
(bit-exact), the standalone lowpass filter against scipy, and the WORLD codec round trip of
the vocoder input against the oracle (parity unpinned: pyworld is absent)."""
import types

import numpy as np
import pytest
import torch

from golden_util import load_case, rel
from oracle import postprocess_oracle as PO

CFG = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5],
                            has_dynamic_features=[False] * 4, num_windows=1)
KW = dict(frame_period=5, trajectory_smoothing=True, trajectory_smoothing_cutoff=50,
          trajectory_smoothing_cutoff_f0=20, vuv_threshold=0.3)


def _cases():
    a, meta = load_case("postprocess")
    return a, meta["cases"]


def _rel(x, y):
    x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
    return np.abs(x - y).max() / max(np.abs(y).max(), 1e-30)


@pytest.mark.parametrize("name", ["song", "short", "edge", "unvoiced", "nonote"])
def test_oracle_matches_reference(name):
    a, _ = _cases()
    p = name + "::"
    out = PO.postprocess_acoustic(a[p + "x"], a[p + "score"], a["gv"], **KW)
    for k, v in zip(("mgc", "lf0", "vuv", "bap"), out):
        assert v.shape == a[p + k].shape, k
        assert _rel(v, a[p + k]) < 1e-6, k


def test_interp1d_restatement_edges():
    f = np.array([0, 0, 5.0, 0, 0, 6.0, 0], dtype=np.float32)
    out = PO.interp1d(f.copy())
    np.testing.assert_allclose(out, [5, 5, 5, 5 + 1 / 3, 5 + 2 / 3, 6, 6], rtol=1e-6)
    z = np.zeros(4, dtype=np.float32)
    assert np.array_equal(PO.interp1d(z.copy()), z)


# ------------------------------------------------------------------------ GPU

@pytest.mark.gpu
@pytest.mark.parametrize("name", ["song", "short", "edge", "unvoiced", "nonote"])
def test_gpu_matches_reference(name):
    from ensemble_svs_with_interactions_amd import postprocess as PP
    a, _ = _cases()
    p = name + "::"
    scaler = types.SimpleNamespace(var_=a["gv"])
    out = PP.postprocess_acoustic("cuda", a[p + "x"], a[p + "score"][:, None], {}, {}, CFG,
                                  scaler, pitch_idx=0, **KW)
    for k, v in zip(("mgc", "lf0", "vuv", "bap"), out):
        ref = a[p + k]
        got = v.cpu().numpy()
        assert got.shape == ref.shape, k
        if k == "vuv":
            assert np.array_equal(got, ref)
        else:
            assert _rel(got, ref) < 1e-5, (k, _rel(got, ref))


@pytest.mark.gpu
def test_gpu_lowpass_matches_scipy():
    from ensemble_svs_with_interactions_amd import postprocess as PP
    r = np.random.default_rng(3)
    x = r.standard_normal((777, 9)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    PP.lowpass_filter(xd, 200, cutoff=30)
    for c in range(9):
        ref = PO.lowpass_filter(x[:, c], 200, cutoff=30).astype(np.float32)
        assert _rel(xd[:, c].cpu().numpy(), ref) < 1e-6


@pytest.mark.gpu
def test_gpu_scalers_bitwise():
    from ensemble_svs_with_interactions_amd import postprocess as PP
    from ensemble_svs_with_interactions_amd import scalers
    r = np.random.default_rng(4)
    x = r.standard_normal((300, 67)).astype(np.float32)
    st = scalers.StandardScaler(r.standard_normal(67), r.random(67) + 0.1)
    mm = scalers.MinMaxScaler(r.standard_normal(67), r.random(67) + 0.5, np.zeros(67),
                              np.ones(67))
    for sc in (st, mm):
        for fwd in (True, False):
            ref = sc.transform(x) if fwd else sc.inverse_transform(x)
            xd = torch.from_numpy(x).cuda()
            (PP.transform if fwd else PP.inverse_transform)(sc, xd)
            assert np.array_equal(xd.cpu().numpy(), ref), (sc.kind, fwd)


@pytest.mark.gpu
def test_gpu_usfgan_inputs():
    from ensemble_svs_with_interactions_amd import postprocess as PP
    r = np.random.default_rng(5)
    T = 400
    mgc = r.standard_normal((T, 60)).astype(np.float32)
    bap = np.clip(-20 + 25 * r.standard_normal((T, 5)), -60, 0).astype(np.float32)
    bap[::7] = -0.1 * r.random((len(bap[::7]), 5))  # mean > -0.5: unvoiced-like frames
    lf0 = (5 + r.random((T, 1))).astype(np.float32)
    vuv = r.random((T, 1)).astype(np.float32)
    d = lambda v: torch.from_numpy(v).cuda()  # noqa: E731
    f0, aux = PP.usfgan_inputs(d(mgc), d(lf0), d(vuv), d(bap), vuv_threshold=0.3)
    ref_bap = PO.world_bap_codec(bap)
    assert np.array_equal(aux[:, :60].cpu().numpy(), mgc)
    assert np.array_equal(aux[:, 60:].cpu().numpy(), ref_bap)
    ref_f0 = np.exp(lf0)
    ref_f0[vuv < 0.3] = 0
    assert _rel(f0.cpu().numpy(), ref_f0) < 1e-6
