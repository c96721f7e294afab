"""The plugin boundary on CPU: PredictionType answers compare equal to the reference's
own enum (the reference's train_step / gen.py dispatch on them), and the C-ABI-free
parts of the drop-in contract (prediction types of every model class)."""
import importlib.util
import os

import pytest

from ensemble_svs_with_interactions_amd import base
from ensemble_svs_with_interactions_amd.base import PredictionType

REF_BASE = "/root/reference/nnsvs/base.py"


def _ref_enum():
    if not os.path.exists(REF_BASE):
        pytest.skip("reference checkout not present (build container only)")
    # nnsvs/base.py imports only enum and torch.nn: load that one file, not the package
    spec = importlib.util.spec_from_file_location("_ref_nnsvs_base", REF_BASE)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.PredictionType


def test_prediction_type_equals_reference_enum():
    Ref = _ref_enum()
    for name in ("DETERMINISTIC", "PROBABILISTIC", "MULTISTREAM_HYBRID", "DIFFUSION"):
        ours, ref = getattr(PredictionType, name), getattr(Ref, name)
        assert ours == ref and ref == ours
        assert not (ours != ref)
        assert ours in [ref] and ref in [ours]
        assert hash(ours) == hash(ref)
        assert {ref: 1}[ours] == 1
    assert PredictionType.DIFFUSION != Ref.MULTISTREAM_HYBRID
    assert Ref.DETERMINISTIC != PredictionType.PROBABILISTIC


def test_reference_dispatch_branch():
    """train_acoustic_multitrack.py:120 takes the multistream branch for our model."""
    Ref = _ref_enum()
    from ensemble_svs_with_interactions_amd import configs
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4, tiny=True))
    assert model.prediction_type() == Ref.MULTISTREAM_HYBRID
    assert model.mgc_model.prediction_type() == Ref.DIFFUSION
    assert model.vuv_model.prediction_type() == Ref.DETERMINISTIC
    assert model.has_residual_lf0_prediction() and model.is_autoregressive()


def test_fallback_enum_is_used_without_nnsvs():
    # this container has no importable nnsvs: the fallback enum is the one exported
    assert PredictionType is base._PredictionType or PredictionType.__module__ == "nnsvs.base"
