"""Plugin interface of the reference (nnsvs/base.py:6-157), unchanged.

Models built here are drop-in ``_target_`` replacements: same constructor
arguments, same ``forward``/``inference`` signatures, same ``state_dict``
keys, same ``PredictionType`` answers.

``PredictionType`` must compare equal to the reference's own enum, because the
reference's callers dispatch on it (train_acoustic_multitrack.py:120,
train_acoustic.py:81, gen.py:507/680/1249).  When nnsvs is importable (a user
switching ``_target_`` strings has it installed) its enum is used as is;
otherwise the fallback enum below compares equal, and hashes equal, to any
member of an enum class named ``PredictionType`` with the same member name.
"""
from enum import Enum

from torch import nn


class _PredictionType(Enum):
    """nnsvs/base.py:6-71 (values and names identical)."""
    DETERMINISTIC = 1
    PROBABILISTIC = 2
    MULTISTREAM_HYBRID = 3
    DIFFUSION = 4

    def __eq__(self, other):
        if isinstance(other, Enum) and type(other).__name__ == "PredictionType":
            return self.name == other.name and self.value == other.value
        return NotImplemented

    def __hash__(self):
        # Enum.__hash__ is hash(self._name_): members of the reference enum hash alike
        return hash(self._name_)


def _reference_enum():
    try:
        from nnsvs.base import PredictionType as Ref  # noqa: WPS433
    except Exception:  # nnsvs (or one of its dependencies) is not installed
        return None
    return Ref


PredictionType = _reference_enum() or _PredictionType


class BaseModel(nn.Module):
    """nnsvs/base.py:74-157."""

    def forward(self, x, lengths=None, y=None):
        raise NotImplementedError()

    def inference(self, x, lengths=None):
        return self(x, lengths)

    def preprocess_target(self, y):
        return y

    def prediction_type(self):
        return PredictionType.DETERMINISTIC

    def is_autoregressive(self):
        return False

    def has_residual_lf0_prediction(self):
        return False
