"""Plugin interface of the reference (nnsvs/base.py:6-157), unchanged.

Models built here are drop-in ``_target_`` replacements: same constructor
arguments, same ``forward``/``inference`` signatures, same ``state_dict``
keys, same ``PredictionType`` answers.
"""
from enum import Enum

from torch import nn


class PredictionType(Enum):
    """nnsvs/base.py:6-71."""
    DETERMINISTIC = 1
    PROBABILISTIC = 2
    MULTISTREAM_HYBRID = 3
    DIFFUSION = 4


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
