"""Feature scalers of the NNSVS pipeline and the residual-F0 constant injection.

The recipe normalises inputs with sklearn MinMaxScaler and outputs with StandardScaler,
saved as joblib pickles (recipes/_common/spsvs/feature_generation_multitrack.sh:30-55).
Pickles are not loaded here (they execute code): a scaler is built from its fitted
arrays -- from any object exposing sklearn's fitted attributes (``from_fitted``), or from
an ``.npz`` of them (``load_npz`` / ``save_npz``).  transform / inverse_transform follow
sklearn's arithmetic: in-place ops of the float64 statistics on a copy of the input in its
own float dtype (numpy computes each op in float64 and rounds into the input dtype).

``check_resf0_config`` is nnsvs/train_util.py:1668-1770: it injects in_lf0_min / max from
the input scaler's data range and out_lf0_mean / scale from the output scaler into a
residual-F0 model whose values are unset, and rejects inconsistent ones.
"""
import numpy as np


class StandardScaler:
    """sklearn.preprocessing.StandardScaler (fitted): x' = (x - mean_) / scale_."""

    kind = "standard"

    def __init__(self, mean_, var_, scale_=None):
        self.mean_ = np.asarray(mean_, dtype=np.float64)
        self.var_ = np.asarray(var_, dtype=np.float64)
        self.scale_ = np.sqrt(self.var_) if scale_ is None else np.asarray(scale_, np.float64)

    def transform(self, x):
        x = np.array(x, dtype=_fdt(x), copy=True)
        x -= self.mean_
        x /= self.scale_
        return x

    def inverse_transform(self, x):
        x = np.array(x, dtype=_fdt(x), copy=True)
        x *= self.scale_
        x += self.mean_
        return x

    def arrays(self):
        return dict(kind=np.array("standard"), mean_=self.mean_, var_=self.var_,
                    scale_=self.scale_)


class MinMaxScaler:
    """sklearn.preprocessing.MinMaxScaler (fitted): x' = x * scale_ + min_."""

    kind = "minmax"

    def __init__(self, min_, scale_, data_min_, data_max_, feature_range=(0.0, 1.0)):
        self.min_ = np.asarray(min_, dtype=np.float64)
        self.scale_ = np.asarray(scale_, dtype=np.float64)
        self.data_min_ = np.asarray(data_min_, dtype=np.float64)
        self.data_max_ = np.asarray(data_max_, dtype=np.float64)
        self.feature_range = tuple(float(v) for v in feature_range)

    def transform(self, x):
        x = np.array(x, dtype=_fdt(x), copy=True)
        x *= self.scale_
        x += self.min_
        return x

    def inverse_transform(self, x):
        x = np.array(x, dtype=_fdt(x), copy=True)
        x -= self.min_
        x /= self.scale_
        return x

    def arrays(self):
        return dict(kind=np.array("minmax"), min_=self.min_, scale_=self.scale_,
                    data_min_=self.data_min_, data_max_=self.data_max_,
                    feature_range=np.asarray(self.feature_range))


def _fdt(x):
    dt = np.asarray(x).dtype
    return dt if dt in (np.float32, np.float64) else np.float64


def from_fitted(obj):
    """A scaler from an object carrying sklearn's fitted attributes (no unpickling)."""
    if hasattr(obj, "data_min_"):
        return MinMaxScaler(obj.min_, obj.scale_, obj.data_min_, obj.data_max_,
                            getattr(obj, "feature_range", (0.0, 1.0)))
    if hasattr(obj, "mean_"):
        return StandardScaler(obj.mean_, obj.var_, obj.scale_)
    raise TypeError(f"not a fitted MinMax/Standard scaler: {type(obj).__name__}")


def save_npz(path, scaler):
    np.savez(path, **scaler.arrays())


def load_npz(path):
    z = np.load(path, allow_pickle=False)
    kind = str(z["kind"])
    if kind == "standard":
        return StandardScaler(z["mean_"], z["var_"], z["scale_"])
    if kind == "minmax":
        return MinMaxScaler(z["min_"], z["scale_"], z["data_min_"], z["data_max_"],
                            tuple(z["feature_range"]))
    raise ValueError(f"unknown scaler kind {kind!r}")


RESF0_KEYS = ("in_lf0_min", "in_lf0_max", "out_lf0_mean", "out_lf0_scale")


def check_resf0_config(model, in_scaler, out_scaler, in_lf0_idx, in_rest_idx, out_lf0_idx,
                       netG=None):
    """nnsvs/train_util.py:1668-1770.  Injects the scaler-derived constants into ``model``
    where they are None, raises ValueError when a set value disagrees with the scalers (or
    an index disagrees with the data config), and writes the final values into the
    ``netG`` config dict when given.  Returns the four values."""
    if in_scaler is None or out_scaler is None:
        raise ValueError("in_scaler and out_scaler must be specified")
    if hasattr(model, "module"):  # DataParallel / DDP (train_util.py:1673-1674)
        model = model.module
    if in_lf0_idx is None or in_rest_idx is None or out_lf0_idx is None:
        raise ValueError("in_lf0_idx, in_rest_idx and out_lf0_idx must be specified")
    ok = True
    if getattr(model, "in_lf0_idx", in_lf0_idx) != in_lf0_idx:
        ok = False
    if getattr(model, "out_lf0_idx", out_lf0_idx) != out_lf0_idx:
        ok = False
    if hasattr(model, "in_lf0_min") and hasattr(model, "in_lf0_max"):
        if model.in_lf0_min is None or model.in_lf0_max is None:
            model.in_lf0_min = in_scaler.data_min_[in_lf0_idx]
            model.in_lf0_max = in_scaler.data_max_[in_lf0_idx]
        ok &= bool(np.allclose(model.in_lf0_min, in_scaler.data_min_[model.in_lf0_idx]))
        ok &= bool(np.allclose(model.in_lf0_max, in_scaler.data_max_[model.in_lf0_idx]))
    if hasattr(model, "out_lf0_mean") and hasattr(model, "out_lf0_scale"):
        if model.out_lf0_mean is None or model.out_lf0_scale is None:
            model.out_lf0_mean = float(out_scaler.mean_[out_lf0_idx])
            model.out_lf0_scale = float(out_scaler.scale_[out_lf0_idx])
        ok &= bool(np.allclose(model.out_lf0_mean, out_scaler.mean_[model.out_lf0_idx]))
        ok &= bool(np.allclose(model.out_lf0_scale, out_scaler.scale_[model.out_lf0_idx]))
    if not ok:
        raise ValueError("The model config has wrong configurations.")
    vals = {}
    for key in RESF0_KEYS:
        if hasattr(model, key):
            vals[key] = float(getattr(model, key))
            if netG is not None:
                netG[key] = vals[key]
    return vals
