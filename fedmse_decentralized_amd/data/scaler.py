"""Host float64 feature scalers, bit-compatible with scikit-learn.

The reference wraps ``sklearn.preprocessing.StandardScaler`` /
``MinMaxScaler((0, 1))`` in ``IoTDataProccessor``
(`src/DataLoader/dataloader.py:32-58`): fit on the client's train split,
transform valid / test / abnormal / new-device splits, labels 0 for normal
and 1 for abnormal.  The same scaler (ddof=0) standardises the CEN latents
(`src/Model/Centroid.py:12-25`).

These are re-implementations of sklearn's algorithms (same accumulation
order: mean of the column sums, variance with the "corrected two-pass"
update of ``_incremental_mean_and_var``; near-zero scales replaced by 1) so
that preprocessing matches the reference bit-for-bit without calling sklearn
on the hot path.  Parity is pinned by ``tests/test_data.py``.
"""
from __future__ import annotations

import numpy as np

_EPS64 = np.finfo(np.float64).eps


def _handle_zeros_in_scale(scale: np.ndarray) -> np.ndarray:
    scale = scale.copy()
    constant_mask = scale < 10 * _EPS64
    scale[constant_mask] = 1.0
    return scale


def column_mean_var(X: np.ndarray):
    """sklearn ``_incremental_mean_and_var`` from an empty state (ddof=0)."""
    X = np.asarray(X)
    n = X.shape[0]
    new_sum = np.sum(X, axis=0, dtype=np.float64)
    mean = new_sum / n
    temp = X - mean
    correction = np.sum(temp, axis=0, dtype=np.float64)
    temp = temp * temp
    unnorm = np.sum(temp, axis=0, dtype=np.float64) - correction ** 2 / n
    var = unnorm / n
    return mean, var


class StandardScaler:
    def __init__(self):
        self.mean_ = None
        self.var_ = None
        self.scale_ = None

    def fit(self, X):
        X = np.asarray(X, dtype=np.float64)
        n = X.shape[0]
        self.mean_, self.var_ = column_mean_var(X)
        # near-constant detection on the raw variance (Chan-Golub-LeVeque bound)
        upper = n * _EPS64 * self.var_ + (n * self.mean_ * _EPS64) ** 2
        scale = np.sqrt(self.var_)
        scale[self.var_ <= upper] = 1.0
        self.scale_ = scale
        return self

    def transform(self, X):
        X = np.array(X, dtype=np.float64, copy=True)
        X -= self.mean_
        X /= self.scale_
        return X

    def fit_transform(self, X):
        return self.fit(X).transform(X)


class MinMaxScaler:
    def __init__(self, feature_range=(0, 1)):
        self.feature_range = feature_range

    def fit(self, X):
        X = np.asarray(X, dtype=np.float64)
        self.data_min_ = np.nanmin(X, axis=0)
        self.data_max_ = np.nanmax(X, axis=0)
        data_range = self.data_max_ - self.data_min_
        lo, hi = self.feature_range
        self.scale_ = (hi - lo) / _handle_zeros_in_scale(data_range)
        self.min_ = lo - self.data_min_ * self.scale_
        return self

    def transform(self, X):
        X = np.array(X, dtype=np.float64, copy=True)
        X *= self.scale_
        X += self.min_
        return X

    def fit_transform(self, X):
        return self.fit(X).transform(X)


class IoTDataProcessor:
    """Scaler + label generator (reference ``IoTDataProccessor``)."""

    def __init__(self, scaler: str = "standard"):
        if scaler == "standard":
            self.scaler = StandardScaler()
        elif scaler == "minmax":
            self.scaler = MinMaxScaler((0, 1))
        else:
            raise ValueError(f"unknown scaler {scaler!r}")

    def transform(self, X, type: str = "normal"):
        data = self.scaler.transform(X)
        label = np.zeros(len(data), dtype=np.int64) if type == "normal" else np.ones(len(data), dtype=np.int64)
        return data, label

    def fit_transform(self, X):
        self.scaler.fit(X)
        return self.transform(X, "normal")

    def get_metadata(self):
        return {"mean": getattr(self.scaler, "mean_", None), "std": getattr(self.scaler, "scale_", None)}
