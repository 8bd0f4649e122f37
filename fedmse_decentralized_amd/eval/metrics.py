"""Detection metrics (reference `src/Evaluator/evaluator.py:21-48`).

* ROC-AUC with sklearn ``roc_curve`` + ``auc`` semantics (positives = label 1,
  ties count one half, non-finite scores replaced by ``nan_to_num``).  The
  trapezoid area under sklearn's ROC is exactly the Mann-Whitney statistic
  with mid-ranks, which is what the host library and the device kernel
  compute; parity against sklearn is pinned in ``tests/test_metrics.py``.
* classification metrics at a fixed score threshold (F1 / precision / recall,
  ``score > 0.5`` -> anomaly, `evaluator.py:30-48`), sklearn zero-division
  conventions (0.0 with a warning there).
"""
from __future__ import annotations

import numpy as np

from ..ops import _host


def roc_auc(labels, scores) -> float:
    s = np.asarray(scores, dtype=np.float64)
    if not np.all(np.isfinite(s)):
        s = np.nan_to_num(s)
    return _host.roc_auc(s, np.asarray(labels))


def classification_metrics(labels, scores, threshold: float = 0.5):
    y = np.asarray(labels).astype(np.int64)
    pred = (np.asarray(scores) > threshold).astype(np.int64)
    tp = int(np.sum((pred == 1) & (y == 1)))
    fp = int(np.sum((pred == 1) & (y == 0)))
    fn = int(np.sum((pred == 0) & (y == 1)))
    precision = tp / (tp + fp) if (tp + fp) else 0.0
    recall = tp / (tp + fn) if (tp + fn) else 0.0
    f1 = 2 * tp / (2 * tp + fp + fn) if (2 * tp + fp + fn) else 0.0
    return f1, precision, recall
