"""Distribution-similarity utilities and the weights of the ``fusion_avg`` rule.

Reference: `src/Utils/utils.py:10-53` (dead code in the reference's run path;
its only consumer was the deleted ``GlobalAggregator.fusion_avg``, whose
behaviour is reconstructed from the strings of
`src/Trainer/__pycache__/global_aggregator.cpython-313.pyc`):

* ``similarity_score(dev_kde_scores, data)`` — Jensen-Shannon distance
  between the (exponentiated) log-densities of a Gaussian KDE fitted on the
  dev set and of a Gaussian KDE fitted on ``data`` (Scott bandwidth), each
  evaluated on its own samples;
* ``kl_divergence`` / ``js_divergence`` — closed forms for multivariate
  Gaussians given by mean and covariance.

``fusion_weights`` turns per-model similarity scores into aggregation
weights: a model whose reconstruction of the dev set is distributed like the
dev set (small JS distance) gets a large weight, ``w_k ∝ 1 / (s_k + eps)``.
KDE on the host is quadratic in the number of rows, so callers subsample
(``ExperimentConfig.fusion_max_rows``).  No reference fixture pins the
numbers ("parity unpinned"); tests check the closed forms and invariants.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


def kde_log_density(data: np.ndarray) -> np.ndarray:
    """Gaussian KDE (Scott bandwidth) fitted on ``data`` and scored on it."""
    from sklearn.neighbors import KernelDensity

    x = np.asarray(data, dtype=np.float64)
    return KernelDensity(kernel="gaussian", bandwidth="scott").fit(x).score_samples(x)


def similarity_score(dev_kde_scores: np.ndarray, dataset_2: np.ndarray) -> float:
    from scipy.spatial.distance import jensenshannon

    s2 = kde_log_density(dataset_2)
    n = min(len(dev_kde_scores), len(s2))
    p = np.exp(np.asarray(dev_kde_scores[:n], dtype=np.float64))
    q = np.exp(s2[:n])
    return float(jensenshannon(p, q))


def kl_divergence(p_mean, p_cov, q_mean, q_cov) -> float:
    """KL(P || Q) of two multivariate Gaussians."""
    p_mean, q_mean = np.asarray(p_mean, np.float64), np.asarray(q_mean, np.float64)
    p_cov, q_cov = np.asarray(p_cov, np.float64), np.asarray(q_cov, np.float64)
    k = p_mean.shape[0]
    q_inv = np.linalg.inv(q_cov)
    diff = q_mean - p_mean
    _, logdet_q = np.linalg.slogdet(q_cov)
    _, logdet_p = np.linalg.slogdet(p_cov)
    return float(0.5 * (np.trace(q_inv @ p_cov) + diff @ q_inv @ diff - k + (logdet_q - logdet_p)))


def js_divergence(p_mean, p_cov, q_mean, q_cov) -> float:
    """JS divergence via the moment-matched mixture Gaussian M = N((mu_p+mu_q)/2, (S_p+S_q)/2)."""
    p_mean, q_mean = np.asarray(p_mean, np.float64), np.asarray(q_mean, np.float64)
    m_mean = 0.5 * (p_mean + q_mean)
    m_cov = 0.5 * (np.asarray(p_cov, np.float64) + np.asarray(q_cov, np.float64))
    return 0.5 * (kl_divergence(p_mean, p_cov, m_mean, m_cov) + kl_divergence(q_mean, q_cov, m_mean, m_cov))


def fusion_weights(sim_scores: Sequence[float], eps: float = 1e-12) -> np.ndarray:
    s = np.asarray(sim_scores, dtype=np.float64)
    inv = 1.0 / (np.where(np.isfinite(s), s, np.inf) + eps)
    tot = inv.sum()
    if not np.isfinite(tot) or tot <= 0:
        return np.full(len(s), 1.0 / max(len(s), 1))
    return inv / tot
