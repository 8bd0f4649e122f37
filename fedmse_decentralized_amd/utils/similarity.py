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

The ``*_t`` functions are the same computations in torch (float64, on any
device): the HIP engine's form, which runs on the GPU with the round's other
work (no host round trip, so the device-resident round protocol can use it):
the exact Gaussian-kernel sum instead of sklearn's tree (which, with its
default zero tolerances, sums the same terms), scipy's JS distance formula.
"""
from __future__ import annotations

import math
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


# ---- torch (device) forms ------------------------------------------------------

def kde_log_density_t(x):
    """``kde_log_density`` in torch float64: Scott bandwidth n^(-1/(d+4)),
    log of the mean normalised Gaussian kernel over all rows (self included)."""
    import torch

    x = x.to(torch.float64)
    n, d = x.shape
    h = float(n) ** (-1.0 / (d + 4))
    d2 = torch.cdist(x, x, compute_mode="donot_use_mm_for_euclid_dist").square()
    log_norm = 0.5 * d * math.log(2.0 * math.pi) + d * math.log(h) + math.log(n)
    return torch.logsumexp(d2 * (-0.5 / (h * h)), dim=1) - log_norm


def js_distance_t(log_p, log_q):
    """scipy.spatial.distance.jensenshannon(exp(log_p), exp(log_q)) (natural
    log) in torch: both normalised to sum 1, sqrt of the mean of the two
    relative entropies to the midpoint."""
    import torch

    n = min(log_p.shape[0], log_q.shape[0])
    p = torch.exp(log_p[:n].to(torch.float64))
    q = torch.exp(log_q[:n].to(torch.float64))
    p = p / p.sum()
    q = q / q.sum()
    m = (p + q) / 2.0

    def rel_entr(a, b):
        return torch.where(a > 0, a * torch.log(a / b), torch.zeros_like(a))

    return torch.sqrt((rel_entr(p, m).sum() + rel_entr(q, m).sum()) / 2.0)


def fusion_weights_t(sim_scores, eps: float = 1e-12):
    """``fusion_weights`` in torch, without a host decision: uniform weights
    when the inverse scores do not sum to a positive finite value."""
    import torch

    s = sim_scores.to(torch.float64)
    inv = 1.0 / (torch.where(torch.isfinite(s), s, torch.full_like(s, math.inf)) + eps)
    tot = inv.sum()
    ok = torch.isfinite(tot) & (tot > 0)
    return torch.where(ok, inv / tot, torch.full_like(inv, 1.0 / max(int(s.numel()), 1)))
