"""Aggregation rules as (source model, weight) plans.

The plan is computed on the host, identically on every rank; the engine then
executes ``sum_k w_k * theta_src(k)`` in plan order on the device
(``weighted_sum``), so every rank produces a bit-identical aggregate.

* ``avg`` / ``fedprox`` — plain mean over the selected clients: every weight
  is ``num_samples / total = 1 / K`` (`src/Trainer/client_trainer.py:107-113`,
  `:132-134`; FedProx's proximal term lives in local training).
* ``mse_avg`` (FedMSE) — weights proportional to ``1 / MSE`` of each model on
  the shared dev set (`src/Trainer/client_trainer.py:115-130`).
* ``fusion_avg`` — the legacy centralised aggregator's KDE/JS-similarity
  weighting: weights from ``utils.similarity.fusion_weights``
  of each model's dev-set reconstruction similarity, computed by the caller.

``compat="reference"`` reproduces the state-dict aliasing of the reference's
``fed_mse_avg``: the aggregator loads every gathered state into
its own module, and its own ``state_dict()`` entries alias that module, so

* its own entry is weighted with the MSE of the model loaded just before it
  (its own model if it is first), and
* its own entry's *values* at averaging time are those of the last model
  loaded (the last selected model, or the second to last if the aggregator is
  itself last).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

Plan = List[Tuple[int, float]]


def plan_mean(selected: Sequence[int], num_samples: Dict[int, float] = None) -> Plan:
    """FedAvg / FedProx.  The reference passes ``num_samples = 1.0`` for every
    model (Q13), i.e. a plain mean; ``num_samples`` (client -> training-set
    size) gives the textbook sample-weighted FedAvg instead."""
    if num_samples is None:
        k = len(selected)
        return [(cid, 1.0 / k) for cid in selected]
    tot = sum(float(num_samples[c]) for c in selected)
    return [(cid, float(num_samples[cid]) / tot) for cid in selected]


def plan_mse_avg(selected: Sequence[int], aggregator: int, dev_mse: Dict[int, float], compat: str = "reference") -> Plan:
    sel = list(selected)
    K = len(sel)
    raw: List[Tuple[int, float]] = []
    if compat == "reference" and aggregator in sel and K >= 1:
        a = sel.index(aggregator)
        for k, cid in enumerate(sel):
            if k != a:
                raw.append((cid, 1.0 / dev_mse[cid]))
                continue
            w_src = sel[a - 1] if a >= 1 else sel[a]
            if a != K - 1:
                v_src = sel[K - 1]
            else:
                v_src = sel[K - 2] if K >= 2 else sel[a]
            raw.append((v_src, 1.0 / dev_mse[w_src]))
    else:
        raw = [(cid, 1.0 / dev_mse[cid]) for cid in sel]
    tot = sum(w for _, w in raw)
    return [(cid, w / tot) for cid, w in raw]


def plan_fusion(selected: Sequence[int], sim: Dict[int, float] = None, weights: Sequence[float] = None) -> Plan:
    """``weights``: already formed (the HIP engine forms them on the device,
    ``utils.similarity.fusion_weights_t``); else from the similarity scores."""
    from ..utils.similarity import fusion_weights

    w = weights if weights is not None else fusion_weights([sim[c] for c in selected])
    return [(cid, float(x)) for cid, x in zip(selected, w)]


UPDATE_TYPES = ("avg", "fedprox", "mse_avg", "fusion_avg")


def make_plan(update_type: str, selected: Sequence[int], aggregator: int, dev_mse: Dict[int, float] = None,
              compat: str = "reference", sim: Dict[int, float] = None, num_samples: Dict[int, float] = None,
              fusion_w: Sequence[float] = None) -> Plan:
    if update_type in ("avg", "fedprox"):
        return plan_mean(selected, num_samples)
    if update_type == "mse_avg":
        return plan_mse_avg(selected, aggregator, dev_mse, compat)
    if update_type == "fusion_avg":
        return plan_fusion(selected, sim, fusion_w)
    raise ValueError(f"Unknown update type: {update_type}")
