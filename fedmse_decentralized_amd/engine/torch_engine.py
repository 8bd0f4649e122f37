"""Pure-PyTorch engine: the reference-exact execution path.

Runs on CPU (tests, plumbing config 1 of BASELINE.json) or any torch device.
It is the numerical oracle the HIP kernels are tested against, so it follows
the reference math literally: sequential clients, canonical parameter
tensors, autograd, ``torch.optim.Adam``'s single-tensor update formula with
persistent state (`src/Trainer/client_trainer.py:66`, `:360-419`, Q10),
mean-of-batch-mean epoch losses, patience-based early stopping.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from ..models.layout import P_PAD, canonical_to_padded, padded_to_canonical
from ..models.reference import functional_forward, functional_loss, unflatten
from ..ops import _host
from .base import Engine, TrainHandle, TrainHParams, TrainResult


def _adam_update(p, g, m, v, step, hp: TrainHParams):
    """torch.optim.adam._single_tensor_adam (no weight decay, no amsgrad)."""
    m.lerp_(g, 1 - hp.beta1)
    v.mul_(hp.beta2).addcmul_(g, g, value=1 - hp.beta2)
    bc1 = 1 - hp.beta1 ** step
    bc2 = 1 - hp.beta2 ** step
    step_size = hp.lr / bc1
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(hp.eps)
    p.addcdiv_(m, denom, value=-step_size)


class TorchEngine(Engine):
    name = "torch"

    # -- training --------------------------------------------------------------
    def train_launch(self, local_ids: Sequence[int], hp: TrainHParams) -> TrainHandle:
        return TrainHandle(list(local_ids), [], self._train_eager(local_ids, hp))

    def train_collect(self, handle: TrainHandle, host=None) -> TrainResult:
        return handle.result

    def _train_eager(self, local_ids: Sequence[int], hp: TrainHParams) -> TrainResult:
        st = self.store
        D = self.dims.d_in
        k = len(local_ids)
        epochs_run = np.zeros(k, dtype=np.int64)
        best_epoch = np.full(k, -1, dtype=np.int64)
        tracking: List[List[Tuple[float, float]]] = []
        for i, c in enumerate(local_ids):
            flat = padded_to_canonical(st.params[c], self.dims)
            params = [t.clone() for t in unflatten(flat, self.dims)]
            for t in params:
                t.requires_grad_(True)
            m = [t.clone() for t in unflatten(padded_to_canonical(st.adam_m[c], self.dims), self.dims)]
            v = [t.clone() for t in unflatten(padded_to_canonical(st.adam_v[c], self.dims), self.dims)]
            anchor = [t.clone() for t in unflatten(padded_to_canonical(st.anchor[c], self.dims), self.dims)]
            step = int(st.adam_step[c].item())
            xt = st.rows("train", c)[:, :D]
            xv = st.rows("valid", c)[:, :D]
            B = hp.batch_size
            min_valid = float("inf")
            worse = 0
            track = []
            for ep in range(hp.epochs):
                epoch_loss = 0.0
                nb = 0
                for s in range(0, xt.shape[0], B):
                    x = xt[s:s + B]
                    z, y = functional_forward(params, x)
                    loss = functional_loss(x, y, z, hp.shrink_lambda)
                    if hp.fedprox_mu != 0.0:
                        prox = 0.0
                        for p_, a_ in zip(params, anchor):
                            prox = prox + torch.sum(torch.square(p_ - a_))
                        loss = loss + hp.fedprox_mu * prox
                    grads = torch.autograd.grad(loss, params)
                    step += 1
                    with torch.no_grad():
                        for p_, g_, m_, v_ in zip(params, grads, m, v):
                            _adam_update(p_, g_, m_, v_, step, hp)
                    epoch_loss += float(loss.item())
                    nb += 1
                epoch_loss /= max(nb, 1)
                with torch.no_grad():
                    vl = 0.0
                    nvb = 0
                    prox_v = 0.0
                    if hp.fedprox_mu != 0.0:
                        pv = 0.0
                        for p_, a_ in zip(params, anchor):
                            pv = pv + torch.sum(torch.square(p_ - a_))
                        prox_v = hp.fedprox_mu * pv
                    for s in range(0, xv.shape[0], B):
                        x = xv[s:s + B]
                        z, y = functional_forward(params, x)
                        loss = functional_loss(x, y, z, hp.shrink_lambda)
                        if hp.fedprox_mu != 0.0:
                            loss = loss + prox_v
                        vl += float(loss.item())
                        nvb += 1
                    vl = vl / nvb if nvb else float("nan")
                track.append((epoch_loss, vl))
                epochs_run[i] = ep + 1
                if vl < min_valid:
                    min_valid = vl
                    best_epoch[i] = ep
                    with torch.no_grad():
                        st.best[c].copy_(canonical_to_padded(torch.cat([p_.detach().reshape(-1) for p_ in params]), self.dims))
                    worse = 0
                else:
                    worse += 1
                    if worse >= hp.patience:
                        break
            with torch.no_grad():
                st.params[c].copy_(canonical_to_padded(torch.cat([p_.detach().reshape(-1) for p_ in params]), self.dims))
                st.adam_m[c].copy_(canonical_to_padded(torch.cat([t.reshape(-1) for t in m]), self.dims))
                st.adam_v[c].copy_(canonical_to_padded(torch.cat([t.reshape(-1) for t in v]), self.dims))
                st.adam_step[c] = step
            tracking.append(track)
        return TrainResult(list(local_ids), epochs_run, tracking, best_epoch)

    # -- inference primitives ----------------------------------------------------
    def forward_rows(self, params, items, want_sse=True, want_latent=False):
        D = self.dims.d_in
        sse_out, lat_out = [], []
        cache = {}
        with torch.no_grad():
            for row, data in items:
                if row not in cache:
                    cache[row] = unflatten(padded_to_canonical(params[row], self.dims), self.dims)
                x = data[:, :D]
                z, y = functional_forward(cache[row], x)
                if want_sse:
                    sse_out.append(((y - x) ** 2).sum(dim=1))
                if want_latent:
                    lat_out.append(z)
        return sse_out, lat_out

    def weighted_sum(self, stack, weights):
        w = torch.tensor(list(weights), dtype=torch.float32, device=stack.device)
        # sequential accumulation in the given order (deterministic on every rank)
        out = torch.zeros(stack.shape[1], dtype=torch.float32, device=stack.device)
        for k in range(stack.shape[0]):
            out = out + stack[k] * w[k]
        return out

    def param_drift(self, hist, new):
        a = padded_to_canonical(hist, self.dims)
        b = padded_to_canonical(new.unsqueeze(0), self.dims)
        from ..models.layout import padded_index
        _, segs = padded_index(self.dims)
        diff = a - b
        tot = torch.zeros(a.shape[0], dtype=torch.float32, device=a.device)
        for s, e in segs:
            tot = tot + torch.linalg.vector_norm(diff[:, s:e], dim=1)
        return tot

    def cen_scores(self, train_lat, test_lat):
        out = []
        for tr, te in zip(train_lat, test_lat):
            trn = tr.detach().cpu().numpy().astype(np.float32)
            ten = te.detach().cpu().numpy().astype(np.float32)
            out.append(torch.from_numpy(cen_score_numpy(trn, ten)))
        return out

    def auc(self, scores, labels):
        res = []
        for s, l in zip(scores, labels):
            sn = np.nan_to_num(s.detach().cpu().numpy().astype(np.float64))
            ln = l.detach().cpu().numpy() if torch.is_tensor(l) else np.asarray(l)
            res.append(_host.roc_auc(sn, ln))
        return np.asarray(res, dtype=np.float64)

    def standardize_ddof1(self, x):
        D = self.dims.d_in
        xr = x[:, :D]
        mean = xr.mean(dim=0, keepdim=True)
        std = xr.std(dim=0, keepdim=True) + 1e-8
        out = torch.zeros_like(x)
        out[:, :D] = (xr - mean) / std
        return out


def cen_score_numpy(train_lat: np.ndarray, test_lat: np.ndarray) -> np.ndarray:
    """SAE-CEN anomaly score (reference ``CentroidBasedOneClassClassifier``,
    `src/Model/Centroid.py:15-35`): StandardScaler fit on the train latents
    (float64 accumulation, float32 in-place transform, as sklearn does on a
    float32 array), Euclidean distance to the origin in float64 (cdist)."""
    from ..data.scaler import StandardScaler

    sc = StandardScaler().fit(train_lat)
    t = test_lat.astype(np.float32).copy()
    t -= sc.mean_          # numpy in-place: computed in float64, stored as float32
    t /= sc.scale_
    t64 = t.astype(np.float64)
    return np.sqrt(np.sum(t64 * t64, axis=1))
