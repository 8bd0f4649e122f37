"""Engine interface and the device-resident client store.

An *engine* owns the clients hosted by one rank (one GPU): their datasets,
parameters and optimiser state, all resident on the device in
structure-of-arrays form, and exposes the compute the federated protocol
needs.  Two levels:

Primitives
  * ``train_launch`` / ``train_collect`` – local training of a set of clients
    (reference ``ClientTrainer.run``, `src/Trainer/client_trainer.py:360-419`);
  * ``forward_rows``   – per-row squared reconstruction error and/or latents of
    (parameter-vector, dataset) pairs (`client_trainer.py:208-247`, `:115-130`,
    `src/Trainer/model_verifier.py:86-99`, `src/Evaluator/evaluator.py:52-94`);
  * ``weighted_sum``   – FedAvg / MSEAvg reduction (`client_trainer.py:107-134`);
  * ``param_drift``    – verifier drift (`model_verifier.py:79-84`);
  * ``cen_scores`` + ``auc`` – SAE-CEN scoring and ROC-AUC
    (`src/Model/Centroid.py:15-35`, `src/Evaluator/evaluator.py:21-28`).

Round operations (what the federation calls; results stay on the device
until one ``fetch`` per protocol phase):
  * ``vote_scores`` – vote score on the standardised vote data + dev-set MSE
    for each given client;
  * ``verify_stats`` – MSE of the aggregate on the verification sets + drift
    against the previously received aggregates;
  * ``adopt`` – copy the aggregate into accepted clients (+ FedProx anchor);
  * ``evaluate`` – detection metric of every hosted client.

``TorchEngine`` implements the primitives with reference-exact PyTorch math;
``HipEngine`` runs everything on hand-written gfx950 kernels and never falls
back to torch for them.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.layout import DP, P_PAD, ModelDims, DEFAULT_DIMS, canonical_to_padded, padded_to_canonical


@dataclass
class TrainHParams:
    epochs: int
    batch_size: int = 12
    lr: float = 1e-3
    shrink_lambda: float = 0.0      # 0 for the plain AE
    fedprox_mu: float = 0.0         # 0 unless update_type == "fedprox"
    patience: int = 1
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8


@dataclass
class TrainResult:
    local_ids: List[int]
    epochs_run: np.ndarray               # int [k]
    tracking: List[List[Tuple[float, float]]]  # per client: [(train_loss, valid_loss)] per epoch
    best_epoch: np.ndarray               # int [k] (-1 if never improved)


@dataclass
class TrainHandle:
    local_ids: List[int]
    tensors: List[torch.Tensor] = field(default_factory=list)   # device results to fetch
    result: Optional[TrainResult] = None                        # filled synchronously by eager engines


def pad_features(x: np.ndarray) -> np.ndarray:
    """[n, D] -> [n, DP] float32, zero padded (aligned 512-byte rows)."""
    n, d = x.shape
    out = np.zeros((n, DP), dtype=np.float32)
    out[:, :d] = x
    return out


class ClientStore:
    """Structure-of-arrays state of the clients hosted by this rank.

    Parameters use the padded layout (``models/layout.py``).  Sized once per
    combination: ~37 KB x 5 state vectors per client plus its data
    (~2.2 MB per N-BaIoT client) — trivially resident in 288 GB of HBM.
    """

    def __init__(self, num_clients: int, device: torch.device):
        C = num_clients
        f32 = dict(dtype=torch.float32, device=device)
        self.num_clients = C
        self.device = device
        self.params = torch.zeros(C, P_PAD, **f32)
        self.adam_m = torch.zeros(C, P_PAD, **f32)
        self.adam_v = torch.zeros(C, P_PAD, **f32)
        self.adam_step = torch.zeros(C, dtype=torch.int32, device=device)
        self.anchor = torch.zeros(C, P_PAD, **f32)
        self.best = torch.zeros(C, P_PAD, **f32)
        self.train = self.valid = self.test = None
        self.train_off = self.valid_off = self.test_off = None
        self.test_label = None

    # zero rows after the last client's training rows: the helper-wave
    # kernel's batch loads read whole 12-row (batch <= 12) or 16-row (larger
    # batches) chunks without clamping rows past a client's end (those
    # columns are masked).  Contract checked by ops/_hip.TrainBuffers before
    # the first launch on a store: >= 15 rows after the last client, column
    # DP-1 of train/valid holding 1
    # (``bias_column_rows`` records which buffers _concat filled).
    TRAIN_TAIL_ROWS = 16

    @staticmethod
    def _concat(arrays: Sequence[np.ndarray], device, bias_column: bool = False, tail_rows: int = 0):
        offs = np.zeros(len(arrays) + 1, dtype=np.int64)
        for i, a in enumerate(arrays):
            offs[i + 1] = offs[i] + a.shape[0]
        parts = [pad_features(a) for a in arrays] + [np.zeros((tail_rows, DP), np.float32)]
        buf = np.concatenate(parts, 0)
        if bias_column:
            # the training kernels read X's padded column DP-1 as the constant 1
            # that feeds W1a's bias column: stored, so the helper-wave kernel
            # need not overwrite it after every batch load.  Every other reader
            # ignores the column (forward SSEs sum d < d_in, the oracle slices).
            buf[:, DP - 1] = 1.0
        return torch.from_numpy(buf).to(device), offs

    def load_data(self, train: Sequence[np.ndarray], valid: Sequence[np.ndarray],
                  test: Sequence[np.ndarray], test_label: Sequence[np.ndarray]):
        self.train, self.train_off = self._concat(train, self.device, bias_column=True,
                                                  tail_rows=self.TRAIN_TAIL_ROWS)
        self.valid, self.valid_off = self._concat(valid, self.device, bias_column=True)
        self.bias_column_rows = ("train", "valid")
        self.test, self.test_off = self._concat(test, self.device)
        lab = np.concatenate([np.asarray(l, dtype=np.int32) for l in test_label]) if test_label else np.zeros(0, np.int32)
        self.test_label = torch.from_numpy(lab).to(self.device)
        self.test_label_np = lab

    def rows(self, split: str, c: int) -> torch.Tensor:
        buf = getattr(self, split)
        off = getattr(self, split + "_off")
        return buf[int(off[c]):int(off[c + 1])]

    def labels(self, c: int) -> np.ndarray:
        return self.test_label_np[int(self.test_off[c]):int(self.test_off[c + 1])]

    def label_view(self, c: int) -> torch.Tensor:
        return self.test_label[int(self.test_off[c]):int(self.test_off[c + 1])]


def batch_mean_scores(sse: torch.Tensor, bs: int, d_in: int) -> Tuple[float, float]:
    """(mean over batches of the batch MSE, overall MSE) of a per-row SSE vector
    (`src/Trainer/client_trainer.py:226-241`)."""
    x = sse.detach().double().cpu().numpy()
    n = x.shape[0]
    if n == 0:
        return float("inf"), float("nan")
    tot, nb = 0.0, 0
    for s in range(0, n, bs):
        seg = x[s:s + bs]
        tot += float(seg.sum() / (seg.shape[0] * d_in))
        nb += 1
    return tot / nb, float(x.sum() / (n * d_in))


class Engine:
    name = "abstract"

    def __init__(self, dims: ModelDims = DEFAULT_DIMS, device: Optional[torch.device] = None):
        self.dims = dims
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.store: Optional[ClientStore] = None

    # -- setup -----------------------------------------------------------------
    def setup(self, train, valid, test, test_label, init_canonical: torch.Tensor):
        C = len(train)
        self.store = ClientStore(C, self.device)
        self.store.load_data(train, valid, test, test_label)
        p = canonical_to_padded(init_canonical.to(torch.float32), self.dims).to(self.device)
        self.store.params.copy_(p)
        self.store.anchor.copy_(p)  # FedProx anchor starts at the init weights (Q11)
        self.store.best.copy_(p)

    def to_device(self, x: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(pad_features(np.asarray(x, dtype=np.float32))).to(self.device)

    def canonical(self, padded: torch.Tensor) -> torch.Tensor:
        return padded_to_canonical(padded, self.dims)

    def fetch(self, tensors: Sequence[torch.Tensor]) -> List[np.ndarray]:
        """Device -> host for several results with (at most) one synchronisation."""
        return [t.detach().cpu().numpy() for t in tensors]

    # -- primitives (implemented by subclasses) --------------------------------
    def train(self, local_ids: Sequence[int], hp: TrainHParams) -> TrainResult:
        return self.train_collect(self.train_launch(local_ids, hp))

    def train_launch(self, local_ids: Sequence[int], hp: TrainHParams) -> TrainHandle:
        raise NotImplementedError

    def train_collect(self, handle: TrainHandle, host: Optional[List[np.ndarray]] = None) -> TrainResult:
        raise NotImplementedError

    def forward_rows(self, params: torch.Tensor, items: Sequence[Tuple[int, torch.Tensor]],
                     want_sse: bool = True, want_latent: bool = False):
        """For each (param_row, data[n, DP]) item: per-row SSE over the real
        D columns and/or latents [n, Z].  Returns (sse_list, latent_list)."""
        raise NotImplementedError

    def weighted_sum(self, stack: torch.Tensor, weights: Sequence[float]) -> torch.Tensor:
        raise NotImplementedError

    def param_drift(self, hist: torch.Tensor, new: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def cen_scores(self, train_lat: Sequence[torch.Tensor], test_lat: Sequence[torch.Tensor]) -> List[torch.Tensor]:
        raise NotImplementedError

    def auc(self, scores: Sequence[torch.Tensor], labels: Sequence[torch.Tensor]) -> np.ndarray:
        raise NotImplementedError

    def standardize_ddof1(self, x: torch.Tensor) -> torch.Tensor:
        """(x - mean) / (std_ddof1 + 1e-8) over the real D columns
        (`src/Trainer/client_trainer.py:220-223`)."""
        raise NotImplementedError

    # -- round operations (defaults in terms of the primitives) -----------------
    def vote_scores(self, local_rows: Sequence[int], vote_data: torch.Tensor, dev_set: Optional[torch.Tensor],
                    vote_bs: int) -> torch.Tensor:
        """float64 [k, 2]: (vote score on standardised vote data, dev-set MSE or nan)."""
        k = len(local_rows)
        out = torch.full((k, 2), float("nan"), dtype=torch.float64)
        if k == 0:
            return out
        vs = self.standardize_ddof1(vote_data)
        items = [(c, vs) for c in local_rows]
        if dev_set is not None:
            items += [(c, dev_set) for c in local_rows]
        sse, _ = self.forward_rows(self.store.params, items, want_sse=True)
        D = self.dims.d_in
        for i in range(k):
            out[i, 0] = batch_mean_scores(sse[i], vote_bs, D)[0]
            if dev_set is not None:
                out[i, 1] = batch_mean_scores(sse[k + i], 1 << 30, D)[1]
        return out

    def verify_stats(self, agg: torch.Tensor, datasets: Sequence[torch.Tensor], hist: Optional[torch.Tensor]):
        """(MSE of ``agg`` on each dataset [float64], drift of each hist row vs agg)."""
        aggp = agg.unsqueeze(0)
        sse, _ = self.forward_rows(aggp, [(0, x) for x in datasets], want_sse=True) if datasets else ([], None)
        D = self.dims.d_in
        mse = torch.tensor([batch_mean_scores(s, 1 << 30, D)[1] for s in sse], dtype=torch.float64)
        drift = self.param_drift(hist, agg) if hist is not None and hist.shape[0] else torch.zeros(0)
        return mse, drift

    def model_mse(self, local_rows: Sequence[int], datasets: Sequence[torch.Tensor]) -> np.ndarray:
        """float64 [k]: MSE of each local row's own current model on its dataset
        (thesis verification's old loss)."""
        if not len(local_rows):
            return np.zeros(0)
        sse, _ = self.forward_rows(self.store.params, list(zip(local_rows, datasets)), want_sse=True)
        D = self.dims.d_in
        return np.array([batch_mean_scores(s, 1 << 30, D)[1] for s in sse], dtype=np.float64)

    def adopt(self, local_rows: Sequence[int], agg: torch.Tensor, anchor: bool = True) -> None:
        st = self.store
        if not len(local_rows):
            return
        idx = torch.tensor(list(local_rows), dtype=torch.long, device=st.params.device)
        rows = agg.unsqueeze(0).expand(len(local_rows), -1)
        st.params.index_copy_(0, idx, rows)
        if anchor:
            st.anchor.index_copy_(0, idx, rows)

    def evaluate(self, model_type: str, metric: str = "AUC", keep_latents: bool = False):
        from ..eval.evaluator import evaluate_clients

        return evaluate_clients(self, list(range(self.store.num_clients)), model_type, metric, keep_latents)

    def synchronize(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
