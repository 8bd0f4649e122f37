"""ctypes bindings of ``libfedmx_hip.so`` (hand-written gfx950 kernels).

The library has a plain C ABI (no torch headers); device memory is owned by
torch tensors and passed as raw pointers together with the current HIP
stream, so the kernels interleave correctly with torch work on that stream.
Work lists (forward row blocks, CEN / AUC jobs) are small descriptor arrays
built on the host and copied to the device per call.

Loading fails loudly: on a GPU box the HIP engine must run these kernels,
never a silent PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import build

_lock = threading.Lock()
_lib = None

FWD_DTYPE = np.dtype([
    ("params", "<u8"), ("x", "<u8"), ("sse", "<u8"), ("lat", "<u8"),
    ("nrows", "<i4"), ("lat_stride", "<i4"), ("d_in", "<i4"), ("latent", "<i4"),
    ("hidden", "<i4"), ("pad0", "<i4"), ("pad1", "<i8"),
])
CEN_DTYPE = np.dtype([
    ("train_lat", "<u8"), ("test_lat", "<u8"), ("out", "<u8"),
    ("n_train", "<i4"), ("n_test", "<i4"), ("latent", "<i4"), ("stride", "<i4"),
])
AUC_DTYPE = np.dtype([
    ("score", "<u8"), ("label", "<u8"), ("out", "<u8"),
    ("n", "<i4"), ("score_is_f64", "<i4"), ("score_scale", "<f4"), ("pad", "<i4"),
])

FWD_ROWS_PER_BLOCK = 256   # 4 waves x 4 tiles of 16 rows


class TrainArgs(ctypes.Structure):
    _fields_ = [
        ("params", ctypes.c_void_p), ("adam_m", ctypes.c_void_p), ("adam_v", ctypes.c_void_p),
        ("anchor", ctypes.c_void_p), ("best", ctypes.c_void_p), ("adam_step", ctypes.c_void_p),
        ("train_x", ctypes.c_void_p), ("train_off", ctypes.c_void_p),
        ("valid_x", ctypes.c_void_p), ("valid_off", ctypes.c_void_p),
        ("client_idx", ctypes.c_void_p), ("tracking", ctypes.c_void_p),
        ("epochs_run", ctypes.c_void_p), ("best_epoch", ctypes.c_void_p),
        ("epochs", ctypes.c_int32), ("batch", ctypes.c_int32), ("patience", ctypes.c_int32),
        ("d_in", ctypes.c_int32), ("hidden", ctypes.c_int32), ("latent", ctypes.c_int32),
        ("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
        ("eps", ctypes.c_float), ("lam", ctypes.c_float), ("mu", ctypes.c_float),
    ]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = build.HIP_LIB
            if not path.exists():
                # build in-tree on first use (hipcc cross-compiles for gfx950)
                build.build_hip()
            L = ctypes.CDLL(str(path))
            vp, i32 = ctypes.c_void_p, ctypes.c_int
            L.fedmx_forward_rows.argtypes = [vp, i32, vp]
            L.fedmx_weighted_sum.argtypes = [vp, vp, i32, i32, vp, vp]
            L.fedmx_param_drift.argtypes = [vp, i32, vp, vp, vp, vp]
            L.fedmx_standardize_ddof1.argtypes = [vp, i32, i32, vp, vp]
            L.fedmx_cen_score.argtypes = [vp, i32, vp]
            L.fedmx_auc.argtypes = [vp, i32, vp]
            L.fedmx_train.argtypes = [ctypes.POINTER(TrainArgs), i32, vp]
            L.fedmx_probe_mfma.argtypes = [vp, vp]
            for f in ("fedmx_forward_rows", "fedmx_weighted_sum", "fedmx_param_drift", "fedmx_standardize_ddof1",
                      "fedmx_cen_score", "fedmx_auc", "fedmx_train", "fedmx_probe_mfma"):
                getattr(L, f).restype = ctypes.c_int
            assert L.fedmx_fwd_desc_size() == FWD_DTYPE.itemsize
            assert L.fedmx_cen_desc_size() == CEN_DTYPE.itemsize
            assert L.fedmx_auc_desc_size() == AUC_DTYPE.itemsize
            assert L.fedmx_train_args_size() == ctypes.sizeof(TrainArgs)
            _lib = L
    return _lib


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _upload(arr: np.ndarray, device) -> torch.Tensor:
    buf = torch.from_numpy(arr.view(np.uint8).reshape(-1))
    return buf.to(device)


# ---------------------------------------------------------------------------
def forward_rows(params: torch.Tensor, items, dims, want_sse=True, want_latent=False):
    """items: sequence of (param_row, x[n, DP]).  Returns (sse list, latent list)."""
    dev = params.device
    n_items = len(items)
    sizes = [int(x.shape[0]) for _, x in items]
    tot = sum(sizes)
    sse_all = torch.empty(tot, dtype=torch.float32, device=dev) if want_sse else None
    lat_all = torch.empty(tot, dims.latent, dtype=torch.float32, device=dev) if want_latent else None
    nblocks = sum((n + FWD_ROWS_PER_BLOCK - 1) // FWD_ROWS_PER_BLOCK for n in sizes)
    desc = np.zeros(nblocks, dtype=FWD_DTYPE)
    P = params.shape[1]
    base_p = params.data_ptr()
    bi = 0
    off = 0
    for (row, x), n in zip(items, sizes):
        if x.dtype != torch.float32 or x.dim() != 2 or x.shape[1] != 128 or not x.is_contiguous():
            raise ValueError("forward_rows expects contiguous float32 [n, 128] inputs")
        if x.device != dev:
            raise ValueError("inputs must live on the params device")
        for r0 in range(0, n, FWD_ROWS_PER_BLOCK):
            nr = min(FWD_ROWS_PER_BLOCK, n - r0)
            d = desc[bi]
            d["params"] = base_p + 4 * P * int(row)
            d["x"] = x.data_ptr() + 4 * 128 * r0
            d["sse"] = (sse_all.data_ptr() + 4 * (off + r0)) if want_sse else 0
            d["lat"] = (lat_all.data_ptr() + 4 * dims.latent * (off + r0)) if want_latent else 0
            d["nrows"] = nr
            d["lat_stride"] = dims.latent
            d["d_in"] = dims.d_in
            d["latent"] = dims.latent
            d["hidden"] = dims.hidden
            bi += 1
        off += n
    if nblocks:
        dbuf = _upload(desc, dev)
        _check(lib().fedmx_forward_rows(dbuf.data_ptr(), nblocks, _stream(dev)), "fedmx_forward_rows")
    sse_l, lat_l = [], []
    off = 0
    for n in sizes:
        if want_sse:
            sse_l.append(sse_all[off:off + n])
        if want_latent:
            lat_l.append(lat_all[off:off + n])
        off += n
    return sse_l, lat_l


def weighted_sum(stack: torch.Tensor, weights: Sequence[float]) -> torch.Tensor:
    dev = stack.device
    K, P = stack.shape
    w = torch.tensor(np.asarray(weights, dtype=np.float32), device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    st = stack.contiguous()
    _check(lib().fedmx_weighted_sum(st.data_ptr(), w.data_ptr(), K, P, out.data_ptr(), _stream(dev)),
           "fedmx_weighted_sum")
    return out


def param_drift(hist: torch.Tensor, new: torch.Tensor, seg: torch.Tensor) -> torch.Tensor:
    dev = hist.device
    M = hist.shape[0]
    out = torch.empty(M, dtype=torch.float32, device=dev)
    h = hist.contiguous()
    nw = new.contiguous()
    _check(lib().fedmx_param_drift(h.data_ptr(), M, nw.data_ptr(), seg.data_ptr(), out.data_ptr(), _stream(dev)),
           "fedmx_param_drift")
    return out


def standardize_ddof1(x: torch.Tensor, d_in: int) -> torch.Tensor:
    dev = x.device
    y = torch.empty_like(x)
    _check(lib().fedmx_standardize_ddof1(x.data_ptr(), x.shape[0], d_in, y.data_ptr(), _stream(dev)),
           "fedmx_standardize_ddof1")
    return y


def cen_scores(train_lat: Sequence[torch.Tensor], test_lat: Sequence[torch.Tensor], latent: int):
    dev = train_lat[0].device
    n = len(train_lat)
    sizes = [int(t.shape[0]) for t in test_lat]
    out_all = torch.empty(sum(sizes), dtype=torch.float64, device=dev)
    desc = np.zeros(n, dtype=CEN_DTYPE)
    off = 0
    for i, (tr, te) in enumerate(zip(train_lat, test_lat)):
        desc[i]["train_lat"] = tr.data_ptr()
        desc[i]["test_lat"] = te.data_ptr()
        desc[i]["out"] = out_all.data_ptr() + 8 * off
        desc[i]["n_train"] = tr.shape[0]
        desc[i]["n_test"] = te.shape[0]
        desc[i]["latent"] = latent
        desc[i]["stride"] = tr.stride(0)
        off += te.shape[0]
    dbuf = _upload(desc, dev)
    _check(lib().fedmx_cen_score(dbuf.data_ptr(), n, _stream(dev)), "fedmx_cen_score")
    res, off = [], 0
    for s in sizes:
        res.append(out_all[off:off + s])
        off += s
    return res


def auc(scores: Sequence[torch.Tensor], labels: Sequence[torch.Tensor], f32_scale: float = 1.0) -> torch.Tensor:
    """Exact tie-aware ROC-AUC per (scores, labels) pair; returns float64 [n] on device.
    A value of -1 marks sets too large for the LDS sort (caller falls back to host)."""
    dev = scores[0].device
    n = len(scores)
    out = torch.empty(n, dtype=torch.float64, device=dev)
    desc = np.zeros(n, dtype=AUC_DTYPE)
    for i, (s, l) in enumerate(zip(scores, labels)):
        if l.dtype != torch.int32:
            raise ValueError("labels must be int32")
        desc[i]["score"] = s.data_ptr()
        desc[i]["label"] = l.data_ptr()
        desc[i]["out"] = out.data_ptr() + 8 * i
        desc[i]["n"] = s.shape[0]
        desc[i]["score_is_f64"] = 1 if s.dtype == torch.float64 else 0
        desc[i]["score_scale"] = f32_scale
    dbuf = _upload(desc, dev)
    _check(lib().fedmx_auc(dbuf.data_ptr(), n, _stream(dev)), "fedmx_auc")
    return out


def train(store, local_ids: Sequence[int], hp, dims):
    dev = store.params.device
    k = len(local_ids)
    idx = torch.tensor(list(local_ids), dtype=torch.int32, device=dev)
    tracking = torch.full((k, hp.epochs, 2), float("nan"), dtype=torch.float64, device=dev)
    epochs_run = torch.zeros(k, dtype=torch.int32, device=dev)
    best_epoch = torch.full((k,), -1, dtype=torch.int32, device=dev)
    if not hasattr(store, "_train_off_dev"):
        store._train_off_dev = torch.from_numpy(store.train_off).to(dev)
        store._valid_off_dev = torch.from_numpy(store.valid_off).to(dev)
    a = TrainArgs()
    a.params = store.params.data_ptr()
    a.adam_m = store.adam_m.data_ptr()
    a.adam_v = store.adam_v.data_ptr()
    a.anchor = store.anchor.data_ptr()
    a.best = store.best.data_ptr()
    a.adam_step = store.adam_step.data_ptr()
    a.train_x = store.train.data_ptr()
    a.train_off = store._train_off_dev.data_ptr()
    a.valid_x = store.valid.data_ptr()
    a.valid_off = store._valid_off_dev.data_ptr()
    a.client_idx = idx.data_ptr()
    a.tracking = tracking.data_ptr()
    a.epochs_run = epochs_run.data_ptr()
    a.best_epoch = best_epoch.data_ptr()
    a.epochs = hp.epochs
    a.batch = hp.batch_size
    a.patience = hp.patience
    a.d_in, a.hidden, a.latent = dims.d_in, dims.hidden, dims.latent
    a.lr, a.beta1, a.beta2, a.eps = hp.lr, hp.beta1, hp.beta2, hp.eps
    a.lam, a.mu = hp.shrink_lambda, hp.fedprox_mu
    rc = lib().fedmx_train(ctypes.byref(a), k, _stream(dev))
    if rc == -2:
        raise ValueError(f"fused training kernel supports batch sizes 1..16, got {hp.batch_size}")
    _check(rc, "fedmx_train")
    return tracking, epochs_run, best_epoch, idx


def probe_mfma(device) -> np.ndarray:
    """Runs one v_mfma_f32_16x16x4_f32 on known operands: returns D [16,16]
    computed from A[i][k] = i + 100k, B[k][j] = 1000k + j (asymmetric)."""
    out = torch.zeros(16 * 16, dtype=torch.float32, device=device)
    dummy = torch.zeros(1, dtype=torch.float32, device=device)
    _check(lib().fedmx_probe_mfma(out.data_ptr(), _stream(device)), "fedmx_probe_mfma")
    return out.view(16, 16).cpu().numpy()
