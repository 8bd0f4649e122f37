"""Synthetic N-BaIoT / Kitsune-shaped federated intrusion data.

No dataset can be downloaded here, and parts of the reference's data are
missing (`.MISSING_LARGE_BLOBS`), so benchmarks run on
synthetic data with the *shape and statistics* of the shipped client CSVs:

* 115 features = 5 streams x 5 damped windows (lambda = 5, 3, 1, 0.1, 0.01)
  in N-BaIoT/Kitsune column order: MI_dir (weight, mean, variance), H (same),
  HH (weight, mean, std, magnitude, radius, covariance, pcc), HH_jit
  (weight, mean, variance), HpHp (as HH);
* benign traffic of 9 device profiles (the 9 N-BaIoT devices,
  `src/Configuration/nba-iot-training.json`), heavy-tailed variance/jitter
  columns (the real data reach ~1e17 in the jitter-variance columns);
* Mirai / Gafgyt-style attack profiles (floods with fixed packet sizes and
  very high rates, scans over many channels) plus a configurable share of
  low-and-slow "stealthy" rows that overlap benign traffic, so AUC is high
  but not trivially 1;
* per-client sizes drawn from the shipped IID-10 ranges (N-BaIoT: normal
  1,651-1,700, abnormal 3,182-3,303, test_normal 552; Kitsune: 925-994 /
  1,865-1,944 / 632);
* client mixtures over device profiles from Dirichlet(alpha): alpha=1000 for
  IID, alpha=0.5 for non-IID (label skew as in the data notebook).

Every client is generated from its own PCG64 stream (seed, client id), so a
rank can materialise any subset of clients without generating the rest.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from .partition import dirichlet_proportions

WINDOWS = (5.0, 3.0, 1.0, 0.1, 0.01)
N_FEATURES = 115


@dataclass
class ClientRaw:
    name: str
    normal: np.ndarray          # float64 [n_normal, 115], unscaled
    abnormal: np.ndarray        # float64 [n_abnormal, 115]
    test_normal: np.ndarray     # float64 [n_test_normal, 115] ("new device" benign rows)
    normal_profile: Optional[np.ndarray] = None   # device-profile id per normal row


@dataclass
class SyntheticSpec:
    kind: str = "nbaiot"            # "nbaiot" | "kitsune"
    n_clients: int = 10
    iid: bool = True
    alpha: Optional[float] = None   # default 1000 (IID) / 0.5 (non-IID)
    seed: int = 2025
    stealth_fraction: float = 0.03  # share of attack rows that mimic benign traffic
    normal_rows: Optional[Tuple[int, int]] = None
    abnormal_rows: Optional[Tuple[int, int]] = None
    test_normal_rows: Optional[int] = None
    name_prefix: Optional[str] = None

    def resolved(self) -> "SyntheticSpec":
        s = SyntheticSpec(**self.__dict__)
        if s.alpha is None:
            s.alpha = 1000.0 if s.iid else 0.5
        if s.kind == "nbaiot":
            s.normal_rows = s.normal_rows or (1651, 1700)
            s.abnormal_rows = s.abnormal_rows or (3182, 3303)
            s.test_normal_rows = s.test_normal_rows or 552
            s.name_prefix = s.name_prefix or "NBa-Synth-Client"
        elif s.kind == "kitsune":
            s.normal_rows = s.normal_rows or (925, 994)
            s.abnormal_rows = s.abnormal_rows or (1865, 1944)
            s.test_normal_rows = s.test_normal_rows or 632
            s.name_prefix = s.name_prefix or "Kitsune-Synth-Client"
        else:
            raise ValueError(f"unknown synthetic kind {s.kind!r}")
        return s


# --- traffic profiles -------------------------------------------------------
# (log10 packet rate [pkt/s], packet size mean [B], size std [B], jitter scale [s],
#  channel share, response ratio, pcc)
_NBAIOT_DEVICES = np.array([
    [0.3, 66.0, 4.0, 0.9, 0.8, 0.9, 0.10],    # doorbell
    [0.0, 98.0, 30.0, 1.5, 0.6, 0.7, 0.05],   # thermostat
    [1.2, 340.0, 180.0, 0.2, 0.5, 0.4, 0.30],  # baby monitor
    [0.6, 120.0, 60.0, 0.6, 0.7, 0.8, 0.15],  # webcam (PT737E)
    [0.7, 150.0, 70.0, 0.5, 0.7, 0.7, 0.20],  # webcam (PT838)
    [0.2, 80.0, 12.0, 1.1, 0.9, 0.9, 0.05],   # doorbell (Ennio)
    [1.5, 520.0, 260.0, 0.1, 0.4, 0.3, 0.35],  # security cam 1002
    [1.4, 480.0, 240.0, 0.12, 0.4, 0.3, 0.33],  # security cam 1003
    [0.9, 210.0, 110.0, 0.4, 0.6, 0.5, 0.25],  # webcam (XCS7)
])
_KITSUNE_DEVICES = np.array([
    [1.8, 700.0, 420.0, 0.05, 0.5, 0.2, 0.40],  # video stream
    [1.1, 180.0, 90.0, 0.3, 0.7, 0.6, 0.20],
    [0.5, 90.0, 25.0, 0.8, 0.8, 0.9, 0.08],
    [2.0, 900.0, 500.0, 0.03, 0.4, 0.15, 0.45],
    [0.8, 240.0, 130.0, 0.4, 0.6, 0.5, 0.22],
    [1.3, 420.0, 210.0, 0.15, 0.5, 0.35, 0.30],
    [0.4, 75.0, 10.0, 1.0, 0.9, 0.95, 0.04],
    [1.6, 610.0, 330.0, 0.08, 0.45, 0.25, 0.38],
    [0.9, 300.0, 160.0, 0.25, 0.55, 0.45, 0.27],
])
_ATTACKS = np.array([
    [3.6, 60.0, 0.5, 0.0005, 1.0, 0.05, 0.00],   # syn flood
    [3.4, 60.0, 0.5, 0.0008, 1.0, 0.0, 0.00],    # ack flood
    [3.8, 554.0, 1.0, 0.0003, 1.0, 0.0, 0.00],   # udp flood
    [3.7, 590.0, 1.0, 0.0003, 1.0, 0.0, 0.00],   # udpplain
    [2.2, 60.0, 2.0, 0.005, 0.02, 0.5, 0.01],    # scan (many channels)
    [2.6, 74.0, 3.0, 0.004, 0.05, 0.3, 0.02],    # gafgyt scan
    [3.0, 300.0, 150.0, 0.002, 0.3, 0.1, 0.05],  # combo
    [3.1, 1030.0, 20.0, 0.002, 0.9, 0.0, 0.00],  # junk
])


def _stream_features(logr, mu, sd, jit, share, resp, pcc, rng) -> np.ndarray:
    n = logr.shape[0]
    out = np.empty((n, N_FEATURES), dtype=np.float64)
    rate = 10.0 ** logr
    burst = rng.lognormal(0.0, 0.6, size=n)          # recent-activity multiplier
    tail = rng.pareto(2.5, size=n) + 1.0              # heavy-tailed variance inflation
    col = 0
    for stream in ("MI", "H", "HH", "HHjit", "HpHp"):
        sh = 1.0 if stream in ("MI", "H") else (share if stream != "HpHp" else share * 0.6)
        for li, lam in enumerate(WINDOWS):
            horizon = 1.0 / lam
            g = (len(WINDOWS) - li) / len(WINDOWS)        # short windows follow bursts
            w = rate * horizon * sh * burst ** g * rng.lognormal(0.0, 0.05, size=n)
            w = np.maximum(w, 1.0 + 1e-3 * rng.random(n))
            mdrift = 1.0 + 0.02 * (1.0 - g) * rng.standard_normal(n)
            m = mu * mdrift
            var = (sd * (1.0 + 0.3 * (1.0 - g) * (tail - 1.0))) ** 2 + 1e-12 * rng.random(n)
            if stream in ("MI", "H"):
                out[:, col:col + 3] = np.stack([w, m, var], 1)
                col += 3
            elif stream == "HHjit":
                jm = jit * horizon * (1.0 + 0.1 * rng.standard_normal(n)) * burst ** (-g)
                jv = (jit * horizon) ** 2 * tail ** (2.0 + 2.0 * (1.0 - g))
                out[:, col:col + 3] = np.stack([w, np.abs(jm), jv], 1)
                col += 3
            else:
                m_in = m * resp
                std = np.sqrt(var)
                std_in = std * resp
                mag = np.sqrt(m * m + m_in * m_in)
                rad = np.sqrt(var + std_in ** 2)
                p = np.clip(pcc + 0.05 * rng.standard_normal(n), -1.0, 1.0)
                cov = p * std * std_in
                out[:, col:col + 7] = np.stack([w, m, std, mag, rad, cov, p], 1)
                col += 7
    assert col == N_FEATURES
    return out


def _sample_rows(profiles: np.ndarray, ids: np.ndarray, rng: np.random.Generator, spread: float = 1.0) -> np.ndarray:
    P = profiles[ids]
    n = ids.shape[0]
    logr = P[:, 0] + spread * 0.25 * rng.standard_normal(n)
    mu = P[:, 1] * np.exp(spread * 0.08 * rng.standard_normal(n))
    sd = P[:, 2] * np.exp(spread * 0.15 * rng.standard_normal(n))
    jit = P[:, 3] * np.exp(spread * 0.2 * rng.standard_normal(n))
    share = np.clip(P[:, 4] * np.exp(0.1 * rng.standard_normal(n)), 1e-3, 1.0)
    resp = np.clip(P[:, 5] + 0.05 * rng.standard_normal(n), 0.0, 2.0)
    return _stream_features(logr, mu, sd, jit, share, resp, P[:, 6], rng)


def generate_client(spec: SyntheticSpec, client: int) -> ClientRaw:
    s = spec.resolved()
    devices = _NBAIOT_DEVICES if s.kind == "nbaiot" else _KITSUNE_DEVICES
    # federation-level mixture (shared by all clients) from the spec seed
    fed_rng = np.random.Generator(np.random.PCG64([s.seed, 0xFED]))
    mix = dirichlet_proportions(s.n_clients, len(devices), s.alpha, fed_rng)
    atk_mix = dirichlet_proportions(s.n_clients, len(_ATTACKS), max(s.alpha, 1.0), fed_rng)
    rng = np.random.Generator(np.random.PCG64([s.seed, 1 + client]))
    n_norm = int(rng.integers(s.normal_rows[0], s.normal_rows[1] + 1))
    n_abn = int(rng.integers(s.abnormal_rows[0], s.abnormal_rows[1] + 1))
    n_tn = int(s.test_normal_rows)
    if not s.iid:
        # non-IID also skews sizes (notebook: 1,357 / 1,573 / 801 for client 1)
        n_norm = int(n_norm * rng.uniform(0.6, 1.2))
        n_abn = int(n_abn * rng.uniform(0.4, 1.1))
        n_tn = int(n_tn * rng.uniform(0.8, 1.5))
    dev_ids = rng.choice(len(devices), size=n_norm, p=mix[client])
    normal = _sample_rows(devices, dev_ids, rng)
    # "new device" benign rows: drawn from the federation-wide device pool
    pool = mix.mean(axis=0)
    tn_ids = rng.choice(len(devices), size=n_tn, p=pool / pool.sum())
    test_normal = _sample_rows(devices, tn_ids, rng)
    atk_ids = rng.choice(len(_ATTACKS), size=n_abn, p=atk_mix[client])
    abnormal = _sample_rows(_ATTACKS, atk_ids, rng, spread=1.5)
    n_stealth = int(round(s.stealth_fraction * n_abn))
    if n_stealth:
        # low-and-slow rows: benign-looking rate/size with mildly shifted stats
        st_ids = rng.choice(len(devices), size=n_stealth, p=mix[client])
        stealth = _sample_rows(devices, st_ids, rng, spread=1.6)
        stealth[:, 1::3] *= rng.uniform(1.05, 1.4, size=(n_stealth, 1))
        pos = rng.choice(n_abn, size=n_stealth, replace=False)
        abnormal[pos] = stealth
    return ClientRaw(name=f"{s.name_prefix}-{client + 1}", normal=normal, abnormal=abnormal,
                     test_normal=test_normal, normal_profile=dev_ids)


def generate_federation(spec: SyntheticSpec, clients: Optional[List[int]] = None) -> List[ClientRaw]:
    s = spec.resolved()
    ids = range(s.n_clients) if clients is None else clients
    return [generate_client(s, c) for c in ids]


def write_dataset(out_dir: str, spec: SyntheticSpec, config_name: Optional[str] = None) -> str:
    """Materialise a synthetic federation on disk in the reference's layout —
    headerless 115-column CSVs under ``Client-k/{normal,abnormal,test_normal}/data.csv``
    plus a device-list JSON with the schema of `src/Configuration/*.json`
     — so the CSV ingest path (``--config-file``) runs end to end
    without the reference's data.  Returns the JSON path."""
    import json
    import os

    data_dir = os.path.join(out_dir, "Data")
    cfg_dir = os.path.join(out_dir, "Configuration")
    os.makedirs(cfg_dir, exist_ok=True)
    devices = []
    for i, raw in enumerate(generate_federation(spec)):
        base = f"Client-{i + 1}"
        for split, arr in (("normal", raw.normal), ("abnormal", raw.abnormal), ("test_normal", raw.test_normal)):
            d = os.path.join(data_dir, base, split)
            os.makedirs(d, exist_ok=True)
            np.savetxt(os.path.join(d, "data.csv"), arr, delimiter=",", fmt="%.10g")
        devices.append({"id": i + 1, "name": raw.name, "normal_data_path": f"{base}/normal",
                        "abnormal_data_path": f"{base}/abnormal", "test_normal_data_path": f"{base}/test_normal"})
    name = config_name or f"synthetic-{spec.kind}-{spec.n_clients}clients.json"
    path = os.path.join(cfg_dir, name)
    # data_path is relative to the directory the driver resolves from (the JSON's parent's parent)
    with open(path, "w") as f:
        json.dump({"data_path": "Data", "devices_list": devices}, f, indent=4)
    return path
