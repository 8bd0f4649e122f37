"""Data ingest: scaler parity with sklearn, split/RNG parity with the
reference's pandas pipeline (`src/main.py:126-223`), native CSV reader,
synthetic generator."""
import os

import numpy as np
import pandas as pd
import pytest
from sklearn.preprocessing import MinMaxScaler as SkMinMax
from sklearn.preprocessing import StandardScaler as SkStd

from fedmse_decentralized_amd.data.csv import load_data
from fedmse_decentralized_amd.data.partition import dirichlet_split, js_distance
from fedmse_decentralized_amd.data.prepare import prepare_federation, split_sizes
from fedmse_decentralized_amd.data.scaler import MinMaxScaler, StandardScaler
from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, generate_client, generate_federation
from fedmse_decentralized_amd.ops import _host

REF = "/root/reference"


def _heavy(n=500, d=20, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.lognormal(0, 3, size=(n, d)) * rng.choice([1, 1e6], size=d)
    X[:, 3] = 7.0          # constant column -> scale 1
    X[:, 5] = 1e-300       # near-constant
    return X


def test_standard_scaler_bit_parity_with_sklearn():
    X = _heavy()
    ours = StandardScaler().fit(X)
    sk = SkStd().fit(X)
    assert np.array_equal(ours.mean_, sk.mean_)
    assert np.array_equal(ours.var_, sk.var_)
    assert np.array_equal(ours.scale_, sk.scale_)
    Y = _heavy(seed=1)
    assert np.array_equal(ours.transform(Y), sk.transform(Y))


def test_standard_scaler_float32_latents_parity():
    rng = np.random.default_rng(3)
    Z = rng.normal(size=(300, 7)).astype(np.float32) * 5 + 2
    ours = StandardScaler().fit(Z)
    sk = SkStd().fit(Z)
    assert np.array_equal(ours.mean_, sk.mean_)
    assert np.array_equal(ours.scale_, sk.scale_)


def test_minmax_parity():
    X = _heavy()
    assert np.allclose(MinMaxScaler().fit_transform(X), SkMinMax((0, 1)).fit_transform(X), rtol=0, atol=1e-15)


def test_split_sizes():
    assert split_sizes(1691) == (676, 169, 676, 170)
    assert split_sizes(10) == (4, 1, 4, 1)


def _reference_pipeline(raws, seed):
    """The reference's pandas code path (src/main.py:131-223), verbatim in spirit."""
    np.random.seed(seed)
    infos = []
    for r in raws:
        normal = pd.DataFrame(r.normal).sample(frac=1).reset_index(drop=True)
        abnormal = pd.DataFrame(r.abnormal).sample(frac=1).reset_index(drop=True)
        n = len(normal)
        tr, va, de = int(0.4 * n), int(0.1 * n), int(0.4 * n)
        sc = SkStd().fit(normal[:tr])
        train = sc.transform(normal[:tr])
        valid = sc.transform(normal[tr:tr + va])
        test = sc.transform(normal[tr + va + de:])
        abn = sc.transform(abnormal)
        newn = sc.transform(pd.DataFrame(r.test_normal))
        test = np.concatenate([test, newn, abn])
        infos.append((train, valid, test, normal[tr + va:tr + va + de]))
    min_len = min(len(i[3]) for i in infos)
    dev = pd.concat([i[3].sample(n=min_len) for i in infos], axis=0)
    dev = SkStd().fit_transform(dev)
    return infos, dev


def test_prepare_matches_reference_pandas_pipeline():
    spec = SyntheticSpec(kind="nbaiot", n_clients=3, normal_rows=(120, 140), abnormal_rows=(200, 220),
                         test_normal_rows=30, seed=5)
    raws = generate_federation(spec)
    clients, dev = prepare_federation(raws, data_seed=1234)
    ref, ref_dev = _reference_pipeline(raws, 1234)
    for c, (tr, va, te, _) in zip(clients, ref):
        assert np.array_equal(c.train, tr.astype(np.float32))
        assert np.array_equal(c.valid, va.astype(np.float32))
        assert np.array_equal(c.test, te.astype(np.float32))
        n_norm_test = c.test.shape[0] - raws[clients.index(c)].abnormal.shape[0]
        assert (c.test_label[:n_norm_test] == 0).all() and (c.test_label[n_norm_test:] == 1).all()
    assert np.array_equal(dev, ref_dev.astype(np.float32))


def test_native_csv_reader_matches_pandas(tmp_path):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(300, 9)) * 10.0 ** rng.integers(-20, 20, size=(300, 9))
    X[0, 0] = 0.0
    p = tmp_path / "d"
    p.mkdir()
    pd.DataFrame(X).to_csv(p / "data.csv", header=False, index=False)
    ours = load_data(str(p), cache=False)
    ref = pd.read_csv(p / "data.csv", header=None, float_precision="round_trip").values
    assert np.array_equal(ours, ref)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "Data/N-BaIoT/IID-10-Client_Data/Client-1/normal")),
                    reason="reference data not mounted")
def test_native_csv_reader_on_reference_file():
    d = os.path.join(REF, "Data/N-BaIoT/IID-10-Client_Data/Client-1/normal")
    ours = load_data(d, cache=False)
    ref = pd.read_csv(os.path.join(d, "data.csv"), header=None, float_precision="round_trip").values
    assert ours.shape == (1691, 115)
    assert np.array_equal(ours, ref)


def test_synthetic_shapes_and_determinism():
    spec = SyntheticSpec(kind="nbaiot", n_clients=4, seed=9)
    a = generate_client(spec, 2)
    b = generate_client(spec, 2)
    assert np.array_equal(a.normal, b.normal) and np.array_equal(a.abnormal, b.abnormal)
    assert a.normal.shape[1] == 115 and 1651 <= a.normal.shape[0] <= 1700
    assert 3182 <= a.abnormal.shape[0] <= 3303 and a.test_normal.shape[0] == 552
    assert np.isfinite(a.normal).all() and np.isfinite(a.abnormal).all()
    k = generate_client(SyntheticSpec(kind="kitsune", n_clients=4, seed=9), 0)
    assert 925 <= k.normal.shape[0] <= 994 and k.test_normal.shape[0] == 632
    # heavy tails like the real jitter-variance columns
    assert a.normal.max() > 1e6


def test_dirichlet_split_and_js():
    rng = np.random.default_rng(0)
    labels = rng.integers(0, 5, size=5000)
    parts = dirichlet_split(labels, 10, 1000.0, rng)
    assert sum(len(p) for p in parts) == 5000
    assert len(np.unique(np.concatenate(parts))) == 5000
    parts_skew = dirichlet_split(labels, 10, 0.1, np.random.default_rng(1), min_count=10)
    for p in parts_skew:
        lab = labels[p]
        for cl in np.unique(lab):
            assert (lab == cl).sum() >= 10
    assert js_distance([1, 0], [1, 0]) == 0.0
    assert abs(js_distance([1, 0], [0, 1]) - 1.0) < 1e-12


def test_notebook_splitters():
    import numpy as np

    from fedmse_decentralized_amd.data import partition as P

    rng = np.random.default_rng(0)
    labels = rng.integers(0, 9, size=5000)
    # equal-size clients, each cycling through its classes
    parts = P.split_by_balancedness(labels, 10, 3, 1.0, np.random.default_rng(1))
    assert [len(p) for p in parts] == [500] * 10
    allidx = np.concatenate(parts)
    assert len(np.unique(allidx)) == allidx.size          # disjoint
    # skewed sizes: smallest first, geometric in balancedness
    parts = P.split_by_balancedness(labels, 10, 3, 0.8, np.random.default_rng(1))
    sizes = [len(p) for p in parts]
    assert sizes == sorted(sizes) and sizes[0] < sizes[-1]
    fr = 0.8 ** np.linspace(0, 9, 10)
    fr = 0.01 + 0.9 * fr / fr.sum()
    assert sizes == [int(np.floor(f * 5000)) for f in fr][::-1]
    # fixed label percentage: floor(count * pct) first unassigned rows per label
    dist = [[0, 2, 4], [0, 4, 3, 1], [5, 3, 0]]
    parts = P.split_fixed_label_percentage(labels, dist, 0.1)
    for k, labs in enumerate(dist):
        for lab in labs:
            got = parts[k][labels[parts[k]] == lab]
            assert len(got) == int(np.floor((labels == lab).sum() * 0.1))
    assert len(np.unique(np.concatenate(parts))) == sum(len(p) for p in parts)
    # label 0 appears in three clients: later clients take the next rows
    z = np.flatnonzero(labels == 0)
    k0 = int(np.floor(len(z) * 0.1))
    assert np.array_equal(parts[0][labels[parts[0]] == 0], z[:k0])
    assert np.array_equal(parts[1][labels[parts[1]] == 0], z[k0:2 * k0])
    # per-device subsample and the 40 % test_normal holdout
    s = P.subsample_rows(10000, 0.05, rng)
    assert s.size == 500 and np.unique(s).size == 500
    held, rest = P.holdout_split(1000, 0.4, rng)
    assert held.size == 400 and rest.size == 600 and not set(held) & set(rest)
