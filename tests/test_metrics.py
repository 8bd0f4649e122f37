"""ROC-AUC / classification metrics and the SAE-CEN scorer vs sklearn/scipy
(`src/Evaluator/evaluator.py:21-48`, `src/Model/Centroid.py`)."""
import numpy as np
import scipy.spatial
from sklearn.metrics import auc, f1_score, precision_score, recall_score, roc_curve
from sklearn.preprocessing import StandardScaler

from fedmse_decentralized_amd.engine.torch_engine import cen_score_numpy
from fedmse_decentralized_amd.eval.metrics import classification_metrics, roc_auc


def _sk_auc(y, s):
    fpr, tpr, _ = roc_curve(y, s)
    return auc(fpr, tpr)


def test_auc_matches_sklearn_with_ties():
    rng = np.random.default_rng(0)
    for trial in range(20):
        n = int(rng.integers(20, 3000))
        y = rng.integers(0, 2, size=n)
        s = np.round(rng.normal(size=n) + y * rng.uniform(0, 2), int(rng.integers(0, 3)))  # many ties
        assert abs(roc_auc(y, s) - _sk_auc(y, s)) < 1e-12


def test_auc_nan_inf_handling():
    y = np.array([0, 0, 1, 1, 1])
    s = np.array([0.1, np.nan, np.inf, 0.5, -np.inf])
    assert abs(roc_auc(y, s) - _sk_auc(y, np.nan_to_num(s))) < 1e-12


def test_classification_metrics():
    rng = np.random.default_rng(1)
    y = rng.integers(0, 2, size=400)
    s = rng.uniform(0, 1, size=400) + 0.3 * y
    f1, p, r = classification_metrics(y, s)
    pred = (s > 0.5).astype(int)
    assert abs(f1 - f1_score(y, pred)) < 1e-12
    assert abs(p - precision_score(y, pred)) < 1e-12
    assert abs(r - recall_score(y, pred)) < 1e-12


def test_cen_score_matches_reference_classifier():
    rng = np.random.default_rng(2)
    tr = (rng.normal(size=(680, 7)) * rng.uniform(0.1, 5, size=7) + 3).astype(np.float32)
    te = (rng.normal(size=(4000, 7)) * 4).astype(np.float32)
    # reference CentroidBasedOneClassClassifier.fit / get_density
    sc = StandardScaler().fit(tr)
    ref = np.mean(scipy.spatial.distance.cdist(sc.transform(te), np.zeros((1, 7)), metric="euclidean"), axis=1)
    ours = cen_score_numpy(tr, te)
    assert np.array_equal(ours, ref)
