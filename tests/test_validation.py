"""validation.py (reference src/ocvfacerec/facerec/validation.py) on the host: fold construction,
counting and batching checked against a reference-faithful per-face loop with a host model."""
import random

import numpy as np
import pytest

from ocvfacerec.facerec.classifier import AbstractClassifier
from ocvfacerec.facerec.feature import Identity
from ocvfacerec.facerec.model import PredictableModel
from ocvfacerec.facerec import validation as V

import facerec_oracle as O


class _HostNN(AbstractClassifier):
    """1-NN on the host (the oracle's reference-faithful loop): no device needed."""

    def compute(self, X, y):
        self.X, self.y = list(X), np.asarray(y)

    def predict(self, q):
        return O.nn_predict_faithful(self.X, self.y, np.asarray(q).reshape(-1, 1))[0]


def _data(seed, c=5, per=(7, 9, 6, 8, 10), d=6):
    r = np.random.default_rng(seed)
    means = r.normal(0, 2, (c, d))
    y = np.concatenate([np.full(p, i) for i, p in enumerate(per)])
    X = [means[i] + r.normal(0, 1.2, d) for i in y]
    return X, y


def _kfold_faithful(model_factory, X, y, k, seed):
    """validation.py:202-258 with one model.predict per test item."""
    random.seed(seed)
    idx = np.argsort([random.random() for _ in range(len(y))])
    y = np.asarray(y)[idx]
    X = [X[i] for i in idx]
    c = len(np.unique(y))
    folds = [np.where(y == i)[0].tolist() for i in range(c)]
    n = min(len(f) for f in folds)
    k = min(k, n)
    size = n // k
    tp = fp = 0
    for i in range(k):
        lo, hi = i * size, (i + 1) * size
        test = [folds[r][j] for j in range(lo, hi) for r in range(c)]
        train = [folds[r][j] for j in range(0, lo) for r in range(c)] + \
                [folds[r][j] for j in range(hi, n) for r in range(c)]
        m = model_factory()
        m.compute([X[t] for t in train], y[train])
        for j in test:
            if m.predict(X[j])[0] == y[j]:
                tp += 1
            else:
                fp += 1
    return tp, fp


@pytest.mark.parametrize("k", [3, 10])
def test_kfold_matches_reference_loop(k):
    X, y = _data(1)
    random.seed(42)
    v = V.KFoldCrossValidation(PredictableModel(Identity(), _HostNN()), k=k)
    v.validate(X, y, description="t")
    tp, fp = _kfold_faithful(lambda: PredictableModel(Identity(), _HostNN()), X, y, k, 42)
    r = v.validation_results[0]
    assert (r.true_positives, r.false_positives) == (tp, fp) and tp + fp > 0
    assert v.k == min(k, 6)                               # lowered to the smallest class (:223-224)
    assert "Precision=" in repr(r) and r.description == "t"


def test_leave_one_out_and_class_out_and_simple():
    X, y = _data(2)
    v = V.LeaveOneOutCrossValidation(PredictableModel(Identity(), _HostNN()))
    v.validate(X, y)
    r = v.validation_results[0]
    n = len(y)
    tp = sum(O.nn_predict_faithful([X[t] for t in range(n) if t != i], np.delete(y, i),
                                   np.asarray(X[i]).reshape(-1, 1))[0][0] == y[i] for i in range(n))
    assert (r.true_positives, r.false_positives) == (tp, n - tp)
    g = y % 2
    v2 = V.LeaveOneClassOutCrossValidation(PredictableModel(Identity(), _HostNN()))
    v2.validate(X, y, g)
    r2 = v2.validation_results[0]
    assert r2.true_positives + r2.false_positives == n
    v3 = V.SimpleValidation(PredictableModel(Identity(), _HostNN()))
    ytest = np.array([0, 1, 2, 1])                          # labels that index Xtest (:407-410)
    v3.validate(X, y, X[:3], ytest)
    assert v3.validation_results[0].true_positives + v3.validation_results[0].false_positives == 4


def test_validation_type_check_and_metrics():
    with pytest.raises(TypeError, match="PredictableModel"):
        V.KFoldCrossValidation(object())
    assert V.precision(3, 1) == 0.75 and V.accuracy(0, 0, 0, 0) == 0.0
    assert V.slice_2d([[1, 2, 3, 4], [5, 6, 7, 8]], range(0, 2), range(0, 1)) == [1, 5]
