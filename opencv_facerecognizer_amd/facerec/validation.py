"""Model validation (reference ``src/ocvfacerec/facerec/validation.py``).

The reference's strategies each hand-roll the same loop: build index lists, ``model.compute`` on
the training items, then one ``model.predict`` per test item (validation.py:202-258, 281-317,
344-371, 392-414).  Here a strategy only states its folds -- ``(train indices, test indices)``
pairs over the data it was given -- and ``ValidationStrategy._run`` scores every fold the same
way: one ``compute`` and ONE ``predict_batch`` (a single device batch) of the fold's test items.
The fold contents, the order of their items, the counts and the printed results are the
reference's (``tests/test_validation.py`` replays its loops):

* ``KFoldCrossValidation`` (:178-261): shuffle with Python's ``random`` (argsort of one
  ``random.random()`` per item, :66), then a [class][position] grid of each class's first n
  items (n = the smallest class; k is lowered to n); fold f tests grid columns
  [f*w, (f+1)*w), w = n // k, visited column-major, and trains on the other columns < n.
* ``LeaveOneOutCrossValidation`` (:264-322): no shuffle, one fold per item.
* ``LeaveOneClassOutCrossValidation`` (:325-375): fold per class label, trained on the groups g.
* ``SimpleValidation`` (:378-418): as in the reference, ``ytest``'s LABELS index ``Xtest``.
"""
from __future__ import annotations

import logging
import random

import numpy as np

from .model import PredictableModel


def shuffle(X, y):
    """validation.py:54-70: the same permutation of X (list) and y (array)."""
    order = np.argsort([random.random() for _ in range(len(y))])
    return [X[i] for i in order], np.asarray(y)[order]


def slice_2d(X, rows, cols):
    """validation.py:73-91: the items X[r][c], c-major (all rows of column c before c + 1)."""
    return [X[r][c] for c in cols for r in rows]


def accuracy(true_positives, true_negatives, false_positives, false_negatives, description=None):
    """validation.py:103-115: (tp + tn) / (tp + tn + fp + fn); 0.0 for no observations."""
    right = float(true_positives) + float(true_negatives)
    total = right + float(false_positives) + float(false_negatives)
    return 0.0 if total < 1e-15 else right / total


def precision(true_positives, false_positives):
    """validation.py:94-100: tp / (tp + fp)."""
    return accuracy(true_positives, 0, false_positives, 0)


class ValidationResult(object):
    """validation.py:118-134 (counts of one validation run)."""

    def __init__(self, true_positives, true_negatives, false_positives, false_negatives, description):
        self.true_positives = true_positives
        self.true_negatives = true_negatives
        self.false_positives = false_positives
        self.false_negatives = false_negatives
        self.description = description

    def __repr__(self):
        p = 100 * precision(self.true_positives, self.false_positives)
        a = 100 * accuracy(self.true_positives, self.true_negatives, self.false_positives, self.false_negatives)
        return "ValidationResult (Description=%s, Precision=%.2f%%, Accuracy=%.2f%%)" % (self.description, p, a)


class ValidationStrategy(object):
    """validation.py:137-175, plus the shared fold engine."""

    def __init__(self, model):
        if not isinstance(model, PredictableModel):
            raise TypeError("Validation can only validate the type PredictableModel.")
        self.model = model
        self.validation_results = []

    def add(self, validation_result):
        self.validation_results.append(validation_result)

    def validate(self, X, y, description):
        raise NotImplementedError("Every Validation module must implement the validate method!")

    def print_results(self):
        print(self.model)
        for r in self.validation_results:
            print(r)

    def _run(self, folds, X, fit_labels, truth, description):
        """Score (train, test) index folds: tp = test items predicted as their truth label."""
        fit_labels = np.asarray(fit_labels)
        hits = misses = 0
        for train, test in folds:
            self.model.compute([X[t] for t in train], fit_labels[np.asarray(train, dtype=np.int64)])
            test = list(test)
            if not test:
                continue
            predicted = [p[0] for p in self.model.predict_batch([X[t] for t in test])]
            ok = sum(1 for t, p in zip(test, predicted) if p == truth[t])
            hits += ok
            misses += len(test) - ok
        self.add(ValidationResult(hits, 0, misses, 0, description))

    def __repr__(self):
        return "Validation Kernel (model=%s)" % (self.model)


class KFoldCrossValidation(ValidationStrategy):
    """validation.py:178-261."""

    def __init__(self, model, k=10):
        super(KFoldCrossValidation, self).__init__(model=model)
        self.k = k
        self.logger = logging.getLogger("facerec.validation.KFoldCrossValidation")

    def folds(self, y):
        """(train, test) per fold over the (already shuffled) labels y; lowers self.k to the
        smallest class size as the reference does."""
        y = np.asarray(y)
        members = [np.flatnonzero(y == label) for label in range(len(np.unique(y)))]
        n = min(len(m) for m in members)
        self.k = min(self.k, n)
        w = n // self.k
        grid = np.stack([m[:n] for m in members])          # [class][position]
        cmajor = lambda cols: grid[:, cols].T.reshape(-1)   # noqa: E731 -- column-major flattening
        for f in range(self.k):
            lo, hi = f * w, (f + 1) * w
            self.logger.info("Processing fold %d/%d." % (f + 1, self.k))
            yield (np.concatenate([cmajor(slice(0, lo)), cmajor(slice(hi, n))]), cmajor(slice(lo, hi)))

    def validate(self, X, y, description="ExperimentName"):
        X, y = shuffle(X, y)
        self._run(self.folds(y), X, y, y, description)

    def __repr__(self):
        return "k-Fold Cross Validation (model=%s, k=%s)" % (self.model, self.k)


class LeaveOneOutCrossValidation(ValidationStrategy):
    """validation.py:264-322: no shuffle, each item tested against a model of all the others."""

    def __init__(self, model):
        super(LeaveOneOutCrossValidation, self).__init__(model=model)
        self.logger = logging.getLogger("facerec.validation.LeaveOneOutCrossValidation")

    def validate(self, X, y, description="ExperimentName"):
        y = np.asarray(y)
        n = y.shape[0]
        everything = np.arange(n)

        def folds():
            for i in range(n):
                self.logger.info("Processing fold %d/%d." % (i + 1, n))
                yield np.delete(everything, i), [i]
        self._run(folds(), X, y, y, description)

    def __repr__(self):
        return "Leave-One-Out Cross Validation (model=%s)" % (self.model)


class LeaveOneClassOutCrossValidation(ValidationStrategy):
    """validation.py:325-375: per class label, train on the groups g of the other classes."""

    def __init__(self, model):
        super(LeaveOneClassOutCrossValidation, self).__init__(model=model)
        self.logger = logging.getLogger("facerec.validation.LeaveOneClassOutCrossValidation")

    def validate(self, X, y, g, description="ExperimentName"):
        y, g = np.asarray(y), np.asarray(g)

        def folds():
            for label in range(len(np.unique(y))):
                self.logger.info("Validating Class %s." % label)
                yield np.flatnonzero(y != label), np.flatnonzero(y == label)
        self._run(folds(), X, g, g, description)

    def __repr__(self):
        return "Leave-One-Class-Out Cross Validation (model=%s)" % (self.model)


class SimpleValidation(ValidationStrategy):
    """validation.py:378-418 on a caller-made partition."""

    def __init__(self, model):
        super(SimpleValidation, self).__init__(model=model)
        self.logger = logging.getLogger("facerec.validation.SimpleValidation")

    def validate(self, Xtrain, ytrain, Xtest, ytest, description="ExperimentName"):
        self.logger.info("Simple Validation.")
        self.model.compute(Xtrain, ytrain)
        self.logger.debug("Model computed.")
        visit = [i for i in ytest]                # :407: the labels index the test items
        predicted = [p[0] for p in self.model.predict_batch([Xtest[i] for i in visit])] if visit else []
        hits = sum(1 for i, p in zip(visit, predicted) if p == ytest[i])
        self.add(ValidationResult(hits, 0, len(visit) - hits, 0, description))

    def __repr__(self):
        return "Simple Validation (model=%s)" % (self.model)


for _c in (ValidationResult, ValidationStrategy, KFoldCrossValidation, LeaveOneOutCrossValidation,
           LeaveOneClassOutCrossValidation, SimpleValidation):
    _c.__module__ = "ocvfacerec.facerec.validation"
