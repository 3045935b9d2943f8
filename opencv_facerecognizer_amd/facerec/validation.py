"""Model validation (reference ``src/ocvfacerec/facerec/validation.py``).

Same classes, arguments, results and fold construction as the reference.  What
changes: each fold's test faces go through ``PredictableModel.predict_batch``
(one device batch per fold) instead of one ``predict`` call per face
(validation.py:251-256, 312-317, 365-371, 407-414); the labels are the same,
since ``predict`` is ``predict_batch`` of one face.  ``shuffle`` draws its
permutation from Python's ``random`` exactly as the reference (argsort of one
``random.random()`` per item, :66), so a seeded ``random`` gives the
reference's folds.
"""
from __future__ import annotations

import logging
import math
import random

import numpy as np

from .model import PredictableModel


def shuffle(X, y):
    """validation.py:54-70."""
    idx = np.argsort([random.random() for _ in range(len(y))])
    y = np.asarray(y)
    X = [X[i] for i in idx]
    y = y[idx]
    return (X, y)


def slice_2d(X, rows, cols):
    """validation.py:73-91: X[i][j] for j in cols for i in rows (column-major flattening)."""
    return [X[i][j] for j in cols for i in rows]


def precision(true_positives, false_positives):
    """validation.py:94-100."""
    return accuracy(true_positives, 0, false_positives, 0)


def accuracy(true_positives, true_negatives, false_positives, false_negatives, description=None):
    """validation.py:103-115."""
    true_positives = float(true_positives)
    true_negatives = float(true_negatives)
    false_positives = float(false_positives)
    false_negatives = float(false_negatives)
    if (true_positives + true_negatives + false_positives + false_negatives) < 1e-15:
        return 0.0
    return (true_positives + true_negatives) / (true_positives + false_positives + true_negatives + false_negatives)


def _labels(model, X, idx):
    """Predicted labels of the items X[j], j in idx, as one batch."""
    if len(idx) == 0:
        return []
    return [p[0] for p in model.predict_batch([X[j] for j in idx])]


class ValidationResult(object):
    """validation.py:118-134."""

    def __init__(self, true_positives, true_negatives, false_positives, false_negatives, description):
        self.true_positives = true_positives
        self.true_negatives = true_negatives
        self.false_positives = false_positives
        self.false_negatives = false_negatives
        self.description = description

    def __repr__(self):
        res_precision = precision(self.true_positives, self.false_positives) * 100
        res_accuracy = accuracy(self.true_positives, self.true_negatives, self.false_positives,
                                self.false_negatives) * 100
        return "ValidationResult (Description=%s, Precision=%.2f%%, Accuracy=%.2f%%)" % (
            self.description, res_precision, res_accuracy)


class ValidationStrategy(object):
    """validation.py:137-175."""

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
        for validation_result in self.validation_results:
            print(validation_result)

    def __repr__(self):
        return "Validation Kernel (model=%s)" % (self.model)


class KFoldCrossValidation(ValidationStrategy):
    """validation.py:178-261: k folds of equal size per class (k is lowered to the smallest class)."""

    def __init__(self, model, k=10):
        super(KFoldCrossValidation, self).__init__(model=model)
        self.k = k
        self.logger = logging.getLogger("facerec.validation.KFoldCrossValidation")

    def validate(self, X, y, description="ExperimentName"):
        X, y = shuffle(X, y)
        c = len(np.unique(y))
        foldIndices = []
        n = np.iinfo(int).max
        for i in range(0, c):
            idx = np.where(y == i)[0]
            n = min(n, idx.shape[0])
            foldIndices.append(idx.tolist())
        if n < self.k:
            self.k = n
        foldSize = int(math.floor(n / self.k))
        true_positives, false_positives, true_negatives, false_negatives = (0, 0, 0, 0)
        for i in range(0, self.k):
            self.logger.info("Processing fold %d/%d." % (i + 1, self.k))
            l = int(i * foldSize)
            h = int((i + 1) * foldSize)
            testIdx = slice_2d(foldIndices, cols=range(l, h), rows=range(0, c))
            trainIdx = slice_2d(foldIndices, cols=range(0, l), rows=range(0, c))
            trainIdx.extend(slice_2d(foldIndices, cols=range(h, n), rows=range(0, c)))
            Xtrain = [X[t] for t in trainIdx]
            ytrain = y[trainIdx]
            self.model.compute(Xtrain, ytrain)
            for j, prediction in zip(testIdx, _labels(self.model, X, testIdx)):
                if prediction == y[j]:
                    true_positives = true_positives + 1
                else:
                    false_positives = false_positives + 1
        self.add(ValidationResult(true_positives, true_negatives, false_positives, false_negatives, description))

    def __repr__(self):
        return "k-Fold Cross Validation (model=%s, k=%s)" % (self.model, self.k)


class LeaveOneOutCrossValidation(ValidationStrategy):
    """validation.py:264-322: one training per observation (no shuffle)."""

    def __init__(self, model):
        super(LeaveOneOutCrossValidation, self).__init__(model=model)
        self.logger = logging.getLogger("facerec.validation.LeaveOneOutCrossValidation")

    def validate(self, X, y, description="ExperimentName"):
        true_positives, false_positives, true_negatives, false_negatives = (0, 0, 0, 0)
        y = np.asarray(y)
        n = y.shape[0]
        for i in range(0, n):
            self.logger.info("Processing fold %d/%d." % (i + 1, n))
            trainIdx = []
            trainIdx.extend(range(0, i))
            trainIdx.extend(range(i + 1, n))
            Xtrain = [X[t] for t in trainIdx]
            ytrain = y[trainIdx]
            self.model.compute(Xtrain, ytrain)
            prediction = self.model.predict(X[i])[0]
            if prediction == y[i]:
                true_positives = true_positives + 1
            else:
                false_positives = false_positives + 1
        self.add(ValidationResult(true_positives, true_negatives, false_positives, false_negatives, description))

    def __repr__(self):
        return "Leave-One-Out Cross Validation (model=%s)" % (self.model)


class LeaveOneClassOutCrossValidation(ValidationStrategy):
    """validation.py:325-375: train on the groups g of every other class, test one class."""

    def __init__(self, model):
        super(LeaveOneClassOutCrossValidation, self).__init__(model=model)
        self.logger = logging.getLogger("facerec.validation.LeaveOneClassOutCrossValidation")

    def validate(self, X, y, g, description="ExperimentName"):
        true_positives, false_positives, true_negatives, false_negatives = (0, 0, 0, 0)
        y, g = np.asarray(y), np.asarray(g)
        for i in range(0, len(np.unique(y))):
            self.logger.info("Validating Class %s." % i)
            trainIdx = np.where(y != i)[0]
            testIdx = np.where(y == i)[0]
            Xtrain = [X[t] for t in trainIdx]
            gtrain = g[trainIdx]
            self.model.compute(Xtrain, gtrain)
            for j, prediction in zip(testIdx, _labels(self.model, X, testIdx)):
                if prediction == g[j]:
                    true_positives = true_positives + 1
                else:
                    false_positives = false_positives + 1
        self.add(ValidationResult(true_positives, true_negatives, false_positives, false_negatives, description))

    def __repr__(self):
        return "Leave-One-Class-Out Cross Validation (model=%s)" % (self.model)


class SimpleValidation(ValidationStrategy):
    """validation.py:378-418.  As in the reference, the test items are visited as Xtest[i] for i in
    ytest (:407-410: the LABELS index the test list), so ytest must hold valid indices."""

    def __init__(self, model):
        super(SimpleValidation, self).__init__(model=model)
        self.logger = logging.getLogger("facerec.validation.SimpleValidation")

    def validate(self, Xtrain, ytrain, Xtest, ytest, description="ExperimentName"):
        self.logger.info("Simple Validation.")
        self.model.compute(Xtrain, ytrain)
        self.logger.debug("Model computed.")
        true_positives, false_positives, true_negatives, false_negatives = (0, 0, 0, 0)
        idx = [i for i in ytest]
        for i, prediction in zip(idx, _labels(self.model, Xtest, idx)):
            if prediction == ytest[i]:
                true_positives = true_positives + 1
            else:
                false_positives = false_positives + 1
        self.add(ValidationResult(true_positives, true_negatives, false_positives, false_negatives, description))

    def __repr__(self):
        return "Simple Validation (model=%s)" % (self.model)


for _c in (ValidationResult, ValidationStrategy, KFoldCrossValidation, LeaveOneOutCrossValidation,
           LeaveOneClassOutCrossValidation, SimpleValidation):
    _c.__module__ = "ocvfacerec.facerec.validation"
