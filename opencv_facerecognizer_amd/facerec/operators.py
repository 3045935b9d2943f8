"""Feature combinators (reference ``src/ocvfacerec/facerec/operators.py``).

``ChainOperator`` (operators.py:58-81) is the glue Fisherfaces uses to chain
PCA into LDA (feature.py:222-224).  CombineOperator/CombineOperatorND
(operators.py:84-157) are not on the hot path and are out of scope.
"""
from __future__ import annotations

from .feature import AbstractFeature


class FeatureOperator(AbstractFeature):
    """operators.py:39-55."""

    def __init__(self, model1, model2):
        if (not isinstance(model1, AbstractFeature)) or (not isinstance(model2, AbstractFeature)):
            raise Exception("A FeatureOperator only works on classes implementing an AbstractFeature!")
        self.model1 = model1
        self.model2 = model2

    def __repr__(self):
        return "FeatureOperator(" + repr(self.model1) + "," + repr(self.model2) + ")"


class ChainOperator(FeatureOperator):
    """operators.py:58-81: model2.compute(model1.compute(X, y), y)."""

    def __init__(self, model1, model2):
        FeatureOperator.__init__(self, model1, model2)

    def compute(self, X, y):
        X = self.model1.compute(X, y)
        return self.model2.compute(X, y)

    def extract(self, X):
        X = self.model1.extract(X)
        return self.model2.extract(X)

    def __repr__(self):
        return "ChainOperator(" + repr(self.model1) + "," + repr(self.model2) + ")"


for _c in (FeatureOperator, ChainOperator):
    _c.__module__ = "ocvfacerec.facerec.operators"
