"""PredictableModel (reference ``src/ocvfacerec/facerec/model.py:39-60``).

``compute``/``predict`` keep the reference contract; ``predict_batch`` is the
batched entry point of the device path: for Fisherfaces + NearestNeighbor
(Euclidean/Cosine) a batch of faces is projected (fp32 MFMA kernel, with the
gallery centring folded into the projection's shift) and searched without
the features ever leaving the GPU.
"""
from __future__ import annotations

import numpy as np

from .classifier import AbstractClassifier, NearestNeighbor, vote
from .feature import AbstractFeature, Fisherfaces


class PredictableModel(object):
    def __init__(self, feature, classifier):
        if not isinstance(feature, AbstractFeature):
            raise TypeError("feature must be of type AbstractFeature!")
        if not isinstance(classifier, AbstractClassifier):
            raise TypeError("classifier must be of type AbstractClassifier!")
        self.feature = feature
        self.classifier = classifier

    def compute(self, X, y):
        """model.py:49-51.  When the feature left its training features on the device, the classifier
        builds its device gallery from them (no host round trip of the gallery)."""
        features = self.feature.compute(X, y)
        self.classifier.compute(features, y)
        dev = self.feature.__dict__.pop("_dev_features", None)
        if dev is not None and dev[0] == id(features) and hasattr(self.classifier, "adopt_device_rows"):
            self.classifier.adopt_device_rows(dev[1])

    def shard(self, group=None):
        """Shard the classifier's gallery over the ranks of ``group`` (NearestNeighbor.shard): every
        rank then predicts the same faces and gets the global result."""
        self.classifier.shard(group)
        return self

    def predict(self, X):
        """model.py:53-55 (one face)."""
        return self.predict_batch([X])[0]

    def search_batch(self, X, k=None):
        """Batch of faces -> (distances fp64 [B,k], gallery indices int64 [B,k]) host arrays."""
        d, i = self._search_device(X, k)
        return d.cpu().numpy(), i.cpu().numpy()

    def _fused(self):
        return (isinstance(self.feature, Fisherfaces) and type(self.classifier) is NearestNeighbor
                and getattr(self.classifier.dist_metric, "metric_id", None) in (0, 1))

    def _search_device(self, X, k=None):
        clf = self.classifier
        k = int(clf.k if k is None else k)
        g = clf._gallery()
        if g.N and g.d != self.feature._proj().d:
            raise ValueError("feature dimension does not match the classifier gallery")
        # Euclidean: the gallery centring is folded into the projection (W^T x - c, fp64, rounded once)
        Qd = self.feature.project_device(X, shift64=g.shift64)
        return clf._search_prepared(Qd, k)

    def predict_batch(self, X):
        """Predict a batch of faces (list of 2-D arrays, an array [B, H, W], or a uint8 device
        tensor [B, H, W] such as ``ingest.faces`` returns)."""
        if not self._fused():
            if hasattr(X, "data_ptr"):   # a device face batch: the generic path works on host items
                X = list(X.cpu().numpy())
            qs = [self.feature.extract(x) for x in X]
            return self.classifier.predict_batch(qs) if hasattr(self.classifier, "predict_batch") else \
                [self.classifier.predict(q) for q in qs]
        if len(X) == 0:
            return []
        d_all, i_all = self.search_batch(X)
        y = np.asarray(self.classifier.y)
        out = []
        for dist, idx in zip(d_all, i_all):
            valid = idx >= 0
            sorted_y = y[idx[valid]]
            out.append([vote(sorted_y), {"labels": sorted_y, "distances": dist[valid]}])
        return out

    def __repr__(self):
        feature_repr = repr(self.feature)
        classifier_repr = repr(self.classifier)
        return "PredictableModel (feature=%s, classifier=%s)" % (feature_repr, classifier_repr)


PredictableModel.__module__ = "ocvfacerec.facerec.model"
