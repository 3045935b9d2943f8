"""PredictableModel (reference ``src/ocvfacerec/facerec/model.py:39-60``).

``compute``/``predict`` keep the reference contract; ``predict_batch`` is the
batched entry point of the device path.  Two fused pipelines, in which the
features never leave the GPU:
* Fisherfaces + NearestNeighbor (Euclidean/Cosine): a batch of faces is
  projected (exact int8-slice MFMA kernel, the gallery centring folded into the
  projection's shift) and searched by the certified tiers;
* LBPH, SpatialHistogram(ExtendedLBP) + NearestNeighbor(ChiSquare)
  (feature.py:266-305, distance.py:101-116): ONE ``ofr_elbp_hist`` launch per
  batch gives the integer cell histograms, searched as counts against the
  counts gallery ``compute`` left on the device (``ofr_chi2_knn``).
"""
from __future__ import annotations

import numpy as np

from .. import _lib
from .classifier import AbstractClassifier, NearestNeighbor, results
from .feature import AbstractFeature, Fisherfaces, SpatialHistogram
from .lbp import ExtendedLBP


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
        if dev is None or dev[0] != id(features):
            return
        if isinstance(dev[1], tuple) and dev[1][0] == "counts":       # SpatialHistogram counts
            if hasattr(self.classifier, "adopt_device_counts"):
                _, C, cell, cb = dev[1]
                self.classifier.adopt_device_counts(C, cell, cb)
        elif hasattr(self.classifier, "adopt_device_rows"):
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

    def _lbph(self):
        return (type(self.feature) is SpatialHistogram and isinstance(self.feature.lbp_operator, ExtendedLBP)
                and type(self.classifier) is NearestNeighbor
                and getattr(self.classifier.dist_metric, "metric_id", None) == 2)

    def _search_device(self, X, k=None):
        clf = self.classifier
        k = int(clf.k if k is None else k)
        if self._lbph():
            return self._search_lbph(X, k)
        g = clf._gallery()
        if g.N and g.d != self.feature._proj().d:
            raise ValueError("feature dimension does not match the classifier gallery")
        # Euclidean: the gallery centring is folded into the projection (W^T x - c, fp64, rounded once)
        Qd = self.feature.project_device(X, shift64=g.shift64)
        return clf._search_prepared(Qd, k)

    def _search_lbph(self, X, k):
        """LBPH batch: faces grouped by size, one histogram launch + one counts search per group."""
        import torch
        if hasattr(X, "device") or (isinstance(X, np.ndarray) and X.ndim == 3):   # one face size
            groups = [(None, X)]
        else:
            X = list(X)
            shapes = {}
            for i, x in enumerate(X):
                shapes.setdefault(np.asarray(x).shape, []).append(i)
            groups = [(sel, [X[i] for i in sel]) for sel in shapes.values()]
        if len(groups) == 1:
            C, cell, cb = self.feature.counts_batch(groups[0][1])
            return self.classifier.search_counts(C, cell, cb, k)
        # a group whose cell size differs from the counts gallery's comes back on the host
        # (search_counts' float path): every group's result goes to the gallery device
        B = len(X)
        dev = _lib.device()
        d_all = i_all = None
        for sel, xs in groups:
            C, cell, cb = self.feature.counts_batch(xs)
            d, i = self.classifier.search_counts(C, cell, cb, k)
            if d_all is None:
                d_all = torch.empty((B,) + tuple(d.shape[1:]), dtype=d.dtype, device=dev)
                i_all = torch.empty((B,) + tuple(i.shape[1:]), dtype=i.dtype, device=dev)
            idx = torch.tensor(sel, dtype=torch.int64, device=dev)
            d_all.index_copy_(0, idx, d.to(dev, d_all.dtype))
            i_all.index_copy_(0, idx, i.to(dev, i_all.dtype))
        return d_all, i_all

    def predict_batch(self, X):
        """Predict a batch of faces (list of 2-D arrays, an array [B, H, W], or a uint8 device
        tensor [B, H, W] such as ``ingest.faces`` returns)."""
        if not (self._fused() or self._lbph()):
            if hasattr(X, "data_ptr"):   # a device face batch: the generic path works on host items
                X = list(X.cpu().numpy())
            qs = [self.feature.extract(x) for x in X]
            return self.classifier.predict_batch(qs) if hasattr(self.classifier, "predict_batch") else \
                [self.classifier.predict(q) for q in qs]
        if len(X) == 0:
            return []
        d_all, i_all = self.search_batch(X)
        return results(d_all, i_all, self.classifier.y)

    def __repr__(self):
        feature_repr = repr(self.feature)
        classifier_repr = repr(self.classifier)
        return "PredictableModel (feature=%s, classifier=%s)" % (feature_repr, classifier_repr)


PredictableModel.__module__ = "ocvfacerec.facerec.model"
