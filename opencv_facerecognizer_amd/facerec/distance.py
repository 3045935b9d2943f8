"""Distance metrics (reference ``src/ocvfacerec/facerec/distance.py``).

The classes keep the reference interface — ``AbstractDistance(name)``,
``__call__(p, q) -> float``, ``name``, ``__repr__`` (distance.py:38-50) — and
the pickled state ``{'_name': ...}``.  Each metric also names the device
kernel that evaluates it in batch (``metric_id``); ``NearestNeighbor`` never
calls ``__call__`` per gallery item (the reference loop, classifier.py:104-108)
but dispatches the whole gallery to the GPU.  ``__call__`` itself runs the same
kernel on a 1x1 problem, so every distance value comes from the device path.

Out of scope (not named by the hot path): NormalizedCorrelation,
HistogramIntersection and the BinRatio family (distance.py:80-98, 119-183).
"""
from __future__ import annotations

import numpy as np

from .. import _lib


class AbstractDistance(object):
    """distance.py:38-50."""

    metric_id = None

    def __init__(self, name):
        self._name = name

    def __call__(self, p, q):
        raise NotImplementedError("Every AbstractDistance must implement the __call__ method.")

    @property
    def name(self):
        return self._name

    def __repr__(self):
        return self._name


def _pair(metric, p, q):
    from .._device import Chi2Gallery, FloatGallery
    p = np.asarray(p, dtype=np.float64).reshape(1, -1)
    q = np.asarray(q, dtype=np.float64).reshape(1, -1)
    if p.shape != q.shape:
        raise ValueError(f"operands could not be broadcast together with shapes {p.shape} {q.shape}")
    if metric == _lib.METRIC_CHISQUARE:
        g = Chi2Gallery(p)
        d, _ = g.search(g.query_rows(q), 1)
    else:
        g = FloatGallery(p, metric)
        d, _ = g.search(g.query_rows(q), 1)
    return np.float64(d.cpu().numpy()[0, 0])


class EuclideanDistance(AbstractDistance):
    """distance.py:53-60 — sqrt(sum((p-q)^2))."""

    metric_id = _lib.METRIC_EUCLIDEAN

    def __init__(self):
        AbstractDistance.__init__(self, "EuclideanDistance")

    def __call__(self, p, q):
        return _pair(self.metric_id, p, q)


class CosineDistance(AbstractDistance):
    """distance.py:63-77 — negated cosine similarity -p.q/sqrt((p.p)(q.q))."""

    metric_id = _lib.METRIC_COSINE

    def __init__(self):
        AbstractDistance.__init__(self, "CosineDistance")

    def __call__(self, p, q):
        return _pair(self.metric_id, p, q)


class ChiSquareDistance(AbstractDistance):
    """distance.py:101-116 — sum((p-q)^2 / (p+q+eps)), eps = np.finfo('float').eps."""

    metric_id = _lib.METRIC_CHISQUARE

    def __init__(self):
        AbstractDistance.__init__(self, "ChiSquareDistance")

    def __call__(self, p, q):
        return _pair(self.metric_id, p, q)


for _c in (AbstractDistance, EuclideanDistance, CosineDistance, ChiSquareDistance):
    _c.__module__ = "ocvfacerec.facerec.distance"
