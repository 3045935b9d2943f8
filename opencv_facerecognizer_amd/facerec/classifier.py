"""k-nearest-neighbour classifier (reference ``src/ocvfacerec/facerec/classifier.py``).

``NearestNeighbor`` keeps the reference's interface and pickled state
(``X`` list of features, ``y`` labels, ``k``, ``dist_metric``;
classifier.py:53-74) and return format ``[label, {'labels', 'distances'}]``
(classifier.py:129).  The search — the per-gallery-item distance loop
(:104-108), the argsort (:113) and the top-k slice (:118-119) — runs on the
GPU: the gallery is uploaded once into a device-resident layout (derived
state, never pickled) and every query batch is one kernel pipeline
(``_device.FloatGallery`` / ``Chi2Gallery``).  The label vote (:121-123) is a
k-element host operation, as in the reference.

Tie order: exact distance ties resolve to the lowest gallery index (the
reference's quicksort leaves their order unspecified).

Multi-GPU (SURVEY §8e, §8f row 2 "sharding on load"): ``shard()`` under torch.distributed keeps
only this rank's contiguous block of the gallery rows on its GPU; every rank then calls
``predict``/``predict_batch``/``search`` with the same queries (SPMD) and gets the global result
(``parallel.certify_sharded`` for the certified Euclidean tiers, else one all-gather + merge of
the local exact top-k lists).

Out of scope: ``SVM`` (classifier.py:150-222) needs the absent libsvm.
"""
from __future__ import annotations

import operator as op
import threading

import numpy as np
import torch

from .. import _lib
from .._device import Chi2Gallery, FloatGallery, counts_of, infer_count_denom
from .distance import EuclideanDistance


class AbstractClassifier(object):
    """classifier.py:42-50."""

    def compute(self, X, y):
        raise NotImplementedError("Every AbstractClassifier must implement the compute method.")

    def predict(self, X):
        raise NotImplementedError("Every AbstractClassifier must implement the predict method.")

    def update(self, X, y):
        raise NotImplementedError("This Classifier is cannot be updated.")


def vote(sorted_y):
    """classifier.py:121-123: most frequent label among the k nearest, ties -> smallest label.

    The reference walks np.bincount(sorted_y), O(largest label) per query (1.8 s for 4096 queries
    against 10k identities); np.unique gives the same answer in O(k log k).  Empty or negative
    labels take the reference expression, which raises as it does there."""
    sorted_y = np.asarray(sorted_y)
    if sorted_y.size == 0 or sorted_y.min() < 0:
        hist = dict((key, val) for key, val in enumerate(np.bincount(sorted_y)) if val)
        return max(hist.items(), key=op.itemgetter(1))[0]
    vals, counts = np.unique(sorted_y, return_counts=True)
    return int(vals[np.argmax(counts)])


def vote_rows(labels):
    """``vote`` of every row of a non-negative label matrix [B][k] at once: each row sorted, the
    count of every entry's value, the first maximum of the sorted row (= the smallest of the most
    frequent labels)."""
    s = np.sort(labels, axis=1)
    if s.shape[1] == 1:
        return s[:, 0]
    counts = (s[:, :, None] == s[:, None, :]).sum(axis=2)
    return s[np.arange(len(s)), np.argmax(counts, axis=1)]


def results(d_all, i_all, y):
    """classifier.py:113-129 for a batch: host top-k (distances [B][k], gallery rows [B][k], -1 =
    no row) -> the reference's per-query ``[label, {'labels': sorted_y, 'distances': ...}]``.  The
    labels and the vote are formed for the whole batch at once; each query's arrays are row views
    of the two batch arrays."""
    y = np.asarray(y)
    i_all = np.asarray(i_all)
    d_all = np.asarray(d_all)
    valid = i_all >= 0
    if len(i_all) and valid.all() and len(y):
        lab = y[i_all]
        if lab.size == 0 or lab.min() >= 0:
            votes = vote_rows(lab).tolist() if lab.shape[1] else [vote(r) for r in lab]
            return [[v, {"labels": l, "distances": d}] for v, l, d in zip(votes, lab, d_all)]
    out = []
    for dist, idx, ok in zip(d_all, i_all, valid):      # ragged rows (k > N) or labels that raise
        sorted_y = y[idx[ok]]
        out.append([vote(sorted_y), {"labels": sorted_y, "distances": dist[ok]}])
    return out


class NearestNeighbor(AbstractClassifier):
    """classifier.py:53-132 on the GPU."""

    def __init__(self, dist_metric=EuclideanDistance(), k=1):
        AbstractClassifier.__init__(self)
        self.k = k
        self.dist_metric = dist_metric
        self.X = []
        self.y = np.array([], dtype=np.int32)

    # -- reference API ----------------------------------------------------
    def update(self, X, y):
        """classifier.py:65-70."""
        self.X.append(X)
        self.y = np.append(self.y, y)

    def compute(self, X, y):
        """classifier.py:72-74."""
        self.X = X
        self.y = np.asarray(y)
        self._invalidate()

    def predict(self, q):
        """classifier.py:76-129 for one query."""
        return self.predict_batch([q])[0]

    # -- batch API (new) --------------------------------------------------
    def predict_batch(self, Q):
        """Predict a batch: Q is a list of features or a 2-D array [B, d]."""
        d_all, i_all = self.search(Q)
        return results(d_all, i_all, self.y)

    def search(self, Q, k=None):
        """Top-k gallery rows of every query: (distances fp64 [B,k], gallery indices int64 [B,k]) on host."""
        k = int(self.k if k is None else k)
        Qd, B, g = self._queries(Q)
        if B == 0:
            return np.zeros((0, k)), np.zeros((0, k), np.int64)
        dist, idx = self._search_device(Qd, k, g)
        return dist.cpu().numpy(), idx.cpu().numpy()

    # -- device state ----------------------------------------------------------
    def _metric(self):
        mid = getattr(self.dist_metric, "metric_id", None)
        if mid is None:
            raise NotImplementedError(
                f"{self.dist_metric!r} has no device kernel (supported: Euclidean, Cosine, ChiSquare)")
        return mid

    def _invalidate(self):
        for key in ("_dev", "_dev_f32", "_chi2_denom"):
            self.__dict__.pop(key, None)

    # -- multi-GPU ---------------------------------------------------------------
    def shard(self, group=None):
        """Hold only this rank's rows [r*N/G, (r+1)*N/G) of the gallery on this process's GPU
        (torch.distributed initialised, one process per GPU; G = the group's size).  Every rank
        keeps the full host state (X, y: the reference's pickled model) and must call the search
        methods with the same queries.  Returns self."""
        from ..parallel import world
        rank, ws = world(group)
        self.__dict__["_shard"] = (group, rank, ws)
        self._invalidate()
        return self

    def _shard_info(self):
        sh = self.__dict__.get("_shard")
        return sh if sh is not None and sh[2] > 1 else None

    def _gallery_sharded(self, mid, sh):
        from ..parallel import shard_range
        _, rank, ws = sh
        n = len(self.X)
        key = (mid, id(self.X), _lib.device(), "shard", rank, ws)
        cache = self.__dict__.get("_dev")
        if cache is not None and cache[0] == key and cache[1] == n:
            return cache[2]
        if n < ws:
            raise ValueError(f"a gallery of {n} rows cannot be sharded over {ws} ranks")
        n0, n1 = shard_range(n, rank, ws)
        feats = self._stack(self.X[n0:n1])
        if mid == _lib.METRIC_CHISQUARE:
            g = self._chi2_gallery(feats)
        else:
            # the same centre on every rank: the mean of all rows, from the host copy every rank holds
            shift = self._stack(self.X).mean(0) if mid == _lib.METRIC_EUCLIDEAN else None
            g = FloatGallery(feats, mid, shift64=shift)
            if mid == _lib.METRIC_EUCLIDEAN:
                # the column-block scales and the prefix length from the block sums of ALL rows (one
                # all-reduce, every rank builds its shard here on its first search): every rank then picks
                # the same start tier, so their tier chains -- and collectives -- match (certify_sharded)
                from ..parallel import share_block_scales
                share_block_scales(g, sh[0])
        g.index_base = n0
        self.__dict__["_dev"] = (key, n, g)
        return g

    def _gallery(self):
        """Device gallery of self.X, built once and extended in place when items were appended
        (update, or X grown by the caller): an update costs the new rows, not a re-upload."""
        mid = self._metric()
        key = (mid, id(self.X), _lib.device())
        n = len(self.X)
        if n > len(self.y):
            raise Exception("More distances than classes. Is your distance metric correct?")  # classifier.py:109-110
        sh = self._shard_info()
        if sh is not None:
            with _DEVICE_LOCK:
                return self._gallery_sharded(mid, sh)
        cache = self.__dict__.get("_dev")
        if cache is not None and cache[0] == key and cache[1] == n:
            return cache[2]
        with _DEVICE_LOCK:   # a search on another thread must not see a half-grown gallery
            cache = self.__dict__.get("_dev")
            if cache is not None and cache[0] == key:
                n0, g = cache[1], cache[2]
                if n0 == n:
                    return g
                if 0 < n0 < n and g.N == n0:
                    try:
                        g.append(self._stack(self.X[n0:]))
                    except TypeError:      # a counts gallery and rows that are not counts: rebuild below
                        pass
                    else:
                        self.__dict__["_dev"] = (key, n, g)
                        return g
            feats = self._stack(self.X) if n else np.zeros((0, 1))
            g = self._chi2_gallery(feats) if mid == _lib.METRIC_CHISQUARE else FloatGallery(feats, mid)
            self.__dict__["_dev"] = (key, n, g)
            return g

    def _chi2_gallery(self, feats):
        """ChiSquare gallery of host rows: the LBP spatial histograms (count / cell, feature.py:298-299)
        are held as their integer counts (exact, a quarter of the fp32 bytes); anything else as fp32."""
        hint = self.__dict__.get("_chi2_denom")
        denom = hint if hint is not None else (infer_count_denom(feats) if len(feats) else None)
        got = counts_of(feats, denom) if denom else None
        if got is None:
            return Chi2Gallery(feats)
        self.__dict__["_chi2_denom"] = denom
        return Chi2Gallery.from_counts(got[0], got[1], denom)

    def adopt_device_rows(self, F):
        """Seed the device gallery from fp64 device rows F [N][d] equal to self.X (e.g. the training
        features a Fisherfaces.compute just produced on the device)."""
        mid = self._metric()
        if mid == _lib.METRIC_CHISQUARE or int(F.shape[0]) != len(self.X) or self._shard_info() is not None:
            return
        with _DEVICE_LOCK:
            g = FloatGallery(F, mid)
            self.__dict__["_dev"] = ((mid, id(self.X), _lib.device()), len(self.X), g)

    def adopt_device_counts(self, C, cell, count_bytes):
        """Seed the ChiSquare gallery from device counts C [N][nbins] whose histograms (C / cell) are
        self.X (SpatialHistogram.compute just produced them on the device): no float64 upload."""
        mid = self._metric()
        if mid != _lib.METRIC_CHISQUARE or int(C.shape[0]) != len(self.X) or self._shard_info() is not None:
            return
        with _DEVICE_LOCK:
            g = Chi2Gallery.from_counts(C, count_bytes, float(cell))
            self.__dict__["_chi2_denom"] = float(cell)
            self.__dict__["_dev"] = ((mid, id(self.X), _lib.device()), len(self.X), g)

    def search_counts(self, C, cell, count_bytes, k=None):
        """LBPH queries as device counts C [B][nbins] of `cell`-pixel cells (SpatialHistogram.counts_batch):
        the counts go straight to a counts gallery of the same cell size; otherwise (a float gallery,
        another cell size) the histograms C / cell take the host path.  -> (distances, indices) device."""
        k = int(self.k if k is None else k)
        g = self._gallery()
        B = int(C.shape[0])
        if B and len(self.X) and int(C.shape[1]) != g.nbins:
            raise ValueError(f"query dimension {int(C.shape[1])} does not match the gallery")
        if (isinstance(g, Chi2Gallery) and g.count_bytes == count_bytes and g.denom == float(cell)
                and B and g.N):
            Qd = C if C.shape[1] % (16 // count_bytes) == 0 else Chi2Gallery.from_counts(C, count_bytes, cell).G
            return self._search_device(Qd.contiguous(), k, g)
        from .._device import counts_numpy
        H = counts_numpy(C, count_bytes).astype(np.float64) / float(cell)
        d, i = self.search(H, k)
        return torch.from_numpy(d), torch.from_numpy(i)

    @staticmethod
    def _stack(items):
        return np.stack([np.asarray(x, dtype=np.float64).reshape(-1) for x in items])

    def _queries(self, Q):
        g = self._gallery()
        if isinstance(Q, np.ndarray) and Q.ndim == 2 and not isinstance(Q, np.matrix):
            arr = np.asarray(Q, np.float64)
        else:
            arr = np.stack([np.asarray(q, dtype=np.float64).reshape(-1) for q in Q]) if len(Q) else np.zeros((0, 1))
        B = arr.shape[0]
        if B and len(self.X) and arr.shape[1] != (g.nbins if isinstance(g, Chi2Gallery) else g.d):
            raise ValueError(f"query dimension {arr.shape[1]} does not match the gallery")
        Qd = g.query_rows(arr)
        if Qd is None:                 # ChiSquare: counts gallery, rows that are not counts / denom
            g = self._float_twin()
            Qd = g.query_rows(arr)
        return Qd, B, g

    def _float_twin(self):
        """fp32 copy of a counts ChiSquare gallery (built once) for queries that are not counts."""
        g = self._gallery()
        tw = self.__dict__.get("_dev_f32")
        if tw is None or tw[0] is not g or tw[1] != g.N:
            feats = self._stack(self.X[:g.N]) if self._shard_info() is None else None
            if feats is None:
                from ..parallel import shard_range
                _, rank, ws = self._shard_info()
                n0, n1 = shard_range(len(self.X), rank, ws)
                feats = self._stack(self.X[n0:n1])
            t = Chi2Gallery(feats)
            t.index_base = getattr(g, "index_base", 0)
            tw = (g, g.N, t)
            self.__dict__["_dev_f32"] = tw
        return tw[2]

    def _search_device(self, Qd, k, g=None):
        g = g or self._gallery()
        with _DEVICE_LOCK:
            sh = self._shard_info()
            return g.search(Qd, k) if sh is None else self._search_sharded(g, Qd, k, sh)

    def _search_sharded(self, g, Qd, k, sh):
        """Global top-k over the shards.  The path is chosen from values every rank shares (metric,
        batch size, k, search mode), so all ranks run the same collectives."""
        from ..parallel import certify_sharded, exchange_topk, merge_sharded, merge_topk
        group, _, ws = sh
        B = int(Qd.shape[0])
        n0 = getattr(g, "index_base", 0)
        if isinstance(g, FloatGallery) and g.metric == _lib.METRIC_EUCLIDEAN and g.use_q8(B, k):
            # adaptive start tier: every rank holds the same global failure statistics (certify_sharded)
            g.last_start_tier = g.start_tier(B)
            qq = g.quantize_queries(Qd, tier=g.last_start_tier)
            out = g.search_q8_phase(1, Qd, qq, k, n0)
            merge_sharded(g, Qd, qq, k, n0, out, group)
            (md, mi), counts = certify_sharded(g, Qd, qq, k, out, n0, group)
            g.last_fallbacks = tuple(counts)
            return md, mi
        d, i = g.search(Qd, k, n0)                 # this shard's exact top-k, global row indices
        gd, gi = exchange_topk(d.to(torch.float64), i.to(torch.int64), group)
        return merge_topk(gd.contiguous(), gi.contiguous(), ws, k, k)

    def _search_prepared(self, Qd, k):
        """Qd already in the gallery's query layout (centred for Euclidean)."""
        g = self._gallery()
        if Qd.shape[1] != g.ld:
            raise ValueError("query layout does not match the gallery")
        with _DEVICE_LOCK:
            sh = self._shard_info()
            return g.search(Qd, k) if sh is None else self._search_sharded(g, Qd, k, sh)

    def __getstate__(self):
        st = dict(self.__dict__)
        for key in ("_dev", "_shard", "_dev_f32", "_chi2_denom"):   # derived state, never pickled
            st.pop(key, None)
        return st

    def __repr__(self):
        return "NearestNeighbor (k=%s, dist_metric=%s)" % (self.k, repr(self.dist_metric))


# the ROS recognizer calls predict from a rospy callback thread (ocvf_recognizer_ros.py:96-116)
_DEVICE_LOCK = threading.RLock()


for _c in (AbstractClassifier, NearestNeighbor):
    _c.__module__ = "ocvfacerec.facerec.classifier"
