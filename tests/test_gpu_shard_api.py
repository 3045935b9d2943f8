"""Sharding through the reference API (SURVEY §8e, §8f row 2 "sharding on load"):
``NearestNeighbor.shard()`` / ``PredictableModel.shard()`` on 2 gloo ranks sharing the box's one
device.  Every rank keeps the full host model, uploads only its block of gallery rows, predicts
the same queries and must return the global top-k: compared with the float64 oracle
(classifier.py:104-119 over the whole gallery; distance.py:57-60, 74-77, 112-116) and with the
unsharded classifier's labels.  Euclidean runs the certified tiers (a 300-query batch: fp6 sieve,
and 5 queries: the fp6 stream) with the global certificate; Cosine and ChiSquare the local exact
search + one all-gather merge."""
import os
import socket

import numpy as np
import pytest
import torch

import facerec_oracle as O
from test_gpu_parity import _check_search

pytestmark = pytest.mark.gpu

K = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(metric):
    r = np.random.default_rng({"EuclideanDistance": 71, "CosineDistance": 72, "ChiSquareDistance": 73}[metric])
    if metric == "ChiSquareDistance":
        N, d = 2001, 59
        G = r.integers(0, 9, (N, d)) / 64.0
        Q = np.concatenate([G[r.integers(0, N, 150)] + r.integers(0, 2, (150, d)) / 64.0,
                            r.integers(0, 9, (150, d)) / 64.0])
    else:
        N, d = 4001, 48
        protos = r.normal(0, 4, (400, d))
        G = protos[np.arange(N) % 400] + r.normal(0, 1, (N, d))
        Q = protos[r.integers(0, 400, 300)] + r.normal(0, 1, (300, d))
    y = np.arange(N) // 10
    return Q.astype(np.float32).astype(np.float64), G.astype(np.float32).astype(np.float64), y


def _classifier(metric):
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec import distance
    return NearestNeighbor(getattr(distance, metric)(), k=K)


def _worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        res = {}
        for metric in ("EuclideanDistance", "CosineDistance", "ChiSquareDistance"):
            Q, G, y = _data(metric)
            clf = _classifier(metric)
            clf.compute(list(G), y)
            clf.shard()
            for B in (300, 5):
                d, i = clf.search(Q[:B])
                labels = [p[0] for p in clf.predict_batch(Q[:B])]
                res[(metric, B)] = (d, i, labels, clf._gallery().N, clf._gallery().last_fallbacks)
        # the fused model path: Fisherfaces projection + sharded certified search
        from ocvfacerec.facerec.feature import Fisherfaces
        from ocvfacerec.facerec.model import PredictableModel
        X, yf, W = _faces()
        ff = Fisherfaces()
        ff._eigenvectors = np.asmatrix(W)
        ff._eigenvalues = np.ones(W.shape[1])
        ff._num_components = W.shape[1]
        model = PredictableModel(ff, _classifier("EuclideanDistance"))
        model.classifier.compute([ff.project(x.reshape(-1, 1)) for x in X[:-64]], yf[:-64])
        model.shard()
        res["model"] = ([p[0] for p in model.predict_batch(list(X[-64:]))], model.search_batch(list(X[-64:]))[1])
        torch.cuda.synchronize()
        out.put((rank, res))
    finally:
        dist.destroy_process_group()


def _faces():
    r = np.random.default_rng(74)
    ids, per, side, dd = 40, 6, 24, 30
    base = r.integers(40, 200, (ids, side * side))
    X = np.clip(base[np.arange(ids * per) % ids] + r.normal(0, 12, (ids * per, side * side)), 0, 255)
    X = X.astype(np.uint8).reshape(-1, side, side)
    W = r.normal(0, 1, (side * side, dd)) / side
    return X, np.arange(ids * per) % ids, W


@pytest.fixture(scope="module")
def sharded():
    import torch.multiprocessing as mp
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, item = q.get(timeout=400)
        res[rank] = item
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(600)
@pytest.mark.parametrize("metric", ["EuclideanDistance", "CosineDistance", "ChiSquareDistance"])
@pytest.mark.parametrize("B", [300, 5])
def test_sharded_classifier_equals_oracle(sharded, metric, B):
    torch.cuda.set_device(0)
    Q, G, y = _data(metric)
    d0, i0, lab0, n_0, _ = sharded[0][(metric, B)]
    d1, i1, lab1, n_1, _ = sharded[1][(metric, B)]
    assert n_0 + n_1 == len(G) and abs(n_0 - n_1) <= 1          # each rank held half the rows
    assert np.array_equal(i0, i1) and np.array_equal(d0, d1)    # both ranks return the global result
    assert lab0 == lab1
    _check_search(metric, Q[:B], G, d0, i0, K)
    # the same labels as the unsharded classifier (one process, the whole gallery)
    clf = _classifier(metric)
    clf.compute(list(G), y)
    ref = [p[0] for p in clf.predict_batch(Q[:B])]
    dr, ir = clf.search(Q[:B])
    same = (ir == i0).all(1)
    assert same.mean() >= 0.98, same.mean()                     # differences only at oracle near-ties
    assert [a for a, s in zip(lab0, same) if s] == [b for b, s in zip(ref, same) if s]


@pytest.mark.timeout(600)
def test_sharded_predictable_model(sharded):
    torch.cuda.set_device(0)
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    X, yf, W = _faces()
    lab0, idx0 = sharded[0]["model"]
    lab1, idx1 = sharded[1]["model"]
    assert lab0 == lab1 and np.array_equal(idx0, idx1)
    ff = Fisherfaces()
    ff._eigenvectors = np.asmatrix(W)
    ff._eigenvalues = np.ones(W.shape[1])
    ff._num_components = W.shape[1]
    model = PredictableModel(ff, _classifier("EuclideanDistance"))
    model.classifier.compute([ff.project(x.reshape(-1, 1)) for x in X[:-64]], yf[:-64])
    ref = model.search_batch(list(X[-64:]))[1]
    assert (ref == idx0).all(1).mean() >= 0.98
    # against the float64 oracle on the projected features
    F = np.stack([np.asarray(ff.project(x.reshape(-1, 1))).reshape(-1) for x in X])
    Dref = O.pairwise("EuclideanDistance", F[-64:], F[:-64])
    assert (np.argsort(Dref, 1, kind="stable")[:, 0] == idx0[:, 0]).mean() >= 0.98
