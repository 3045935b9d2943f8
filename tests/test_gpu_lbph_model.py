"""LBPH through the reference API, end to end on the GPU:
``PredictableModel(SpatialHistogram(ExtendedLBP(1, 8), (8, 8)), NearestNeighbor(ChiSquareDistance(), k))``
at 128 x 128 (BASELINE configs[3]'s geometry).

Reference: model.py:49-55 (compute / predict), feature.py:266-305 (SpatialHistogram over
ExtendedLBP, lbp.py:80-130), classifier.py:76-129 (NearestNeighbor.predict), distance.py:112-116
(ChiSquareDistance).  The fused path is one ``ofr_elbp_hist`` launch per batch and a counts search
against the counts gallery ``compute`` left on the device.  Checked against:
* the reference's own golden histograms (tests/golden/lbp_golden.npz, made by running the
  reference code) -- bit-exact, as the features ``compute`` returns;
* the oracle's float64 histograms and ChiSquare top-k (``_check_search``: distances within 1e-4,
  indices equal except at oracle near-ties), and the reference-faithful per-item loop
  (``nn_predict_faithful``) for a sample of single-face ``predict`` calls;
* the model after a pickle round trip (gallery rebuilt as counts from the float64 histograms),
  ``update`` (rows appended in place), and float queries that are not counts (fp32 twin).
"""
import os

import numpy as np
import pytest
import torch

import facerec_oracle as O
from test_gpu_parity import _check_search

pytestmark = pytest.mark.gpu

K = 3


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    torch.cuda.set_device(0)


def _faces(golden):
    """20 synthetic identities (coarse prototypes x8 + noise) and the 8 golden 128 x 128 images
    (their own identities 20..27), uint8."""
    r = np.random.Generator(np.random.PCG64(31))
    protos = r.integers(0, 256, (20, 16, 16)).astype(np.float64)
    up = np.kron(protos, np.ones((8, 8)))
    gal = np.clip(up[np.arange(300) % 20] + r.normal(0, 20, (300, 128, 128)), 0, 255).astype(np.uint8)
    qry = np.clip(up[np.arange(70) % 20] + r.normal(0, 20, (70, 128, 128)), 0, 255).astype(np.uint8)
    g = golden("lbp_golden.npz")
    names = sorted(k[4:] for k in g.files if k.startswith("img_") and f"hist_{k[4:]}_r1p8_g8" in g.files
                   and g[k].shape == (128, 128))
    gimg = np.stack([g["img_" + n] for n in names])
    ghist = [g[f"hist_{n}_r1p8_g8"] for n in names]
    X = np.concatenate([gal, gimg])
    y = np.concatenate([np.arange(300) % 20, 20 + np.arange(len(names))])
    return X, y, qry, gimg, ghist


def _model():
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import ChiSquareDistance
    from ocvfacerec.facerec.feature import SpatialHistogram
    from ocvfacerec.facerec.lbp import ExtendedLBP
    from ocvfacerec.facerec.model import PredictableModel
    return PredictableModel(SpatialHistogram(ExtendedLBP(1, 8), (8, 8)), NearestNeighbor(ChiSquareDistance(), k=K))


def _check_predictions(preds, Qh, Gh, y):
    """predict output [label, {'labels', 'distances'}] against the oracle: top-k by _check_search,
    labels by the reference vote (classifier.py:121-123) of the oracle's top-k unless a near-tie
    changed the top-k rows."""
    d = np.array([p[1]["distances"] for p in preds])
    lab = np.array([p[1]["labels"] for p in preds])
    D = O.pairwise("ChiSquareDistance", Qh, Gh)
    order = np.argsort(D, 1, kind="stable")[:, :K]
    # indices are not returned by predict: recover them from the labels + distances of the oracle
    n_ties = 0
    for b, p in enumerate(preds):
        ref_d = D[b, order[b]]
        assert np.allclose(d[b], ref_d, rtol=1e-4, atol=0), (b, d[b], ref_d)
        if np.array_equal(lab[b], y[order[b]]):
            assert p[0] == O._vote(y[order[b]])
        else:
            # differing rows only where the oracle has near-ties at those ranks
            for j in np.nonzero(lab[b] != y[order[b]])[0]:
                assert abs(d[b][j] - ref_d[j]) <= 1e-4 * ref_d[j]
                n_ties += 1
    return n_ties


def test_lbph_model_compute_predict_vs_reference_and_oracle(golden):
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import Chi2Gallery
    X, y, qry, gimg, ghist = _faces(golden)
    model = _model()
    model.compute(list(X), y)
    feats = model.classifier.X
    assert len(feats) == len(X) and all(f.dtype == np.float64 and f.shape == (16384,) for f in feats)
    # the golden images' histograms equal the reference's own output bit for bit
    for h, ref in zip(feats[300:], ghist):
        assert np.array_equal(h, ref)
    for i in range(0, 300, 37):                        # and the synthetic faces' the oracle's
        assert np.array_equal(feats[i], O.spatial_histogram(X[i]))
    # the device gallery is the counts ``compute`` produced (u8 counts, denominator 15 x 15)
    g = model.classifier._gallery()
    assert isinstance(g, Chi2Gallery) and g.dtype == _lib.DT_U8 and g.denom == 225.0 and g.N == len(X)
    # batched predict: one histogram launch + one counts search
    Q = np.concatenate([qry, gimg])
    preds = model.predict_batch(list(Q))
    Qh = np.stack([O.spatial_histogram(q) for q in Q])
    Gh = np.stack(feats)
    _check_predictions(preds, Qh, Gh, y)
    d, i = model.search_batch(list(Q))
    _check_search("ChiSquareDistance", Qh, Gh, d, i, K)
    assert np.array_equal(i[70:, 0], 300 + np.arange(len(gimg)))     # a golden image finds itself
    assert np.all(d[70:, 0] == 0.0)
    # a device face batch takes the same path
    di, ii = model.search_batch(torch.from_numpy(Q).cuda())
    assert np.array_equal(ii, i) and np.array_equal(di, d)
    # single-face predict (model.py:53-55) against the reference-faithful per-item loop
    for b in (0, 13, 41, 69, 72):
        p = model.predict(Q[b])
        ref, _ = O.nn_predict_faithful(list(Gh), y, Qh[b].reshape(-1, 1), "ChiSquareDistance", K)
        assert p[0] == ref[0]
        assert np.array_equal(p[1]["labels"], ref[1]["labels"])
        assert np.allclose(p[1]["distances"], ref[1]["distances"], rtol=1e-4, atol=0)


def test_lbph_model_pickle_update_and_float_queries(golden, tmp_path):
    from ocvfacerec.facerec.serialization import load_model, save_model
    from opencv_facerecognizer_amd import _lib
    X, y, qry, gimg, ghist = _faces(golden)
    model = _model()
    model.compute(list(X[:250]), y[:250])
    # update (classifier.py:65-70): appended float histograms extend the counts gallery in place
    clf = model.classifier
    g0 = clf._gallery()
    for i in range(250, len(X)):
        clf.update(model.feature.extract(X[i]), y[i])
    g1 = clf._gallery()
    assert g1 is g0 and g1.N == len(X) and g1.dtype == _lib.DT_U8
    preds = model.predict_batch(list(qry))
    Gh = np.stack(clf.X)
    Qh = np.stack([O.spatial_histogram(q) for q in qry])
    _check_predictions(preds, Qh, Gh, y)
    # pickle round trip: the float64 histograms come back, the gallery is rebuilt as counts
    path = os.path.join(tmp_path, "lbph.pkl")
    save_model(path, model)
    m2 = load_model(path)
    g2 = m2.classifier._gallery()
    assert g2.dtype == _lib.DT_U8 and g2.denom == 225.0
    p2 = m2.predict_batch(list(qry))
    assert [p[0] for p in p2] == [p[0] for p in preds]
    assert all(np.array_equal(a[1]["distances"], b[1]["distances"]) for a, b in zip(p2, preds))
    # float queries that are not counts / 225 go to an fp32 twin of the counts gallery
    Qf = Qh * (1.0 + 1e-3)
    d, i = m2.classifier.search(Qf)
    _check_search("ChiSquareDistance", Qf, Gh, d, i, K)


def test_lbph_model_mixed_size_batch(golden):
    """a batch of faces of two sizes (the reference predicts any size, one face at a time)
    is grouped by size; the 136 x 136 group has 17 x 17-pixel cells (a different count width and
    denominator than the counts gallery: the float path on the host) -- results equal per-face
    predict, in the batch's order."""
    X, y, qry, gimg, ghist = _faces(golden)
    model = _model()
    model.compute(list(X), y)
    r = np.random.Generator(np.random.PCG64(5))
    big = [np.clip(np.kron(q[::16, ::16].astype(np.float64), np.ones((17, 17))) + r.normal(0, 8, (136, 136)),
                   0, 255).astype(np.uint8) for q in qry[:6]]
    batch = [qry[0], big[0], qry[1], big[1], big[2], qry[2], gimg[0], big[3]]
    got = model.predict_batch(batch)
    assert len(got) == len(batch)
    for g, f in zip(got, batch):
        w = model.predict(f)
        assert g[0] == w[0]
        assert np.array_equal(g[1]["labels"], w[1]["labels"])
        assert np.allclose(g[1]["distances"], w[1]["distances"], rtol=1e-12, atol=0)
