"""BASELINE.json configs exercised at (or near) their own sizes on the GPU.

* configs[1]: 100x100 faces, 10k identities x 10 = 100k gallery, d = 9999, B = 4096 through
  PredictableModel.predict_batch (projection + certified search chain); 64 sampled queries
  against the float64 oracle, every query's identity and the per-tier certificate counts.
* configs[2]: the 1M-gallery sharding path -- parallel.certify_sharded on 2 gloo ranks sharing
  one device (the OFR_ONE_DEVICE rehearsal), with the REAL FloatGallery on data where only
  rank 1's fp6 sieve bucket overflows: the query must go down the chain, never be certified
  from the -inf bound (reference semantics: the k nearest of the whole gallery,
  classifier.py:104-119).
* configs[4]: Fisherfaces training at n = 4,000, D = 10,000, c = 400 against the oracle (PCA mean
  exact, eigenvalues, Sw / Sb, resubstitution), and at the full n = 100,000, c = 10,000 through
  property checks (shapes, finiteness, identity accuracy).
"""
import os
import socket

import numpy as np
import pytest
import torch

import facerec_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    torch.cuda.set_device(0)


def _exact_top1(Q, G, cand=32):
    """Oracle top-1 (distance.py:60 in float64) of each query: BLAS candidates, then the exact
    direct-difference distance on them (the BLAS form is only used to shortlist)."""
    g2 = np.einsum("ij,ij->i", G, G)
    S = g2[None, :] - 2.0 * (Q @ G.T)
    out_i, out_d, second = [], [], []
    for b in range(len(Q)):
        c = np.argpartition(S[b], cand)[:cand]
        d = np.array([O.euclidean(G[j].reshape(-1, 1), Q[b].reshape(-1, 1)) for j in c])
        o = np.lexsort((c, d))
        out_i.append(c[o[0]])
        out_d.append(d[o[0]])
        second.append(d[o[1]])
    return np.array(out_i), np.array(out_d), np.array(second)


def _fisher_model(W):
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    ff = Fisherfaces()
    ff._eigenvectors = np.asmatrix(W)
    ff._num_components = W.shape[1]
    ff._eigenvalues = np.ones(W.shape[1], np.float32)
    return PredictableModel(ff, NearestNeighbor(EuclideanDistance(), k=1))


@pytest.mark.timeout(600)
def test_config1_100k_gallery_d9999_batch4096(monkeypatch):
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank
    monkeypatch.setenv("OFR_SEARCH", "auto")
    dev = torch.device("cuda", 0)
    ids, per, side, d, B = 10_000, 10, 100, 9999, 4096
    N, D = ids * per, side * side
    r = np.random.default_rng(SEED + 31)
    W = r.normal(0, 1 / np.sqrt(D), (D, d))
    model = _fisher_model(W)
    bank = IdentityBank(ids, side, side, device=dev)
    feats = np.empty((N, d))
    for c0 in range(0, N, 8192):
        rows = torch.arange(c0, min(N, c0 + 8192), device=dev)
        imgs = bank.images(rows // per, seed=SEED + 1000 + c0)
        feats[c0:c0 + len(rows)] = model.feature.project_device(imgs, f64=True).cpu().numpy()
    model.classifier.compute(list(feats), np.arange(N) // per)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 37)
    ids_q = torch.randint(0, ids, (B,), generator=gq, device=dev)
    Xq = bank.images(ids_q, seed=SEED + 99).reshape(B, side, side)
    dist, idx = model.search_batch(Xq)
    g = model.classifier._gallery()
    counts = list(g.last_fallbacks)
    acc = float(np.mean(idx[:, 0] // per == ids_q.cpu().numpy()))
    assert acc >= 0.99, acc
    assert counts[0] <= B // 100, counts          # identity-bank data: the fp6 tier certifies almost all
    s = np.random.default_rng(5).choice(B, 64, replace=False)
    Qf = model.feature.project_device(Xq[torch.from_numpy(s).to(dev)], f64=True).cpu().numpy()
    ri, rd, r2 = _exact_top1(Qf, feats)
    near = (r2 - rd) <= 1e-4 * rd
    assert np.all((idx[s, 0] == ri) | near), (idx[s, 0], ri)
    assert np.allclose(dist[s, 0], rd, rtol=1e-4, atol=1e-6 * np.linalg.norm(Qf, axis=1).max())


# ---------------------------------------------------------------------------
# configs[2]: sharded certificate with a real overflowing shard
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _overflow_data():
    r = np.random.default_rng(1234)
    d = 96
    x = r.normal(0, 20, d)
    G = np.concatenate([r.normal(0, 20, (34000, d)), np.tile(x, (34000, 1))]).astype(np.float32).astype(np.float64)
    Q = (x + r.normal(0, 0.5, (40, d))).astype(np.float32).astype(np.float64)
    return Q, G


def _shard_worker(rank, ws, port, k, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from opencv_facerecognizer_amd import _lib
        from opencv_facerecognizer_amd._device import FloatGallery, center_round, f64_dev, round_up
        from opencv_facerecognizer_amd.parallel import certify_sharded, shard_range
        Q, G = _overflow_data()
        n0, n1 = shard_range(len(G), rank, ws)
        # every rank centres on the same vector (the global mean), as bench.py does
        shift = f64_dev(G.mean(0))
        Gd = center_round(f64_dev(G[n0:n1]), shift, max(32, round_up(G.shape[1], 32)))
        g = FloatGallery.from_device_rows(Gd, G.shape[1], _lib.METRIC_EUCLIDEAN, shift64=shift)
        Qd = center_round(f64_dev(Q), shift, g.ld)
        qq = g.quantize_queries(Qd, tier="f6")
        local = g.search_q8_phase(3, Qd, qq, k, index_base=n0)
        kept = g.sieve_counts(len(Q)).cpu().numpy()
        (md, mi), counts = certify_sharded(g, Qd, qq, k, local, n0)
        torch.cuda.synchronize()
        out.put((rank, md.cpu().numpy(), mi.cpu().numpy(), counts, int(kept.max()),
                 qq["bound"].cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_config2_sharded_overflow_rank_not_certified():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    k = 3
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=240)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    Q, G = _overflow_data()
    md, mi, counts, kept1, bound1 = res[1]
    assert kept1 > 32768 and np.all(np.isneginf(bound1))      # rank 1 overflowed on every query
    assert np.all(np.isfinite(res[0][4]))                      # rank 0 did not
    assert counts[0] == len(Q)                                  # so nothing certified at the first tier
    assert np.array_equal(res[0][1], mi)                        # both ranks hold the same merged result
    assert (mi == np.arange(34000, 34000 + k)).all()            # the duplicates, lowest index first
    ref = np.sqrt(((G[34000] - Q) ** 2).sum(1))
    assert np.allclose(md[:, 0], ref, rtol=1e-6)


# ---------------------------------------------------------------------------
# configs[4]: training
# ---------------------------------------------------------------------------
def _faces(n, ids, side, seed):
    from opencv_facerecognizer_amd.synthetic import IdentityBank
    dev = torch.device("cuda", 0)
    y = torch.arange(n, device=dev) % ids
    X = IdentityBank(ids, side, side, device=dev).images(y, seed=seed).reshape(n, side, side).cpu().numpy()
    return X, y.cpu().numpy()


@pytest.mark.timeout(600)
def test_config4_training_4k_vs_oracle():
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import LDA, PCA, Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    n, c, side = 4000, 400, 100
    X, y = _faces(n, c, side, 20261015 + 21)
    Xl = list(X)
    # PCA stage vs the oracle (feature.py:83-108): exact mean, eigenvalues
    pca = PCA(n - c)
    pf = pca.compute(Xl, y)
    A = X.reshape(n, -1).astype(np.float64)
    mean = A.mean(0)
    assert np.array_equal(np.asarray(pca.mean).reshape(-1), mean)
    s = np.linalg.svd(A - mean, compute_uv=False)
    ev = (s ** 2 / n)[: n - c]
    assert np.allclose(pca.eigenvalues[:50], ev[:50], rtol=1e-9)
    # LDA scatter at this size vs the oracle (feature.py:160-168)
    F = np.stack([np.asarray(f).reshape(-1) for f in pf])
    Sw, Sb, _ = LDA.scatter(list(F), y)
    _, oSw, oSb = O.lda_scatter(F.T, y)
    assert np.abs(Sw - oSw).max() <= 1e-10 * np.abs(oSw).max()
    assert np.abs(Sb - oSb).max() <= 1e-10 * np.abs(oSb).max()
    # the full training call and resubstitution
    model = PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))
    model.compute(Xl, y)
    W = np.asarray(model.feature._eigenvectors)
    assert W.shape == (side * side, c - 1) and np.isfinite(W).all()
    labels = np.array([p[0] for p in model.predict_batch(X)])
    assert np.mean(labels == y) >= 0.999
    feats = np.stack([np.asarray(f).reshape(-1) for f in model.classifier.X])
    Qf = model.feature.project_device(X[:64], f64=True).cpu().numpy()
    ri, _, _ = _exact_top1(Qf, feats)
    assert np.array_equal(labels[:64], y[ri])


@pytest.mark.timeout(900)
def test_config4_training_full_100k(monkeypatch):
    """Full configs[4]: 100,000 faces of 10,000 identities, D = 10,000 -> W 10,000 x 9,999 (symmetric-
    definite LDA solve: the reference's general eig of a 9,999^2 matrix takes hours on the host)."""
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    monkeypatch.setenv("OFR_LDA_SOLVER", "eigh")
    n, c, side = 100_000, 10_000, 100
    X, y = _faces(n, c, side, 20261015 + 21)
    model = PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))
    model.compute(list(X), y)
    W = np.asarray(model.feature._eigenvectors)
    assert W.shape == (side * side, c - 1) and np.isfinite(W).all()
    Xq, yq = _faces(4096, c, side, 20261015 + 24)
    labels = np.array([p[0] for p in model.predict_batch(Xq)])
    assert np.mean(labels == yq) >= 0.99


# ---------------------------------------------------------------------------
# Fisherfaces training regimes (training.py) against the oracle
# ---------------------------------------------------------------------------
def _small_faces(n, c, side, seed, noise=12.0):
    from opencv_facerecognizer_amd.synthetic import IdentityBank
    dev = torch.device("cuda", 0)
    y = torch.arange(n, device=dev) % c
    X = IdentityBank(c, side, side, device=dev, seed=seed).images(y, seed=seed + 1, noise=noise)
    return X.reshape(n, side, side).cpu().numpy(), y.cpu().numpy()


@pytest.mark.parametrize("regime,n,c,side", [("pixel", 400, 20, 12), ("cov", 200, 80, 12), ("gram", 120, 12, 12)])
def test_fisherfaces_regimes_vs_oracle(regime, n, c, side):
    """Fisherfaces.compute (feature.py:211-235) in each regime of the exact device pipeline against the
    oracle's PCA (SVD) -> LDA (inv + eig) chain: LDA eigenvalues, W columns up to sign (for distinct
    eigenvalues), and the training features."""
    from ocvfacerec.facerec.feature import Fisherfaces
    X, y = _small_faces(n, c, side, 900 + n)
    ff = Fisherfaces()
    feats = ff.compute(list(X), y)
    assert ff._regime == regime
    ref = O.fisherfaces_compute(list(X), y)
    W, Wr = np.asarray(ff._eigenvectors), np.asarray(ref["W"])
    assert W.shape == Wr.shape
    ev, evr = np.asarray(ff._eigenvalues, np.float64), np.asarray(ref["eigenvalues"], np.float64)
    assert np.allclose(ev, evr, rtol=2e-5, atol=1e-6 * evr.max())
    gap = np.minimum(np.abs(np.diff(np.r_[np.inf, evr])), np.abs(np.diff(np.r_[evr, -np.inf])))
    ok = gap > 1e-3 * evr.max()
    cos = np.abs(np.sum(W * Wr, 0)) / (np.linalg.norm(W, axis=0) * np.linalg.norm(Wr, axis=0))
    assert ok.sum() >= 3 and np.all(cos[ok] > 1 - 1e-6), (cos[ok].min(), ok.sum())
    # features are W^T x of the training faces (feature.py:231-235), on the int8-slice projection
    # engine (W cut at 2^-28 of its column maxima: ~1e-8 relative)
    F = np.stack([np.asarray(f).reshape(-1) for f in feats])
    Fr = X.reshape(n, -1).astype(np.float64) @ W
    assert np.allclose(F, Fr, rtol=0, atol=1e-7 * np.abs(Fr).max())


def _sharded_train_worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from ocvfacerec.facerec.feature import Fisherfaces
        from opencv_facerecognizer_amd.parallel import shard_range, train_fisherfaces_sharded
        X, y = _small_faces(400, 20, 12, 1300)
        n0, n1 = shard_range(len(y), rank, ws)
        ff = Fisherfaces()
        feats = train_fisherfaces_sharded(ff, list(X[n0:n1]), y[n0:n1], 20)
        out.put((rank, np.asarray(ff._eigenvectors), np.asarray(ff._eigenvalues),
                 np.stack([np.asarray(f).reshape(-1) for f in feats])))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_training_equals_single_process():
    """SURVEY §8e training exchange on 2 gloo ranks sharing the device: the exact pieces all-reduce
    bit for bit, so W equals the single-process Fisherfaces.compute; each rank returns the features
    of its own faces (its gallery shard)."""
    import torch.multiprocessing as mp
    from ocvfacerec.facerec.feature import Fisherfaces
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=240)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    X, y = _small_faces(400, 20, 12, 1300)
    ff = Fisherfaces()
    feats = ff.compute(list(X), y)
    assert ff._regime == "pixel"
    W = np.asarray(ff._eigenvectors)
    for r in (0, 1):
        assert np.array_equal(res[r][0], res[0][0])                       # the same model on every rank
    assert np.allclose(res[0][0], W, rtol=0, atol=1e-12)
    assert np.array_equal(res[0][1], np.asarray(ff._eigenvalues))
    F = np.stack([np.asarray(f).reshape(-1) for f in feats])
    assert np.allclose(np.concatenate([res[0][2], res[1][2]]), F, rtol=0, atol=1e-9 * np.abs(F).max())
