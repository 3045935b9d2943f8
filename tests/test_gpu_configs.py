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
