"""BASELINE.json configs exercised at (or near) their own sizes on the GPU.

* configs[1]: 100x100 faces, 10k identities x 10 = 100k gallery, d = 9999, B = 4096 through
  PredictableModel.predict_batch (projection + certified search chain); 64 sampled queries
  against the float64 oracle, every query's identity and the per-tier certificate counts -- with a
  random W and (round 5) with the Fisherfaces W trained on the gallery's own faces (the reference
  trainer's model, thetrainer.py:120-124: its LDA columns put most of the feature variance into the
  leading blocks, which the fp6 tier's column-block scales absorb).
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
@pytest.mark.parametrize("w", ["random", "trained"])
def test_config1_100k_gallery_d9999_batch4096(monkeypatch, w):
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank, build_trained_projection
    monkeypatch.setenv("OFR_SEARCH", "auto")
    dev = torch.device("cuda", 0)
    ids, per, side, d, B = 10_000, 10, 100, 9999, 4096
    N, D = ids * per, side * side
    bank = IdentityBank(ids, side, side, device=dev)
    if w == "trained":
        _, Wt, info = build_trained_projection(bank, per, N, D, dev)
        assert info["regime"] == "pixel" and Wt.shape == (d, D), info
        W = Wt.t().cpu().numpy()
        del Wt
    else:
        r = np.random.default_rng(SEED + 31)
        W = r.normal(0, 1 / np.sqrt(D), (D, d))
    model = _fisher_model(W)
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
    print(f"configs[1] W={w}: uncertified after each tier {counts}, top-1 identity accuracy {acc}")
    assert acc >= 0.99, acc
    assert counts[0] <= B // 100, counts          # identity-bank data: the fp6 tier certifies almost all
    if w == "trained":
        bs = g._block_scales()
        assert bs is not None and int(bs.min()) < 127   # the trained W's variance profile is absorbed
        # the bench's path on the trained W: the prefix tier first (FloatGallery.start_tier), certifying all
        assert g.prefix_stages() >= 1 and g.last_start_tier == "f6p", (g.prefix_stages(), g.last_start_tier)
        assert counts[0] == 0, counts
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
# configs[2] at full size: 1M x 9999 gallery in two 500k shards, B = 4096
# ---------------------------------------------------------------------------
C2 = dict(N=1_000_000, per=10, side=100, d=9999, B=4096, k=1)


def _c2_setup(dev):
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank, build_projection
    n_ids = C2["N"] // C2["per"]
    P, _ = build_projection(C2["side"] ** 2, C2["d"], dev)
    bank = IdentityBank(n_ids, C2["side"], C2["side"], device=dev)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    ids_q = torch.randint(0, n_ids, (C2["B"],), generator=gq, device=dev)
    return P, bank, ids_q, bank.images(ids_q, seed=SEED + 99)


def _c2_worker(rank, ws, port, out):
    """bench.py's sharded step on one rank: gallery rows [r N/G, (r+1) N/G), this rank's block of the
    query batch projected + quantized and all-gathered, the fp6 tile pass, the pruned split merge,
    the global certificate and the collective fallback chain."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from opencv_facerecognizer_amd._device import round_up
        from opencv_facerecognizer_amd.parallel import (certify_sharded, gather_rows, merge_sharded, shard_range,
                                                        share_block_scales)
        from opencv_facerecognizer_amd.synthetic import build_gallery
        dev = torch.device("cuda", 0)
        N, d, B, k = C2["N"], C2["d"], C2["B"], C2["k"]
        P, bank, ids_q, Xq = _c2_setup(dev)
        n0, n1 = shard_range(N, rank, ws)
        g = build_gallery(P, bank, C2["per"], n0, n1 - n0, N, d, max(32, round_up(d, 32)), dev)
        print(f"config2 rank {rank}: shard of {g.N} rows built", flush=True)
        share_block_scales(g)            # the fp6 query panels are all-gathered: one set of block scales
        b0, b1 = shard_range(B, rank, ws)
        Qd_loc = P.project(Xq[b0:b1], shift64=g.shift64)
        qq = g.gather_queries(g.quantize_queries(Qd_loc, tier="f6"))
        Qd = gather_rows(Qd_loc)
        g.search_q8_phase(1, Qd, qq, k, n0)
        out_ = (torch.empty((B, k), dtype=torch.float64, device=dev), torch.empty((B, k), dtype=torch.int64, device=dev))
        merge_sharded(g, Qd, qq, k, n0, out_)
        (md, mi), counts = certify_sharded(g, Qd, qq, k, out_, n0)
        kept = g.sieve_counts(B)
        torch.cuda.synchronize()
        out.put((rank, md.cpu().numpy(), mi.cpu().numpy(), counts, g.N, int(kept.max())))
    finally:
        dist.destroy_process_group()


def _c2_exact_top1(sample, setup=None):
    """float64 top-1 of the sampled queries over the WHOLE 1M gallery (the reference's features,
    feature.py:241-242, exact projection in fp64), streamed in chunks: ||g||^2 - 2 q.g on the host
    (numpy BLAS) shortlists 32 rows per chunk, distance.py:60 (the oracle) ranks the shortlist.
    setup: (P, bank, ids_q, Xq) of the caller (the trained W), else _c2_setup's random W."""
    from opencv_facerecognizer_amd.synthetic import gallery_centre, gallery_chunks
    dev = torch.device("cuda", 0)
    P, bank, ids_q, Xq = setup if setup is not None else _c2_setup(dev)
    centre = gallery_centre(P, bank, C2["per"], C2["N"], dev)
    Q = P.project(Xq[torch.from_numpy(sample).to(dev)], shift64=centre, f64=True).cpu().numpy()
    best_d = np.full(len(sample), np.inf)
    best_i = np.full(len(sample), -1, np.int64)
    second = np.full(len(sample), np.inf)
    for c0, Y in gallery_chunks(P, bank, C2["per"], 0, C2["N"], C2["N"], centre, f64=True):
        if c0 % (16 * 8192) == 0:
            print(f"config2 oracle: gallery rows {c0}/{C2['N']}", flush=True)   # progress (long test)
        G = Y.cpu().numpy()
        S = np.einsum("ij,ij->i", G, G)[None, :] - 2.0 * (Q @ G.T)
        cand = np.argpartition(S, 32, axis=1)[:, :32]
        for b in range(len(sample)):
            for j in cand[b]:
                dj = O.euclidean(G[j].reshape(-1, 1), Q[b].reshape(-1, 1))
                if dj < best_d[b] or (dj == best_d[b] and c0 + j < best_i[b]):
                    second[b] = best_d[b]
                    best_d[b], best_i[b] = dj, c0 + j
                elif dj < second[b]:
                    second[b] = dj
    return best_i, best_d, second, ids_q.cpu().numpy()


@pytest.mark.timeout(1200)
def test_config2_full_size_two_rank_sharded():
    """BASELINE configs[2] at its own size through bench.py's sharded step: 2 gloo ranks on the box's
    one device, each holding 500,000 of the 1,000,000 rows (d = 9,999), a 4,096-face batch.
    Properties on the whole batch (both ranks return the same global top-1, uncertified counts,
    identity accuracy) and 64 sampled queries against the float64 top-1 over the whole gallery
    (classifier.py:104-119 + distance.py:57-60), with the near-tie rule of _check_search."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c2_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=900)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (md0, mi0, c0_, n_0, kept0), (md1, mi1, c1_, n_1, kept1) = res[0], res[1]
    assert n_0 == n_1 == C2["N"] // 2
    assert np.array_equal(mi0, mi1) and np.array_equal(md0, md1)     # the global result on both ranks
    assert list(c0_) == list(c1_) and c0_[0] <= C2["B"] // 100, c0_  # identity data: fp6 certifies ~all
    assert max(kept0, kept1) <= 32768
    sample = np.random.default_rng(6).choice(C2["B"], 64, replace=False)
    ri, rd, r2, ids_q = _c2_exact_top1(sample)
    acc = float(np.mean(mi0[:, 0] // C2["per"] == ids_q))
    assert acc >= 0.99, acc
    near = (r2 - rd) <= 1e-4 * rd
    assert np.all((mi0[sample, 0] == ri) | near), (mi0[sample, 0], ri)
    assert np.allclose(md0[sample, 0], rd, rtol=1e-4, atol=0)


@pytest.mark.timeout(1200)
def test_config2_headline_path_trained_w_full_size():
    """The measured headline path itself (bench.py at N = 1): the Fisherfaces W trained
    on configs[1]'s 100k faces, the 1M-row gallery (d = 9,999), one 4,096-face batch through the bench's
    single-GPU step -- exact projection, the adaptive start tier, the prefix tier f6p on the persistent sieve
    pass, merge + exact re-rank + certificate, the fallback chain.  Asserts that the batch starts at f6p,
    that the prefix pass kernel is the one launched, that every query certifies there, identity accuracy,
    and 64 sampled queries against the float64 top-1 over the WHOLE gallery (classifier.py:104-119,
    distance.py:57-60, feature.py:241-242) with the near-tie rule of _check_search."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import round_up
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank, build_gallery, build_trained_projection
    dev = torch.device("cuda", 0)
    N, per, side, d, B = C2["N"], C2["per"], C2["side"], C2["d"], C2["B"]
    bank = IdentityBank(N // per, side, side, device=dev)
    P, _, info = build_trained_projection(bank, per, 100_000, side * side, dev)
    assert P.d == d and info["regime"] == "pixel", info
    g = build_gallery(P, bank, per, 0, N, N, d, max(32, round_up(d, 32)), dev)
    print(f"headline: W trained ({info['train_s']:.1f} s), gallery of {g.N} rows built", flush=True)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    ids_q = torch.randint(0, N // per, (B,), generator=gq, device=dev)
    Xq = bank.images(ids_q, seed=SEED + 99)
    Qd = P.project(Xq, shift64=g.shift64)                 # bench.py prep(): fp32(W^T x - c), exact int8 MFMA
    pst = g.prefix_stages()
    tier = g.start_tier(B)
    assert pst >= 1 and tier == "f6p", (pst, tier)
    name = _lib.load().ofr_f6p_sieve_kernel(pst)
    name = name.decode() if isinstance(name, bytes) else str(name)
    assert "prefix" in name, name                          # the persistent prefix pass, not the f6w fallback
    qq = g.quantize_queries(Qd, tier=tier)
    out = g.search_q8_phase(3, Qd, qq, 1)
    first = g.fallback(Qd, qq, 1, out)
    kept = g.sieve_counts(B).cpu().numpy()
    md, mi = out[0].cpu().numpy(), out[1].cpu().numpy()
    print(f"headline: prefix stages {pst}, uncertified after each tier {g.last_fallbacks}, "
          f"kept rows per query mean {kept.mean():.0f} max {kept.max()}", flush=True)
    assert first == 0 and list(g.last_fallbacks) == [0], g.last_fallbacks
    assert kept.max() <= g.SIEVE_CAP
    acc = float(np.mean(mi[:, 0] // per == ids_q.cpu().numpy()))
    assert acc >= 0.99, acc
    sample = np.random.default_rng(6).choice(B, 64, replace=False)
    ri, rd, r2, _ = _c2_exact_top1(sample, setup=(P, bank, ids_q, Xq))
    near = (r2 - rd) <= 1e-4 * rd
    assert np.all((mi[sample, 0] == ri) | near), (mi[sample, 0], ri)
    assert np.allclose(md[sample, 0], rd, rtol=1e-4, atol=0)


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


@pytest.mark.timeout(1200)
def test_config4_training_full_100k_default_solver_vs_eigh(monkeypatch):
    """Full configs[4]: 100,000 faces of 10,000 identities, D = 10,000 -> W 10,000 x 9,999, trained
    twice: with the DEFAULT solver (OFR_LDA_SOLVER=auto: above order 1024 the pencil
    Sb v = lambda Sw v on the device, rocSOLVER dsygvd -- the path behind configs[4]'s timing) and
    with the host LAPACK pencil (scipy sygvd).  feature.py:170-176 asks for the eigenpairs of
    inv(Sw) Sb; both solvers give the same pencil's, columns at unit 2-norm.  Checked: the
    eigenvalues agree, the W columns of well-separated eigenvalues agree up to sign
    (|cos| > 1 - 1e-6), the resubstitution labels of the two models are equal, and fresh faces are
    recognised."""
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    n, c, side = 100_000, 10_000, 100
    X, y = _faces(n, c, side, 20261015 + 21)
    Xl = list(X)
    models = {}
    for solver in ("auto", "eigh"):
        print(f"config4: training with OFR_LDA_SOLVER={solver}", flush=True)   # progress (long test)
        monkeypatch.setenv("OFR_LDA_SOLVER", solver)
        model = PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))
        model.compute(Xl, y)
        W = np.asarray(model.feature._eigenvectors)
        assert W.shape == (side * side, c - 1) and np.isfinite(W).all(), solver
        models[solver] = model
    Wa, We = (np.asarray(models[s].feature._eigenvectors) for s in ("auto", "eigh"))
    ea, ee = (np.asarray(models[s].feature._eigenvalues, np.float64) for s in ("auto", "eigh"))
    assert np.allclose(ea, ee, rtol=1e-4, atol=1e-6 * ee.max())
    gap = np.minimum(np.abs(np.diff(np.r_[np.inf, ee])), np.abs(np.diff(np.r_[ee, -np.inf])))
    ok = gap > 1e-3 * ee.max()
    cos = np.abs(np.einsum("ij,ij->j", Wa, We)) / (np.linalg.norm(Wa, axis=0) * np.linalg.norm(We, axis=0))
    assert ok.sum() >= 3 and np.all(cos[ok] > 1 - 1e-6), (ok.sum(), cos[ok].min())
    # resubstitution (every 6th training face, 4,096 per batch): equal labels under both models
    sel = np.arange(0, n, 6)
    lab = {s: np.concatenate([[p[0] for p in models[s].predict_batch(X[sel[i:i + 4096]])]
                              for i in range(0, len(sel), 4096)]) for s in models}
    assert np.array_equal(lab["auto"], lab["eigh"])
    assert np.mean(lab["auto"] == y[sel]) >= 0.999
    Xq, yq = _faces(4096, c, side, 20261015 + 24)
    labels = np.array([p[0] for p in models["auto"].predict_batch(Xq)])
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


def _sharded_train_worker(rank, ws, port, out, shape=(400, 20, 12, 1300)):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from ocvfacerec.facerec.feature import Fisherfaces
        from opencv_facerecognizer_amd.parallel import shard_range, train_fisherfaces_sharded
        n, c, side, seed = shape
        X, y = _small_faces(n, c, side, seed)
        n0, n1 = shard_range(len(y), rank, ws)
        ff = Fisherfaces()
        feats = train_fisherfaces_sharded(ff, list(X[n0:n1]), y[n0:n1], c)
        out.put((rank, np.asarray(ff._eigenvectors), np.asarray(ff._eigenvalues),
                 np.stack([np.asarray(f).reshape(-1) for f in feats]), ff._regime))
    finally:
        dist.destroy_process_group()


def _run_sharded_training(shape, ws=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_train_worker, args=(r, ws, port, q, shape)) for r in range(ws)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(ws):
        item = q.get(timeout=240)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(300)
@pytest.mark.parametrize("regime,shape", [("cov", (200, 80, 12, 1100)), ("gram", (120, 12, 12, 1020))])
def test_sharded_training_cov_and_gram_regimes(regime, shape):
    """VERDICT r3 missing #4: train_fisherfaces_sharded outside the pixel regime, 2 gloo ranks sharing the
    device.  cov (n > D, n - c < D): the covariance all-reduced exactly, the LDA scatter of the
    features all-reduced (global class means, per-rank centred products); gram (n <= D): the faces
    gathered, rank 0 runs the n x n Gram pipeline.  Against the single-process Fisherfaces.compute
    (feature.py:211-235): eigenvalues, W columns of distinct eigenvalues, the features of each rank's
    faces; the same model on every rank."""
    from ocvfacerec.facerec.feature import Fisherfaces
    res = _run_sharded_training(shape)
    n, c, side, seed = shape
    X, y = _small_faces(n, c, side, seed)
    ff = Fisherfaces()
    feats = ff.compute(list(X), y)
    assert ff._regime == regime and res[0][3] == regime and res[1][3] == regime
    W, ev = np.asarray(ff._eigenvectors), np.asarray(ff._eigenvalues, np.float64)
    for r in (0, 1):
        assert np.array_equal(res[r][0], res[0][0]) and np.array_equal(res[r][1], res[0][1])
    evs = np.asarray(res[0][1], np.float64)
    assert np.allclose(evs, ev, rtol=1e-5, atol=1e-7 * ev.max())
    gap = np.minimum(np.abs(np.diff(np.r_[np.inf, ev])), np.abs(np.diff(np.r_[ev, -np.inf])))
    ok = gap > 1e-3 * ev.max()
    Ws = res[0][0]
    cos = np.abs(np.sum(Ws * W, 0)) / (np.linalg.norm(Ws, axis=0) * np.linalg.norm(W, axis=0))
    assert ok.sum() >= 3 and np.all(cos[ok] > 1 - 1e-7), (cos[ok].min(), ok.sum())
    if regime == "gram":                                  # the same pipeline on the same faces
        assert np.array_equal(Ws, W)
    F = np.stack([np.asarray(f).reshape(-1) for f in feats])
    Fs = np.concatenate([res[0][2], res[1][2]])
    Fr = X.reshape(n, -1).astype(np.float64) @ Ws           # each rank's features are W^T x of its faces
    assert np.allclose(Fs, Fr, rtol=0, atol=1e-7 * np.abs(Fr).max())
    assert Fs.shape == F.shape


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


@pytest.mark.timeout(300)
def test_projection_bench_shape_vs_float64():
    """the projection at the bench shape (B = 4,096 faces, D = 10,000, d = 9,999 --
    the 1,680-tile grid of the wide int8 engine, feature.py:241-242) against float64 X @ W on the
    host for 64 sampled faces (not the device's own f64 path), the shifted fp32 search rows (the
    bench's form: W^T x - c rounded once) against the same float64 reference, and the batch's
    faces being independent of their position in the batch (a slice projected alone)."""
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank, build_projection
    dev = torch.device("cuda", 0)
    D, d, B = 10000, 9999, 4096
    P, Wt = build_projection(D, d, dev)
    bank = IdentityBank(100_000, 100, 100, device=dev)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    X = bank.images(torch.randint(0, 100_000, (B,), generator=gq, device=dev), seed=SEED + 99)
    X[17] = 255                                                  # saturated and empty faces
    X[18] = 0
    c = torch.from_numpy(np.random.default_rng(3).normal(0, 2, d)).to(dev)
    Y64 = P.project(X, f64=True)
    Y32 = P.project(X, shift64=c)
    torch.cuda.synchronize()
    s = np.unique(np.concatenate([[0, 17, 18, 255, 256, 4095], np.random.default_rng(8).choice(B, 58, replace=False)]))
    W = Wt.double().cpu().numpy().T                              # D x d, the fp32 weights in float64
    Xs = X[torch.from_numpy(s).to(dev)].cpu().numpy().reshape(len(s), -1).astype(np.float64)
    ref = Xs @ W
    got = Y64[torch.from_numpy(s).to(dev)].cpu().numpy()
    nrm = np.maximum(np.linalg.norm(ref, axis=1), 1.0)
    err = np.abs(got - ref).max(axis=1) / nrm
    assert err.max() < 1e-7, (err.max(), s[np.argmax(err)])
    ref32 = (ref - c.cpu().numpy()).astype(np.float32)
    got32 = Y32[torch.from_numpy(s).to(dev)].cpu().numpy()[:, :d]
    tol = 2.0 ** -23 * np.abs(ref - c.cpu().numpy()) + 1e-7 * nrm[:, None]
    assert np.all(np.abs(got32.astype(np.float64) - ref32.astype(np.float64)) <= tol)
    # a slice of the batch projected alone gives the same bits (no dependence on the tile position)
    part = P.project(X[1000:1300], f64=True)
    assert torch.equal(part, Y64[1000:1300])


@pytest.mark.timeout(600)
def test_config3_lbph_chi2_full_size():
    """BASELINE configs[3] at its own size (VERDICT r3 missing #3): ExtendedLBP(1, 8) + SpatialHistogram
    8x8 of 65,536 gallery faces at 128 x 128 and 4,096 query faces, ChiSquare 1-NN (feature.py:286-302,
    distance.py:112-116, classifier.py:104-119).  Histograms bit-exact against the oracle for sampled
    faces; every query certified by the fp16-MFMA pass; identity accuracy; 32 sampled queries against
    the oracle's chi-square over the whole gallery (a device fp64 shortlist of the reference formula,
    then the oracle on the shortlist and on the returned row), with the near-tie rule of _check_search."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import Chi2Gallery
    from opencv_facerecognizer_amd.facerec.feature import SpatialHistogram
    from opencv_facerecognizer_amd.facerec.lbp import ExtendedLBP
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank
    dev = torch.device("cuda", 0)
    N, B, H, per = 65536, 4096, 128, 8
    bank = IdentityBank(N // per, H, H, device=dev)
    G_img = bank.images(torch.arange(N, device=dev) // per, seed=SEED + 11).reshape(N, H, H)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 12)
    ids_q = torch.randint(0, N // per, (B,), generator=gq, device=dev)
    Q_img = bank.images(ids_q, seed=SEED + 13).reshape(B, H, H)
    sh = SpatialHistogram(ExtendedLBP(1, 8), (8, 8))
    gc, cell, cb = sh.counts_device(G_img)
    qc, _, _ = sh.counts_device(Q_img)
    assert cell == 225 and cb == 1
    nb = gc.shape[1] * gc.shape[2]
    for i in (0, 4097, 65535):                                   # bit-exact histograms (feature.py:298-299)
        assert np.array_equal(gc[i].reshape(-1).cpu().numpy() / 225.0, O.spatial_histogram(G_img[i].cpu().numpy()))
    assert np.array_equal(qc[7].reshape(-1).cpu().numpy() / 225.0, O.spatial_histogram(Q_img[7].cpu().numpy()))
    gal = Chi2Gallery(gc.reshape(N, nb), dtype=_lib.DT_U8, denom=float(cell), nbins=nb)
    Qc = qc.reshape(B, nb).contiguous()
    dd, ii = gal.search(Qc, 1)
    torch.cuda.synchronize()
    assert list(gal.last_fallbacks)[0] == 0, gal.last_fallbacks        # every query certified by the MFMA pass
    acc = float(((ii[:, 0] // per) == ids_q).double().mean().item())
    assert acc >= 0.99, acc
    s = np.sort(np.random.default_rng(17).choice(B, 32, replace=False))
    Gf = gc.reshape(N, nb)
    short = []
    for b in s:                                                   # device fp64 shortlist: best 8 rows
        q = Qc[b].double() / 225.0
        best = []
        for c0 in range(0, N, 8192):
            g = Gf[c0:c0 + 8192].double() / 225.0
            dist = ((g - q) ** 2 / (g + q + np.finfo(np.float64).eps)).sum(1)
            v, j = torch.topk(dist, 8, largest=False)
            best.append(torch.stack([v, (j + c0).double()], 1))
        allb = torch.cat(best)
        short.append(allb[torch.argsort(allb[:, 0])[:8], 1].long().cpu().numpy())
    dd_h, ii_h = dd.cpu().numpy()[:, 0], ii.cpu().numpy()[:, 0]
    for b, cand in zip(s, short):
        qh = Qc[b].cpu().numpy() / 225.0
        rows = np.unique(np.append(cand, ii_h[b]))
        ref = np.array([O.chisquare(Gf[j].cpu().numpy() / 225.0, qh) for j in rows])
        o = np.lexsort((rows, ref))
        best_row, best_d = rows[o[0]], ref[o[0]]
        mine = ref[np.searchsorted(rows, ii_h[b])]
        assert abs(dd_h[b] - mine) <= 1e-9 * mine, (b, dd_h[b], mine)             # exact re-rank of its row
        assert ii_h[b] == best_row or mine <= best_d * (1 + 1e-4), (b, ii_h[b], best_row, mine, best_d)
