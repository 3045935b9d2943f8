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
        # the pruned split merge (parallel.merge_sharded) against the plain per-rank merge, on the
        # same shard: identical global results; the pruned local lists skip foreign queries
        from opencv_facerecognizer_amd.parallel import certify_sharded, merge_sharded
        Q, G, y = _identity_blocks()
        clf = _classifier("EuclideanDistance")
        clf.compute(list(G), y)
        clf.shard()
        g = clf._gallery()
        Qd = g.query_rows(Q)
        qa = g.quantize_queries(Qd, tier="f6")
        plain = g.search_q8_phase(3, Qd, qa, K, g.index_base)
        (pd, pi), pc = certify_sharded(g, Qd, qa, K, plain, g.index_base)
        qb = g.quantize_queries(Qd, tier="f6")
        loc = g.search_q8_phase(1, Qd, qb, K, g.index_base)
        merge_sharded(g, Qd, qb, K, g.index_base, loc)
        skipped = int(torch.isinf(loc[0][:, 0]).sum())
        (rd, ri), rc = certify_sharded(g, Qd, qb, K, loc, g.index_base)
        res["pruned"] = (pd.cpu().numpy(), pi.cpu().numpy(), pc, rd.cpu().numpy(), ri.cpu().numpy(), rc, skipped)
        # round 6: the prefix tier on a sharded gallery whose shards ALONE would choose different prefixes
        # (the choice now comes from all-reduced block sums, so both ranks start at f6p and their
        # collectives match), and its pruned split merge (ofr_knn_f6p_merge_pruned) against the plain one
        from opencv_facerecognizer_amd._device import FloatGallery
        Q, G, y = _split_prefix_data()
        clf = _classifier("EuclideanDistance")
        clf.compute(list(G), y)
        clf.shard()
        g = clf._gallery()
        own = FloatGallery.choose_prefix(g.block_sums().cpu().numpy(), g.d, g.N)   # this shard's own choice
        d, i = clf.search(Q)
        res["prefix"] = (d, i, g.prefix_stages(), own, g.last_start_tier, tuple(g.last_fallbacks))
        Qd = g.query_rows(Q)
        qa = g.quantize_queries(Qd, tier="f6p")
        plain = g.search_q8_phase(3, Qd, qa, K, g.index_base)
        (pd, pi), pc = certify_sharded(g, Qd, qa, K, plain, g.index_base)
        qb = g.quantize_queries(Qd, tier="f6p")
        loc = g.search_q8_phase(1, Qd, qb, K, g.index_base)
        merge_sharded(g, Qd, qb, K, g.index_base, loc)
        skipped = int(torch.isinf(loc[0][:, 0]).sum())
        (rd, ri), rc = certify_sharded(g, Qd, qb, K, loc, g.index_base)
        res["prefix_pruned"] = (pd.cpu().numpy(), pi.cpu().numpy(), pc, rd.cpu().numpy(), ri.cpu().numpy(), rc, skipped)
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
        sd, si = model.search_batch(list(X[-64:]))
        res["model"] = ([p[0] for p in model.predict_batch(list(X[-64:]))], si)
        res["model_d"] = sd
        torch.cuda.synchronize()
        out.put((rank, res))
    finally:
        dist.destroy_process_group()


def _identity_blocks():
    """400 identities x 10 rows, each identity's rows contiguous (so on one shard), 300 queries."""
    r = np.random.default_rng(75)
    protos = r.normal(0, 4, (400, 48))
    G = protos[np.arange(4000) // 10] + r.normal(0, 1, (4000, 48))
    Q = protos[r.integers(0, 400, 300)] + r.normal(0, 1, (300, 48))
    return Q.astype(np.float32).astype(np.float64), G.astype(np.float32).astype(np.float64), np.arange(4000) // 10


def _split_prefix_data():
    """2 x 150 identities x 10 rows, d = 1,280: the first half's identities differ in the leading 64
    features (a Fisherfaces-like profile: alone its shard chooses a one-stage prefix), the second half's
    isotropically (alone: no prefix); together the leading blocks still dominate (prefix 1)."""
    r = np.random.default_rng(76)
    d, nid, per = 1280, 150, 10
    Ca = np.zeros((nid, d))
    Ca[:, :64] = r.normal(0, 60, (nid, 64))
    Cb = r.normal(0, 6, (nid, d))
    C = np.concatenate([Ca, Cb])
    G = C[np.arange(2 * nid * per) // per] + r.normal(0, 3, (2 * nid * per, d))
    Q = C[r.integers(0, 2 * nid, 300)] + r.normal(0, 3, (300, d))
    return Q.astype(np.float32).astype(np.float64), G.astype(np.float32).astype(np.float64), np.arange(2 * nid * per) // per


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
    # the unsharded result differs only where the oracle has near-ties at the differing ranks
    _agree_except_near_ties(metric, Q[:B], G, i0, ir)
    assert [a for a, s in zip(lab0, same) if s] == [b for b, s in zip(ref, same) if s]


def _agree_except_near_ties(metric, Q, G, ia, ib, near_rel=1e-4):
    """Two top-k index lists of the same queries agree except where the oracle distances of the
    differing rows are within near_rel of each other (SURVEY §8c's near-tie rule, as _check_search)."""
    D = O.pairwise(metric, Q, G)
    for b in np.nonzero(~(ia == ib).all(1))[0]:
        for j in np.nonzero(ia[b] != ib[b])[0]:
            a, c = D[b, ia[b, j]], D[b, ib[b, j]]
            assert abs(a - c) <= near_rel * max(abs(c), 1e-300) + 1e-6 * np.linalg.norm(Q[b]), (b, j, a, c)


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
    dref, ref = model.search_batch(list(X[-64:]))
    # against the float64 oracle on the projected features (feature.py:241-242 in fp64), and the
    # unsharded model, both with the near-tie rule
    F = np.stack([np.asarray(ff.project(x.reshape(-1, 1))).reshape(-1) for x in X])
    _agree_except_near_ties("EuclideanDistance", F[-64:], F[:-64], idx0, ref)
    d0 = sharded[0]["model_d"]
    _check_search("EuclideanDistance", F[-64:], F[:-64], d0, idx0, K)


@pytest.mark.timeout(600)
def test_pruned_merge_equals_plain_merge(sharded):
    """parallel.merge_sharded (ofr_knn_f6_merge_pruned): the global top-k and the certificate counts
    equal the plain per-rank merge's; each rank skipped the re-rank of the queries whose neighbours
    live on the other rank."""
    for rank in (0, 1):
        pd, pi, pc, rd, ri, rc, skipped = sharded[rank]["pruned"]
        assert np.array_equal(pi, ri) and np.array_equal(pd, rd)
        assert list(pc) == list(rc)
        assert skipped >= 100, skipped      # of 300 queries, about half belong to the other shard
    Q, G, _ = _identity_blocks()
    _check_search("EuclideanDistance", Q, G, sharded[0]["pruned"][3], sharded[0]["pruned"][4], K)


# ---------------------------------------------------------------------------
# the adaptive start tier on a sharded gallery (VERDICT r4 "do this" #6)
# ---------------------------------------------------------------------------
def _crowded():
    """tests/test_gpu_pipeline.py's clusters (>= 90 % of the fp6 tier's queries uncertified)."""
    r = np.random.default_rng(3)
    d, K_, per, B = 128, 200, 40, 300
    mu = r.normal(0, 1, (K_, d))
    G = (mu[np.arange(K_ * per) % K_] + r.normal(0, 0.5, (K_ * per, d))).astype(np.float32).astype(np.float64)
    Q = (mu[r.integers(0, K_, B)] + r.normal(0, 0.5, (B, d))).astype(np.float32).astype(np.float64)
    return Q, G, np.arange(K_ * per) % K_


def _adaptive_worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from ocvfacerec.facerec.classifier import NearestNeighbor
        from ocvfacerec.facerec.distance import EuclideanDistance
        from opencv_facerecognizer_amd._device import FloatGallery
        Q, G, y = _crowded()
        res = {}
        for mode in ("0", "1"):
            os.environ["OFR_ADAPTIVE_TIER"] = mode
            clf = NearestNeighbor(EuclideanDistance(), k=2)
            clf.compute(list(G), y)
            clf.shard()
            starts, outs = [], []
            for _ in range(FloatGallery.REPROBE + 1):
                d, i = clf.search(Q)
                g = clf._gallery()
                starts.append(g.last_start_tier)
                outs.append((d, i, tuple(g.last_fallbacks)))
            res[mode] = (starts, outs)
        out.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_sharded_adaptive_start_tier_matches_fixed_chain():
    """2 gloo ranks on one device, crowded clusters: with the adaptive start tier both ranks switch to
    the two-slice tier after the first batch and re-probe fp6 every REPROBE-th batch -- identically,
    since the failure counts they learn from are the global certificate's -- and every batch's global
    top-k equals the fixed-start chain's bit for bit (classifier.py:104-119)."""
    import torch.multiprocessing as mp
    from opencv_facerecognizer_amd._device import FloatGallery
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_adaptive_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, r = q.get(timeout=500)
        res[rank] = r
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank in (0, 1):
        fixed_starts, fixed = res[rank]["0"]
        starts, outs = res[rank]["1"]
        assert all(s == "f6" for s in fixed_starts), fixed_starts
        assert fixed[0][2][0] >= 0.9 * 300, fixed[0][2]                # the fp6 tier fails (crowded)
        assert starts[0] == "f6" and starts[1] == "f6x2", starts
        assert starts[FloatGallery.REPROBE - 1] == "f6" and starts.count("f6") == 2, starts
        for (d, i, _), (dw, iw, _) in zip(outs, fixed):
            assert np.array_equal(i, iw) and np.array_equal(d, dw)
    assert res[0]["1"][0] == res[1]["1"][0]                           # both ranks switch identically
    for (d0, i0, c0), (d1, i1, c1) in zip(res[0]["1"][1], res[1]["1"][1]):
        assert np.array_equal(i0, i1) and np.array_equal(d0, d1) and c0 == c1
    oracle_i = np.argsort(O.pairwise("EuclideanDistance", *_crowded()[:2]), axis=1, kind="stable")[:, :2]
    got = res[0]["1"][1][0][1]
    assert (np.sort(got, 1) == np.sort(oracle_i, 1)).mean() > 0.99   # exact top-2 (up to oracle near-ties)


@pytest.mark.timeout(600)
def test_sharded_prefix_tier_shared_choice_and_pruned_merge(sharded):
    """Round 6 (VERDICT r5 do-this #6): shards that alone would pick different prefix
    lengths pick the same one (all-reduced block sums), both start the batch at f6p, the global top-k
    equals the oracle's; the pruned split merge of the prefix tier (exact d^2 of each rank's first k
    candidates as the upper bounds) gives the plain merge's results and certificate counts while the
    rank that does not hold a query's identity skips its re-rank."""
    Q, G, _ = _split_prefix_data()
    r0, r1 = sharded[0]["prefix"], sharded[1]["prefix"]
    assert {r0[3], r1[3]} == {0, 1}, (r0[3], r1[3])                 # the shards' own choices differ
    assert r0[2] == r1[2] == 1, (r0[2], r1[2])                       # the shared choice
    assert r0[4] == r1[4] == "f6p" and r0[5] == r1[5], (r0[4:], r1[4:])
    assert np.array_equal(r0[1], r1[1]) and np.array_equal(r0[0], r1[0])
    _check_search("EuclideanDistance", Q, G, r0[0], r0[1], K)
    for rank in (0, 1):
        pd, pi, pc, rd, ri, rc, skipped = sharded[rank]["prefix_pruned"]
        assert np.array_equal(pi, ri) and np.array_equal(pd, rd)
        assert list(pc) == list(rc)
        assert skipped >= 60, (rank, skipped)                        # ~half the queries live on the other rank
    _check_search("EuclideanDistance", Q, G, sharded[0]["prefix_pruned"][3], sharded[0]["prefix_pruned"][4], K)
