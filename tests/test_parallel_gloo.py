"""Gallery sharding + top-k exchange (opencv_facerecognizer_amd/parallel.py), world_size 2 on gloo (CPU).

The device merge kernel (ofr_topk_merge) is covered by tests/test_gpu_parity.py; here the
exchanged per-rank lists are merged by the oracle's stable ordering and must reproduce the
single-process global top-k exactly (indices and distances).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import facerec_oracle as O
from opencv_facerecognizer_amd.parallel import exchange_topk, gather_rows, gather_rows_async, shard_range, world


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    r = np.random.Generator(np.random.PCG64(7))
    G = r.normal(0, 1, (1001, 24))
    G[500] = G[17]                        # a tie across the shard boundary
    Q = r.normal(0, 1, (33, 24))
    Q[3] = G[17]
    return Q, G


def _worker(rank, ws, port, k, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        Q, G = _data()
        n0, n1 = shard_range(len(G), rank, ws)
        d, i = O.nn_search_vectorized("EuclideanDistance", Q, G[n0:n1], k)
        gd, gi = exchange_topk(torch.from_numpy(d), torch.from_numpy(i + n0))
        assert world() == (rank, ws)
        if rank == 0:
            out.put((gd.numpy(), gi.numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_disjointly():
    for N in (0, 1, 7, 1000, 1000001):
        for ws in (1, 2, 3, 8):
            rs = [shard_range(N, r, ws) for r in range(ws)]
            assert rs[0][0] == 0 and rs[-1][1] == N
            assert all(rs[j][1] == rs[j + 1][0] for j in range(ws - 1))


@pytest.mark.parametrize("k", [1, 4])
def test_two_rank_exchange_reproduces_global_topk(k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    gd, gi = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    Q, G = _data()
    ref_d, ref_i = O.nn_search_vectorized("EuclideanDistance", Q, G, k)
    assert gd.shape == (len(Q), 2 * k)
    for b in range(len(Q)):
        o = np.lexsort((gi[b], gd[b]))[:k]          # merge by (distance, index)
        assert np.array_equal(gi[b][o], ref_i[b]), b
        assert np.array_equal(gd[b][o], ref_d[b]), b


def _gather_worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        x = torch.arange(6 * 5, dtype=torch.float32).reshape(6, 5) + 1000 * rank   # this rank's row block
        g = gather_rows(x)
        pending = gather_rows_async(x)             # the overlapped form (bench.py): same rows
        g2 = pending()
        assert pending.out is g2 and torch.equal(g, g2)
        if rank == 0:
            out.put(g.numpy())
    finally:
        dist.destroy_process_group()


def test_gather_rows_rank_major():
    """Sharded query preparation: every rank's row block, concatenated in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    g = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    base = np.arange(30, dtype=np.float32).reshape(6, 5)
    assert np.array_equal(g, np.concatenate([base, base + 1000]))


def _ragged_worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from opencv_facerecognizer_amd.parallel import allreduce_sum, gather_ragged_rows
        x = (torch.arange((3 + 2 * rank) * 4, dtype=torch.int64).reshape(-1, 4) + 100 * rank).to(torch.uint8)
        g = gather_ragged_rows(x)                  # the gram regime's face gather: 3 + 5 rows
        v = torch.full((2, 3), 0.5 + rank, dtype=torch.float64)
        allreduce_sum([v])
        out.put((rank, g.numpy(), v.numpy()))
    finally:
        dist.destroy_process_group()


def test_gather_ragged_rows_and_allreduce_sum():
    """Sharded training's collectives (parallel.gather_ragged_rows: row blocks of different lengths,
    rank-major; parallel.allreduce_sum: fp64 sums, the same values on every rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ragged_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, g, v = q.get(timeout=120)
        res[r] = (g, v)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = np.concatenate([np.arange(12).reshape(3, 4), np.arange(20).reshape(5, 4) + 100]).astype(np.uint8)
    for r in (0, 1):
        assert np.array_equal(res[r][0], want)
        assert np.array_equal(res[r][1], np.full((2, 3), 2.0))


class _MockShardGallery:
    """CPU stand-in for FloatGallery on one shard: every tier returns the exact local top-k (global
    indices) and, as its certificate bound, the squared distance of the 16th local candidate shrunk
    by a tier-dependent slack -- a valid lower bound for every row outside the candidates, loose
    at the first tier so that the collective fallback chain runs."""
    TIER_CHAIN = ("f6", 1, 2, "fp32")
    SLACK = {"f6": 0.5, 1: 0.97, 2: 0.999}

    def __init__(self, G, n0, overflow=()):
        self.G, self.n0 = G, n0
        self.overflow = np.asarray(overflow, dtype=np.int64)   # first-tier queries whose sieve bucket overflows
        self.noted = []                                        # the adaptive start tier's statistics

    def note_failures(self, tier, B, failed):
        self.noted.append((str(tier), int(B), int(failed)))

    def next_tier(self, tier, nrows):
        return self.TIER_CHAIN[self.TIER_CHAIN.index(tier) + 1]

    def _local(self, Q, k):
        d, i = O.nn_search_vectorized("EuclideanDistance", Q, self.G, min(16, len(self.G)))
        return d, i + self.n0

    def quantize_queries(self, sub, tier):
        return {"tier": tier, "Q": sub.numpy(), "B": len(sub)}

    def search_q8_phase(self, phases, sub, q2, k, index_base):
        d, i = self._local(q2["Q"], k)
        b = d[:, -1] ** 2 * self.SLACK[q2["tier"]] if d.shape[1] == 16 else np.full(len(d), np.inf)
        d, i = d[:, :k].copy(), i[:, :k].copy()
        if q2["tier"] == "f6" and len(self.overflow):
            # merge_kernel on an overflowed bucket: no candidates (inf, -1) and bound -inf
            d[self.overflow], i[self.overflow], b[self.overflow] = np.inf, -1, -np.inf
        q2["bound"] = torch.from_numpy(b)
        return torch.from_numpy(d), torch.from_numpy(i)

    def _search_f32(self, sub, k, index_base):
        d, i = self._local(sub.numpy(), k)
        return torch.from_numpy(d[:, :k].copy()), torch.from_numpy(i[:, :k].copy())


def _cert_worker(rank, ws, port, k, out, overflow=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import opencv_facerecognizer_amd.parallel as par
        _patch_host_kernels(par)                          # the device kernels need a GPU
        Q, G = _data()
        n0, n1 = shard_range(len(G), rank, ws)
        # rank 1 overflows on the queries that are copies of its own rows (their true neighbours)
        g = _MockShardGallery(G[n0:n1], n0, overflow=_OVERFLOW_Q if (overflow and rank == 1) else ())
        if overflow:
            Q = _overflow_queries(Q, G)
        Qt = torch.from_numpy(Q)
        qq = g.quantize_queries(Qt, "f6")
        d, i = g.search_q8_phase(3, Qt, qq, k, n0)
        (md, mi), counts = par.certify_sharded(g, Qt, qq, k, (d, i), n0)
        out.put((rank, md.numpy(), mi.numpy(), counts, g.noted))
    finally:
        dist.destroy_process_group()


_OVERFLOW_Q = np.arange(4, 12)


def _overflow_queries(Q, G):
    Q = Q.copy()
    Q[_OVERFLOW_Q] = G[700:708]          # rows of rank 1's shard [500, 1001)
    return Q


# host restatements of the device kernels the sharded path calls (csrc/ofr_comm.hip: pack_kernel,
# merge_certify_kernel, kth_bound_kernel, open_rows_kernel), for workers without a GPU
def _host_pack(d, i, bound=None):
    B, k = d.shape
    out = np.empty((B, 2 * k + 1))
    out[:, :k] = d.numpy()
    out[:, k:2 * k] = i.numpy().astype(np.int64).view(np.float64)
    out[:, 2 * k] = np.inf if bound is None else bound.numpy()
    return torch.from_numpy(out)


def _host_merge_certify(lists, P, B, k, certify=True):
    g = lists.numpy().reshape(P, B, 2 * k + 1)
    gd = g[:, :, :k].transpose(1, 0, 2).reshape(B, P * k)
    gi = np.ascontiguousarray(g[:, :, k:2 * k]).view(np.int64).transpose(1, 0, 2).reshape(B, P * k)
    md, mi = _host_merge(torch.from_numpy(gd.copy()), torch.from_numpy(gi.copy()), P, k, k)
    if not certify:
        return md, mi, None
    bnd = g[:, :, 2 * k]
    minb = np.where(np.isnan(bnd).any(0), -np.inf, bnd.min(0))
    kth = md.numpy()[:, k - 1]
    cert = ((kth * kth < minb) | np.isposinf(minb)).astype(np.int32)
    return md, mi, torch.from_numpy(cert)


def _host_kth_bound(allb, P, B, k):
    a = allb.numpy().reshape(P, B, k).transpose(1, 0, 2).reshape(B, P * k)
    return torch.from_numpy(np.sort(a, axis=1)[:, k - 1].copy())


def _host_open_rows(cert):
    return torch.from_numpy(np.nonzero(cert.numpy() == 0)[0].astype(np.int64))


def _patch_host_kernels(par):
    par.merge_topk = _host_merge
    par.topk_pack = _host_pack
    par.topk_merge_certify = _host_merge_certify
    par.kth_bound = _host_kth_bound
    par.open_rows = _host_open_rows


def _host_merge(gd, gi, nlists, kin, k):
    d, i = gd.numpy(), gi.numpy()
    od, oi = np.empty((len(d), k)), np.empty((len(d), k), np.int64)
    for b in range(len(d)):
        o = np.lexsort((i[b], d[b]))[:k]
        od[b], oi[b] = d[b][o], i[b][o]
    return torch.from_numpy(od), torch.from_numpy(oi)


@pytest.mark.parametrize("k", [1, 3])
def test_sharded_global_certificate_and_collective_fallback(k):
    """parallel.certify_sharded on 2 ranks: the merged result is the exact global top-k whatever tier
    certifies each query, and both ranks run the same collectives down the chain (no deadlock)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cert_worker, args=(r, 2, port, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, 2)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    md, mi, counts, noted = res[0]
    Q, G = _data()
    ref_d, ref_i = O.nn_search_vectorized("EuclideanDistance", Q, G, k)
    assert np.array_equal(mi, ref_i) and np.allclose(md, ref_d, rtol=0, atol=0)
    assert counts[0] > 0 and len(counts) >= 2            # the loose first-tier bound forced fallbacks
    # the adaptive start tier's statistics: the global counts, the same on both ranks (round 5)
    assert noted == res[1][3] and noted[0] == ("f6", len(Q), counts[0])
    assert [n[2] for n in noted] == counts


def _collect(q, n):
    res = {}
    for _ in range(n):
        item = q.get(timeout=120)
        res[item[0]] = item[1:]
    return res


@pytest.mark.parametrize("k", [1, 3])
def test_sharded_overflowed_rank_is_never_certified(k):
    """A rank whose fp6 sieve bucket overflows returns no candidates and bound -inf for that query.
    The global certificate must send the query down the chain (the bound proves nothing), so the
    merged result still holds the overflowed rank's rows -- the exact global top-k."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cert_worker, args=(r, 2, port, k, q, True)) for r in range(2)]
    for p in procs:
        p.start()
    md, mi, counts, _ = _collect(q, 2)[0]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    Q, G = _data()
    Q = _overflow_queries(Q, G)
    ref_d, ref_i = O.nn_search_vectorized("EuclideanDistance", Q, G, k)
    assert np.array_equal(mi, ref_i) and np.allclose(md, ref_d, rtol=0, atol=0)
    assert np.array_equal(mi[_OVERFLOW_Q, 0], np.arange(700, 708))
    assert counts[0] >= len(_OVERFLOW_Q)


def test_global_certificate_bounds():
    from opencv_facerecognizer_amd.parallel import global_certificate
    kth = torch.tensor([1.0, 1.0, float("inf"), 1.0, 3.0])
    minb = torch.tensor([2.0, -float("inf"), float("inf"), float("inf"), 4.0])
    assert global_certificate(kth, minb).tolist() == [True, False, True, True, False]


def _train_pieces_worker(rank, ws, port, out):
    """Each rank: the exact pixel-space pieces of its shard (X'^T X', class sums, counts as integer-
    valued fp64, the layout training.pixel_pieces produces on the device), then allreduce_exact."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from opencv_facerecognizer_amd.parallel import allreduce_exact
        X, y, c = _train_data()
        n0, n1 = shard_range(len(y), rank, ws)
        Xs = X[n0:n1].astype(np.int64) - 128
        G = torch.from_numpy((Xs.T @ Xs).astype(np.float64))
        S = torch.from_numpy(np.stack([Xs[y[n0:n1] == i].sum(0) for i in range(c)]).astype(np.float64))
        cnt = torch.from_numpy(np.bincount(y[n0:n1], minlength=c).astype(np.float64))
        allreduce_exact([G, S, cnt])
        if rank == 0:
            out.put((G.numpy(), S.numpy(), cnt.numpy()))
    finally:
        dist.destroy_process_group()


def _train_data():
    r = np.random.default_rng(77)
    c, n, D = 7, 301, 36
    y = np.arange(n) % c
    protos = r.integers(40, 216, (c, D))
    X = np.clip(protos[y] + r.integers(-30, 31, (n, D)), 0, 255).astype(np.uint8)
    return X, y, c


def test_sharded_training_pieces_allreduce_exactly():
    """SURVEY §8e's training exchange: per-rank X'^T X' and class sums, one all-reduce; the sums are
    integer-valued, so they equal the single-process pieces BIT FOR BIT, and the pixel-space
    Sw / Sb formed from them (training.pixel_scatter's formula) equal the reference's scatter
    (feature.py:160-168, the oracle) over pixels."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_pieces_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    G, S, cnt = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    X, y, c = _train_data()
    Xs = X.astype(np.int64) - 128
    assert np.array_equal(G, (Xs.T @ Xs).astype(np.float64))
    assert np.array_equal(S, np.stack([Xs[y == i].sum(0) for i in range(c)]).astype(np.float64))
    n = len(y)
    s = S.sum(0)
    T = (S / cnt[:, None]).T @ S
    Sw, Sb = G - T, T - np.outer(s, s) / n
    _, oSw, oSb = O.lda_scatter(X.T.astype(np.float64), y)
    assert np.allclose(Sw, oSw, rtol=0, atol=1e-9 * np.abs(oSw).max())
    assert np.allclose(Sb, oSb, rtol=0, atol=1e-9 * np.abs(oSb).max())


class _PrunedMock:
    """Stands in for FloatGallery.merge_pruned: stage 1 reports rank-specific upper bounds, stage 2
    records the global bound it was given."""

    def __init__(self, rank):
        self.rank = rank
        self.seen = None

    def merge_pruned(self, stage, Qd, qq, k, ub, index_base=0, out=None, workspace=None):
        if stage == 1:
            B = ub.shape[0]
            base = torch.arange(B, dtype=torch.float64)[:, None] * 10.0
            ub.copy_(base + torch.arange(k, dtype=torch.float64)[None, :] + (0.5 if self.rank else 0.0))
            if self.rank == 1:
                ub[0] = float("inf")          # a shard with no candidates for query 0
        else:
            self.seen = ub.clone()
        return out


def _pruned_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import opencv_facerecognizer_amd.parallel as par
        from opencv_facerecognizer_amd.parallel import merge_sharded
        _patch_host_kernels(par)
        g = _PrunedMock(rank)
        B, k = 4, 3
        merge_sharded(g, torch.zeros((B, 8)), {"tier": "f6"}, k, 0, None)
        q.put((rank, g.seen.numpy()))
    finally:
        dist.destroy_process_group()


def test_merge_sharded_global_bound():
    """The bound handed to stage 2 is, per query, the k-th smallest of every rank's k upper bounds."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pruned_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    B, k = 4, 3
    for b in range(B):
        vals = sorted([10.0 * b + j for j in range(k)] + ([] if b == 0 else [10.0 * b + j + 0.5 for j in range(k)])
                      + ([float("inf")] * k if b == 0 else []))
        for r in (0, 1):
            assert res[r][b] == vals[k - 1]


def _gather_queries_worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from opencv_facerecognizer_amd._device import FloatGallery
        g = FloatGallery.__new__(FloatGallery)
        r = np.random.Generator(np.random.PCG64(11 + rank))
        qq = dict(tier="f6", B=256, Qs=torch.full((64,), rank, dtype=torch.uint8),
                  scale=torch.from_numpy(r.random(256).astype(np.float32)),
                  stats=torch.from_numpy(r.random((256, 3))))
        o = g.gather_queries(qq)
        if rank == 0:
            out.put((o["Qs"].numpy(), o["scale"].numpy(), o["stats"].numpy(), o["B"], str(o["scale"].dtype)))
    finally:
        dist.destroy_process_group()


def test_gather_queries_packs_scales_and_stats():
    """Sharded query preparation (FloatGallery.gather_queries): the fp6 tiles, the fp32 scales and the
    fp64 stats of every rank's 256-row block, rank-major, scales exact through their fp64 packing."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_queries_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    Qs, scale, stats, B, dt = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert B == 512 and dt == "torch.float32"
    assert np.array_equal(Qs, np.concatenate([np.zeros(64, np.uint8), np.ones(64, np.uint8)]))
    for rank in range(2):
        r = np.random.Generator(np.random.PCG64(11 + rank))
        s, st = r.random(256).astype(np.float32), r.random((256, 3))
        assert np.array_equal(scale[256 * rank:256 * (rank + 1)], s)
        assert np.array_equal(stats[256 * rank:256 * (rank + 1)], st)


def _subgroup_worker(rank, ws, port, out):
    """Ranks 0 and 2 of a 3-rank job form a sub-group; every collective of parallel.py runs on it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from opencv_facerecognizer_amd.parallel import sharded_search
        grp = dist.new_group([0, 2])          # every rank takes part in the creation
        if rank in (0, 2):
            gr, gws = world(grp)
            assert gws == 2 and gr == (0 if rank == 0 else 1)
            x = torch.arange(12, dtype=torch.float32).reshape(4, 3) + 100 * gr
            g = gather_rows(x, grp)
            g2 = gather_rows_async(x, grp)()
            Q, G = _data()
            n0, n1 = shard_range(len(G), gr, gws)

            def local(k):
                d, i = O.nn_search_vectorized("EuclideanDistance", Q, G[n0:n1], k)
                return torch.from_numpy(d), torch.from_numpy(i + n0)

            import opencv_facerecognizer_amd.parallel as par
            par.merge_topk = _host_merge
            md, mi = sharded_search(local, 2, grp)
            if gr == 0:
                out.put((g.numpy(), g2.numpy(), md.numpy(), mi.numpy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_collectives_on_a_sub_group():
    """gather_rows / gather_rows_async / sharded_search take the sub-group's size, not the world's
    (NearestNeighbor.shard(group) records a sub-group's rank and size): 2 of 3 ranks, exact results."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    g, g2, md, mi = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    base = np.arange(12, dtype=np.float32).reshape(4, 3)
    assert np.array_equal(g, np.concatenate([base, base + 100])) and np.array_equal(g2, g)
    Q, G = _data()
    ref_d, ref_i = O.nn_search_vectorized("EuclideanDistance", Q, G, 2)
    assert np.array_equal(mi, ref_i) and np.array_equal(md, ref_d)
