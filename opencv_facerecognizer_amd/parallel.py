"""Gallery sharding across the GPUs of one node (one process per GPU).

The reference has no parallelism.  Search shards naturally by
gallery rows: rank r of G holds rows [r*N/G, (r+1)*N/G) of the
gallery, W and the query batch are replicated, every rank computes its local
top-k (exact fp64 distances, global row indices via ``index_base``), and the
only data-path exchange is ONE all-gather of the B x k (distance, index)
lists (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X, "gloo"
on CPU for tests), followed by the ``ofr_topk_merge`` kernel.

Query preparation can be sharded too (``gather_rows``): each rank projects and
quantizes B/G of the faces and the rows are all-gathered, so at G GPUs the
projection costs 1/G instead of being replicated.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_range(N, rank, world_size):
    """Contiguous, disjoint, covering row ranges."""
    return (N * rank) // world_size, (N * (rank + 1)) // world_size


def gather_rows(x, group=None):
    """All-gather equal-size row blocks (dim 0) of every rank of `group`, rank-major: [G * rows, ...]."""
    _, ws = world(group)
    if ws == 1:
        return x
    x = x.contiguous()
    if dist.get_backend(group) == "nccl":
        out = torch.empty((ws * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out
    parts = [torch.empty_like(x) for _ in range(ws)]
    dist.all_gather(parts, x, group=group)
    return torch.cat(parts, 0)


class PendingRows:
    """An all-gather of gather_rows in flight: .out is the destination (valid to hand to kernels
    that do not read it yet, e.g. the quantized search's tile pass), calling it waits (a stream
    dependency on the collective's stream for RCCL, not a host wait) and returns the rows."""

    def __init__(self, out, work=None, parts=None):
        self.out, self._work, self._parts = out, work, parts

    def __call__(self):
        if self._work is not None:
            self._work.wait()
            self._work = None
            if self._parts is not None:
                self.out.copy_(torch.cat(self._parts, 0))
                self._parts = None
        return self.out


def gather_rows_async(x, group=None):
    """Start gather_rows(x) and return a PendingRows (the query rows' all-gather overlaps the
    quantized tile pass, which reads only the gathered fp6 / int8 query tiles)."""
    _, ws = world(group)
    if ws == 1:
        return PendingRows(x)
    x = x.contiguous()
    out = torch.empty((ws * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if dist.get_backend(group) == "nccl":
        return PendingRows(out, dist.all_gather_into_tensor(out, x, group=group, async_op=True))
    parts = [torch.empty_like(x) for _ in range(ws)]
    return PendingRows(out, dist.all_gather(parts, x, group=group, async_op=True), parts)


def exchange_topk(d, i, group=None):
    """All-gather per-rank (B x k) lists -> (B x world*k) tensors, rank-major (list p = rank p)."""
    gd, gi, _ = exchange_lists(d, i, None, group)
    return gd, gi


def topk_pack(d, i, bound=None):
    """This rank's (B x k) lists + bound -> one [B][2k+1] fp64 block (device kernel)."""
    from ._device import topk_pack as _pack
    return _pack(d, i, bound)


def topk_merge_certify(lists, P, B, k, certify=True):
    """Gathered [P][B][2k+1] blocks -> merged (d, i) and the global certificate (device kernel)."""
    from ._device import topk_merge_certify as _mc
    return _mc(lists, P, B, k, certify)


def kth_bound(allb, P, B, k):
    """[P][B][k] ascending per-rank upper bounds -> [B] k-th smallest over the ranks (device kernel)."""
    from ._device import kth_bound as _kb
    return _kb(allb, P, B, k)


def open_rows(cert):
    """int32 certificate -> int64 indices of the uncertified queries (device compaction, one count read)."""
    from ._device import open_rows as _or
    return _or(cert)


def merge_topk(gd, gi, nlists, kin, k):
    """Device merge of the gathered lists (ofr_topk_merge)."""
    if nlists == 1 and kin == k:
        return gd, gi
    from ._device import topk_merge
    return topk_merge(gd, gi, nlists, kin, k)


def sharded_search(local_search, k, group=None):
    """local_search(k) -> (d, i) on this rank's shard with global indices; returns the global top-k."""
    d, i = local_search(k)
    _, ws = world(group)
    gd, gi = exchange_topk(d, i, group)
    return merge_topk(gd, gi, ws, k, k)


def exchange_lists(d, i, bound=None, group=None):
    """ONE all-gather of every rank's (B x k) lists and per-query bound -> (gd, gi, min bound).

    The fp64 distances, the int64 indices (bit-copied as fp64 words: a collective only moves
    bytes) and the bound travel as one [B][2k+1] fp64 block per rank, so a tier of the sharded
    search costs one collective instead of three.  gd/gi are [B][world*k], rank-major."""
    _, ws = world(group)
    B, k = d.shape
    if ws == 1:
        return d, i, bound
    cols = [d.to(torch.float64), i.to(torch.int64).contiguous().view(torch.float64)]
    if bound is not None:
        cols.append(bound.to(torch.float64).reshape(B, 1))
    g = gather_rows(torch.cat(cols, 1).contiguous(), group).reshape(ws, B, -1)
    gd = g[:, :, :k].permute(1, 0, 2).reshape(B, ws * k).contiguous()
    gi = g[:, :, k:2 * k].contiguous().view(torch.int64).permute(1, 0, 2).reshape(B, ws * k).contiguous()
    minb = g[:, :, 2 * k].min(0).values if bound is not None else None
    return gd, gi, minb


def merge_sharded(gallery, Qd, qq, k, index_base, out, group=None, workspace=None):
    """Phase 2 of the certified search on a sharded gallery, after phase 1 (the tile pass) on every
    rank.  fp6 tier: the split merge -- every rank selects its candidates and bounds the squared
    distance of its best k from above (ofr_knn_f6_merge_pruned stage 1), ONE all-gather of those
    B x k bounds gives per query the k-th smallest over the ranks, an upper bound of the GLOBAL k-th
    squared distance, and each rank re-ranks only the candidates that can still fall below it
    (stage 2): a rank that holds none of a query's neighbours skips its exact re-rank (the rows it
    skips are farther than k rows of another rank, so the global top-k and the certificate of
    certify_sharded are unchanged).  The prefix tier f6p (round 6) too: its keys bound no distance from
    above, so stage 1 takes the exact squared distances of each rank's first k candidates instead.  Other
    tiers: the local merge.  workspace: the one phase 1 ran on (the gallery's by default).  Returns out."""
    _, ws = world(group)
    if ws == 1 or qq["tier"] not in ("f6", "f6p"):
        return gallery.search_q8_phase(2, Qd, qq, k, index_base=index_base, out=out, workspace=workspace)
    B = Qd.shape[0]
    ub_local = torch.empty((B, k), dtype=torch.float64, device=Qd.device)
    gallery.merge_pruned(1, Qd, qq, k, ub_local, index_base, workspace=workspace)
    ub = kth_bound(gather_rows(ub_local, group), ws, B, k)     # [ws][B][k] rank-major -> [B]
    return gallery.merge_pruned(2, Qd, qq, k, ub, index_base, out, workspace=workspace)


def global_certificate(kth, minb):
    """Query certified iff its GLOBAL k-th squared distance is below every rank's bound.

    A rank whose sieve bucket overflowed reports bound = -inf (no bound: its candidates were
    dropped) and never certifies; +inf (every local row was a candidate) always does, even when
    the gallery holds fewer than k rows (kth = inf)."""
    return (kth * kth < minb) | torch.isposinf(minb)


def certify_sharded(gallery, Qd, qq, k, out, index_base, group=None):
    """Global certificate + collective fallback of the certified tiers on a sharded gallery.

    ``out`` is this rank's local top-k (exact fp64 distances, global row indices) of the whole
    batch from the tier of ``qq``; the merge kernel left in ``qq["bound"]`` a lower bound of the
    squared distance of every local row outside its candidates (-inf when the rank could not
    bound them).  After the all-gather + merge, query q is certified iff its GLOBAL k-th squared
    distance is below every rank's bound: a row that is not among its rank's candidates is then
    farther than the global k-th, and one that is a candidate but not in its rank's top-k has k
    better rows on that rank, so the merged list is the exact global top-k.  (A per-rank
    certificate would fail for every query whose identity lives on another rank: its local
    neighbours are not separated from its 16th candidate.)  Uncertified queries -- the same set on
    every rank, it is computed from gathered data -- go down the tier chain on every rank, each
    stage with its own exchange; the fp32 stage is exact.  Reference semantics:
    classifier.py:104-119 (the k nearest of the whole gallery).
    Returns ((d, i) global top-k, [uncertified after each quantized tier]).
    """
    _, ws = world(group)

    def merged(d, i, bound):
        # one [B][2k+1] block per rank (ofr_topk_pack), ONE all-gather, then the merge and the global
        # certificate in one kernel (ofr_topk_merge_certify; bound None: +inf, the certificate unused)
        B = d.shape[0]
        lists = gather_rows(topk_pack(d.to(torch.float64), i.to(torch.int64), bound), group)
        return topk_merge_certify(lists, ws, B, k, certify=bound is not None)

    md, mi, cert = merged(out[0], out[1], qq["bound"])
    rows = open_rows(cert)
    counts = [int(rows.numel())]
    tier = qq["tier"]
    # the adaptive start tier's statistics (FloatGallery.start_tier): the counts are global -- the same on
    # every rank -- so every rank's gallery takes the same start-tier decisions and the collectives match
    gallery.note_failures(tier, int(qq["B"]), counts[0])
    while rows.numel():
        tier = gallery.next_tier(tier, int(rows.numel()))
        sub = Qd.index_select(0, rows).contiguous()
        if tier == "fp32":
            d2, i2 = gallery._search_f32(sub, k, index_base)
            md2, mi2, _ = merged(d2, i2, None)
        else:
            q2 = gallery.quantize_queries(sub, tier=tier)
            d2, i2 = gallery.search_q8_phase(3, sub, q2, k, index_base)
            md2, mi2, c2 = merged(d2, i2, q2["bound"])
        md.index_copy_(0, rows, md2)
        mi.index_copy_(0, rows, mi2)
        if tier == "fp32":
            break
        still = open_rows(c2)
        counts.append(int(still.numel()))
        gallery.note_failures(tier, int(rows.numel()), counts[-1])
        rows = rows.index_select(0, still)
    return (md, mi), counts


# ---------------------------------------------------------------------------
# training: the one exchange step of SURVEY §8e
# ---------------------------------------------------------------------------
def allreduce_exact(tensors, group=None):
    """Sum integer-valued fp64 tensors (partial Grams / class sums) over the ranks.  Every partial
    value and every sum is an integer below 2^53, so the floating-point additions are exact and the
    result does not depend on the reduction order or the number of ranks."""
    _, ws = world(group)
    if ws == 1:
        return tensors
    for t in tensors:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return tensors


def allreduce_sum(tensors, group=None):
    """Sum fp64 tensors over the ranks in place (not integer-valued: the result depends on the
    reduction order at the last bit, but every rank receives the same values)."""
    _, ws = world(group)
    if ws > 1:
        for t in tensors:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return tensors


def share_block_scales(gallery, group=None):
    """Column-block scales of a sharded gallery's fp6 tiers from the block sums of squares of ALL its
    rows (one all-reduce of ceil(d / 32) fp64 values): every rank then quantizes its shard and its
    share of a query batch alike, as the all-gathered fp6 query panels require (bench.py's sharded
    preparation).  Before the fp6 tiers are built."""
    sums = gallery.block_sums()
    allreduce_sum([sums], group)
    return gallery.set_block_scales(sums)


def gather_ragged_rows(x, group=None):
    """All-gather row blocks of different lengths (dim 0), rank-major: pads every block to the longest
    one for the collective and trims it again."""
    _, ws = world(group)
    if ws == 1:
        return x
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    ns = gather_rows(n, group).cpu().numpy()
    mx = int(ns.max())
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[:x.shape[0]].copy_(x)
    allr = gather_rows(pad, group)
    return torch.cat([allr[r * mx:r * mx + int(ns[r])] for r in range(ws)], 0)


def train_fisherfaces_sharded(feature, X_local, y_local, num_classes, group=None):
    """Fisherfaces.compute (feature.py:211-235) with the training faces sharded over the ranks.

    Each rank holds its own faces (uint8) and their labels (global 0..c-1); the regime is chosen from
    the global n, c, D exactly as Fisherfaces.compute chooses it:
    * pixel (PCA keeps every dimension: n - c >= D and n >= D, e.g. BASELINE configs[4]): the
      statistics are sums over faces -- rank r forms its exact pieces (X'^T X', class sums, column
      sums; int8 MFMA) and ONE all-reduce (RCCL over xGMI; gloo in tests) combines them exactly;
      rank 0 solves the pencil.  W equals the single-process model's bit for bit.
    * cov (n > D, PCA(n - c) < D): X'^T X' and the column sums all-reduce exactly into the
      covariance (the same bits on every rank), rank 0 takes its leading eigenvectors P and
      broadcasts them, each rank projects its own faces, and the LDA scatter of the features is
      all-reduced (training.feature_scatter_sharded: global class means, then per-rank centred
      products); rank 0 solves LDA, W = P L.  Equal to the single-process model up to the order of
      the fp64 feature sums.
    * gram (n <= D: at most D faces of D pixels, <= D^2 bytes): the faces and labels are all-gathered
      and rank 0 runs the single-process n x n Gram pipeline (training.fisher_gram); the same W.
    W and the eigenvalues are broadcast, and each rank projects its own faces: the features come back
    as this rank's gallery shard.  Returns this rank's features (list of (d,1) matrices, the
    reference's return type)."""
    from . import _device, training
    from .facerec.feature import lda_eigen
    rank, ws = world(group)
    Xd, D, kind = _device_rows_u8(X_local)
    lay = training.Layout(y_local, Xd.device, c=num_classes)
    counts = torch.from_numpy(lay.counts.astype(np.float64)).to(Xd.device)
    allreduce_exact([counts], group)
    cnt = counts.cpu().numpy()
    n, c = int(cnt.sum()), int(num_classes)
    k = n - c                                              # PCA(n - c), as Fisherfaces.compute
    if k <= 0 or k > n - 1:
        k = n - 1
    k = min(k, D, n)
    m = feature._num_components
    if m <= 0 or m > c - 1:
        m = c - 1
    W = torch.empty((D, m), dtype=torch.float64, device=Xd.device)
    ev = torch.empty(m, dtype=torch.float64, device=Xd.device)

    def solve(Sw, Sb, P=None):            # rank 0: LDA (host, as the reference), W = P L (cov)
        evals, V = lda_eigen(Sw, Sb, m)
        if P is None:
            W.copy_(torch.from_numpy(np.ascontiguousarray(V, dtype=np.float64)))
        else:
            L32 = np.asarray(V, dtype=np.float32).astype(np.float64)       # feature.py:176
            W.copy_(_device.gemm_f64(P, _device.f64_dev(L32, device=P.device)))
        ev.copy_(torch.from_numpy(np.asarray(evals, dtype=np.float64)))

    if k >= D:
        regime = "pixel"
        pieces = training.pixel_pieces(Xd, D, lay)
        allreduce_exact([pieces["G"], pieces["S"], pieces["s"]], group)
        Sw, Sb = training.finite("pixel_scatter", *training.pixel_scatter(pieces, cnt, n))
        del pieces
        if rank == 0:
            solve(Sw, Sb)
        del Sw, Sb
    elif n <= D:
        regime = "gram"
        Xall = gather_ragged_rows(Xd, group)
        yall = gather_ragged_rows(torch.from_numpy(np.asarray(y_local, np.int64).reshape(-1)).to(Xd.device),
                                  group).cpu().numpy()
        if rank == 0:
            evals, Wd = training.fisher_gram(Xall, D, training.Layout(yall, Xd.device, c=c), yall, k, m)
            W.copy_(Wd)
            ev.copy_(torch.from_numpy(np.asarray(evals, dtype=np.float64)))
        del Xall
    else:
        regime = "cov"
        pieces = training.pixel_pieces(Xd, D, lay)
        del pieces["S"]
        colsum = training.column_sums(Xd, D, lay, shift=0)[0].reshape(1, D).contiguous()   # exact sums of x
        allreduce_exact([pieces["G"], pieces["s"], colsum], group)
        mu = torch.empty_like(colsum)
        nd = torch.tensor([float(n)], dtype=torch.float64, device=Xd.device)
        _lib_call("ofr_row_div_f64", colsum, 1, D, D, nd, mu, D)                # mean image, rounded once
        C = training.finite("covariance", training.covariance(pieces, n))
        del pieces
        P = torch.empty((D, k), dtype=torch.float64, device=Xd.device)
        if rank == 0:
            _, Pd = training.finite("eigh_desc", *training.eigh_desc(C, k))
            P.copy_(Pd)
            del Pd
        del C
        if ws > 1:
            dist.broadcast(P, 0, group=group)
        shift = _device.gemm_f64(mu, P).reshape(-1)
        Fd = _device.Projection(Wt_device=P.t().contiguous(), D=D).project(Xd, shift64=shift, f64=True)
        Sw, Sb = training.finite("feature_scatter", *training.feature_scatter_sharded(
            Fd, lay, counts, n, lambda ts: allreduce_sum(ts, group)))
        del Fd
        if rank == 0:
            solve(Sw, Sb, P)
        del Sw, Sb, P
    if ws > 1:
        dist.broadcast(W, 0, group=group)
        dist.broadcast(ev, 0, group=group)
    feature._regime = regime
    feature._eigenvalues = ev.cpu().numpy().astype(np.float32)
    feature._num_components = m
    feature._eigenvectors = np.asmatrix(W.cpu().numpy())
    feature.__dict__.pop("_dev_proj", None)
    Fd = feature.project_device(Xd, f64=True)
    return [np.asmatrix(r.reshape(-1, 1)) for r in Fd.cpu().numpy()]


def _lib_call(name, *args):
    from . import _lib
    _lib.call(name, _lib.stream(), *[_lib.ptr(a) if isinstance(a, torch.Tensor) else a for a in args])


def _device_rows_u8(X):
    from .facerec.feature import _device_rows
    Xd, D, kind = _device_rows(X)
    if kind != "u8":
        raise TypeError("sharded training takes uint8 faces")
    return Xd, D, kind


# ---------------------------------------------------------------------------
# single-process multi-GPU search through the C ABI (ofr_comm_init_all / ofr_knn_sharded)
# ---------------------------------------------------------------------------
class DeviceComm:
    """RCCL communicator over the given devices of this process (ofr_comm_init_all), for C / C++
    style callers that drive every GPU from one process; the package's own multi-GPU path is one
    process per GPU over torch.distributed (functions above)."""

    def __init__(self, devices):
        import ctypes
        from . import _lib
        self.devices = list(devices)
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _lib.call("ofr_comm_init_all", len(self.devices), ctypes.cast(arr, ctypes.c_void_p), ctypes.byref(h))
        self.handle = h

    def close(self):
        if self.handle:
            from . import _lib
            _lib.call("ofr_comm_destroy", self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def knn(self, galleries, queries, k, tiers=("f6x2", 2), prefix=True):
        """galleries[r]: the FloatGallery of shard r (on devices[r], global row offset in
        .index_base, default 0 for one shard); queries[r]: the centred fp32 query rows [B][ld] on
        devices[r] (the same batch on every device).  tiers: the finer stages the open queries may
        take before the exact pass ("f6x2" and / or 2 = int8 x2; built on the galleries if missing).
        prefix: run the prefix tier f6p first when the galleries have one (prefix_stages(); a sharded
        caller makes it the same on every shard: parallel.share_block_scales).
        Returns per device (out_d, out_i, cert); self.last_tier_counts = open queries after fp6,
        after f6x2, after int8 x2, and the number the exact pass ran (-1: stage not run);
        self.last_prefix_open = open queries after the prefix tier (-1: not run)."""
        import ctypes
        from . import _lib
        lib = _lib.load()
        B, d = int(queries[0].shape[0]), galleries[0].d
        shards = (_lib.KnnShard * len(galleries))()
        counts = np.full(4, -1, dtype=np.int64)
        popen = np.full(1, -1, dtype=np.int64)
        keep = [counts, popen]
        for r, (g, Qd) in enumerate(zip(galleries, queries)):
            with torch.cuda.device(Qd.device):
                qq = g.quantize_queries(Qd, tier="f6")
                t = g._tier_gallery("f6")
                nbytes = lib.ofr_knn_sharded_workspace_bytes(B, g.N, Qd.shape[1], k, len(galleries))
                ws = torch.empty(nbytes, dtype=torch.uint8, device=Qd.device)
                out_d = torch.empty((B, k), dtype=torch.float64, device=Qd.device)
                out_i = torch.empty((B, k), dtype=torch.int64, device=Qd.device)
                cert = torch.empty(B, dtype=torch.int32, device=Qd.device)
                s = shards[r]
                s.stream = torch.cuda.current_stream(Qd.device).cuda_stream
                s.Q, s.ldq, s.Qt = Qd.data_ptr(), Qd.shape[1], qq["Qs"].data_ptr()
                s.qscale, s.qstats = qq["scale"].data_ptr(), qq["stats"].data_ptr()
                s.G, s.N, s.ldg, s.Gt = g.G.data_ptr(), g.N, g.ld, t["Gs"].data_ptr()
                s.gscale, s.aux, s.gmax = t["scale"].data_ptr(), g.aux.data_ptr(), t["gmax"].data_ptr()
                s.index_base = int(getattr(g, "index_base", 0))
                s.bscale = g.bscale.data_ptr() if g.bscale is not None else None   # the shard's (and qq's)
                s.workspace, s.workspace_bytes = ws.data_ptr(), nbytes
                s.out_d, s.out_i, s.cert = out_d.data_ptr(), out_i.data_ptr(), cert.data_ptr()
                if g.row_sample():                        # the sieve thresholds from the shard's row sample
                    s.St, s.Ns = t["St"].data_ptr(), -(-g.N // lib.ofr_f6_sample_step())
                    s.sscale, s.saux = t["sscale"].data_ptr(), t["saux"].data_ptr()
                if "f6x2" in tiers:
                    t2 = g._tier_gallery("f6x2")
                    s.Gt2, s.gscale2, s.gmax2 = t2["Gs2"].data_ptr(), t2["scale"].data_ptr(), t2["gmax"].data_ptr()
                    if g.row_sample():
                        s.St2 = t2["St2"].data_ptr()
                if 2 in tiers:
                    t8 = g._tier_gallery(2)
                    s.G8, s.ld8 = t8["Gs"].data_ptr(), t8["ld"]
                    s.gscale8, s.gmax8 = t8["scale"].data_ptr(), t8["gmax"].data_ptr()
                if r == 0:
                    s.tier_counts = counts.ctypes.data
                    s.prefix_open = popen.ctypes.data
                qp = None
                if prefix and g.prefix_stages() and g.row_sample():
                    qp = g.quantize_queries(Qd, tier="f6p")
                    tp = g._tier_gallery("f6p")
                    s.pstages = tp["pst"]
                    s.Qtp, s.qscalep, s.qstatsp = qp["Qs"].data_ptr(), qp["scale"].data_ptr(), qp["stats"].data_ptr()
                    s.paux, s.spaux = tp["paux"].data_ptr(), tp["spaux"].data_ptr()
                    s.Gtp, s.gscalep, s.gmaxp = tp["Gs"].data_ptr(), tp["scale"].data_ptr(), tp["gmax"].data_ptr()
                keep.append((qq, ws, out_d, out_i, cert, qp))
        _lib.call("ofr_knn_sharded", self.handle, ctypes.cast(shards, ctypes.c_void_p), B, d, k)
        self.last_tier_counts = [int(x) for x in counts]
        self.last_prefix_open = int(popen[0])
        return [(o[2], o[3], o[4]) for o in keep[2:]]
