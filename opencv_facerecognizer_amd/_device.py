"""Device-resident layouts and the host side of every kernel call.

torch is used only for device memory, the current stream and (in
``parallel.py``) torch.distributed; all arithmetic of the hot path runs in the
HIP kernels of libocvf_hip.so.

Layouts:
* fp32 feature rows  [rows][ld], ld = round_up(d, 32), columns >= d zero
* projection matrix  W^T [d][ldw], ldw = round_up(D, 32), fp32, pad zero
* uint8 image rows   [rows][ldx], ldx = round_up(D, 16)
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream


SMALL_BATCH = 32   # B <= 32: HBM-streaming passes (fp6 first tier, fp32); larger batches: fp6/int8 tiles
# the int8 pass keeps 16 candidates per query; a certificate needs slack between the k-th
# exact distance and the 16th coarse score, so k is limited to half of that
Q8_MAX_K = 8


def round_up(x, m):
    return (int(x) + m - 1) // m * m


def dev():
    return _lib.device()


# ---------------------------------------------------------------------------
# uploads
# ---------------------------------------------------------------------------
def f32_rows(a, ld=None, device=None):
    """2-D float array (host or device) -> zero-padded fp32 [rows][ld] device tensor."""
    device = device or dev()
    if isinstance(a, torch.Tensor):
        t = a.to(device=device, dtype=torch.float32)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float32))).to(device)
    rows, d = t.shape
    ld = ld or max(32, round_up(d, 32))
    out = torch.zeros((rows, ld), dtype=torch.float32, device=device)
    out[:, :d] = t
    return out


def u8_rows(a, device=None):
    """Stack of uint8 images (n, ...) -> [n][round_up(D,16)] device tensor (D = prod of the image shape)."""
    device = device or dev()
    if isinstance(a, torch.Tensor):
        t = a.to(device=device, dtype=torch.uint8).reshape(a.shape[0], -1)
    else:
        arr = np.asarray(a)
        if arr.dtype != np.uint8:
            raise TypeError("image batch must be uint8")
        t = torch.from_numpy(np.ascontiguousarray(arr.reshape(arr.shape[0], -1))).to(device)
    n, D = t.shape
    ldx = round_up(max(D, 1), 16)
    if ldx == D:
        return t.contiguous()
    out = torch.zeros((n, ldx), dtype=torch.uint8, device=device)
    out[:, :D] = t
    return out


class _PinnedStage:
    """Page-locked staging for host face batches (predict_batch / compute on a host list of images): the
    items are stacked chunk by chunk into one of two 8 MiB pinned halves while the other half's copy to
    the device runs, so neither a fresh pageable stack (page faults on 41 MB at B = 4,096) nor a
    synchronous pageable copy sits on the call's path, and the pinned memory stays 16 MiB whatever
    the batch.  One stage per process; a lock serialises its users; per half an event keeps the host
    from overwriting bytes a copy (of this call or an earlier one) still reads."""

    HALF = 8 << 20

    def __init__(self):
        self.buf = None
        self.ev = [None, None]
        self.lock = threading.Lock()

    def upload(self, items, D, device):
        n = len(items)
        ldx = round_up(max(D, 1), 16)
        out = torch.empty((n, ldx), dtype=torch.uint8, device=device)
        if ldx != D:
            out[:, D:] = 0
        rows = max(1, self.HALF // max(D, 1))
        shape = np.asarray(items[0]).shape
        with self.lock:
            if self.buf is None or self.buf.numel() < 2 * rows * D:
                self.buf = torch.empty(2 * max(rows * D, self.HALF), dtype=torch.uint8, pin_memory=True)
                self.ev = [None, None]
            half = self.buf.numel() // 2
            host = self.buf.numpy()
            for j, c0 in enumerate(range(0, n, rows)):
                c1, h = min(n, c0 + rows), j & 1
                if self.ev[h] is not None:
                    self.ev[h].synchronize()
                np.stack(items[c0:c1], out=host[h * half:h * half + (c1 - c0) * D].reshape((c1 - c0,) + shape))
                out[c0:c1, :D].copy_(self.buf[h * half:h * half + (c1 - c0) * D].view(c1 - c0, D), non_blocking=True)
                self.ev[h] = torch.cuda.Event()
                self.ev[h].record()
        return out


_STAGE = _PinnedStage()


def upload_u8_items(items, device=None):
    """A host list of equally-shaped uint8 images -> device rows [n][round_up(D, 16)] through the pinned
    staging buffer; None when the items are not such a list (the caller stacks them itself)."""
    if not len(items) or isinstance(items, np.ndarray):
        return None
    first = np.asarray(items[0])
    if first.dtype != np.uint8 or type(items[0]) is not np.ndarray:
        return None
    # (identity first: the canonical uint8 dtype object is shared, so the common case skips the == compare;
    # 4,096 faces: 1.1 -> 0.6 ms of host time per call)
    dt, sh = first.dtype, first.shape
    if any(type(x) is not np.ndarray or (x.dtype is not dt and x.dtype != dt) or x.shape != sh for x in items):
        return None
    return _STAGE.upload(items, int(first.size), device or dev())


def u8_images(a, device=None):
    """uint8 image stack (n, H, W) -> contiguous device tensor."""
    device = device or dev()
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=torch.uint8).contiguous()
    arr = np.asarray(a)
    if arr.dtype != np.uint8 or arr.ndim != 3:
        raise TypeError("expected a uint8 image stack (n, H, W)")
    return torch.from_numpy(np.ascontiguousarray(arr)).to(device)


def f64_dev(a, device=None):
    device = device or dev()
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=torch.float64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float64))).to(device)


# ---------------------------------------------------------------------------
# projection  (feature.py:114-116, 184-185, 241-242)
# ---------------------------------------------------------------------------
class Projection:
    """Device form of a projection matrix W (D x d) for the exact int8-slice kernel.

    W is given as a host array (fp64 model weights) or as a device tensor Wt
    (d x >=D, fp32/fp64).  ``project(Xd, shift64, out_dtype)`` returns
    (x . W - shift) rounded once to fp32 (search layout, [B][ldy] with zero pad
    columns) or fp64.
    """

    def __init__(self, W=None, Wt_device=None, D=None, device=None):
        device = device or dev()
        if Wt_device is not None:
            Wt = Wt_device
            self.d = int(Wt.shape[0])
            self.D = int(D if D is not None else Wt.shape[1])
        else:
            W = np.asarray(W, dtype=np.float64)
            self.D, self.d = W.shape
            Wt = torch.from_numpy(np.ascontiguousarray(W.T)).to(device)
        dt = {torch.float32: _lib.DT_F32, torch.float64: _lib.DT_F64}[Wt.dtype]
        self.ldk = round_up(self.D, 128)
        nbytes = _lib.load().ofr_qproj_bytes(self.D, self.d)
        self.Aq = torch.empty(nbytes, dtype=torch.int8, device=device)
        self.scale = torch.empty(self.d, dtype=torch.float64, device=device)
        self.K = torch.empty(self.d, dtype=torch.float64, device=device)
        call("ofr_qproj_prepare", stream(), dt, ptr(Wt), self.d, self.D, Wt.shape[1], ptr(self.Aq), self.ldk,
             ptr(self.scale), ptr(self.K))
        self.ldy = max(32, round_up(self.d, 32))
        self._Wt_src = Wt_device             # the caller's W^T (device), or None: weights_f64 rebuilds W from it

    def weights_f64(self):
        """W (D x d) as fp64 on the device: the training's fp64 W (_W64, set by Fisherfaces._prime_proj), else
        the W^T this projection was made from."""
        if getattr(self, "_W64", None) is not None:
            return self._W64
        if self._Wt_src is not None:
            return self._Wt_src[:, :self.D].double().t()
        return f64_dev(np.asarray(self.W_host, np.float64))

    def project(self, Xd, shift64=None, out=None, f64=False, tiles=None):
        """Xd: uint8 [B][ldx] device rows.  fp32 [B][ldy] (zero pad) or fp64 [B][d].
        tiles=(t0, t1): only the grid's tiles [t0, t1) (ofr_project_u8_exact_range; see tile_count)."""
        B = Xd.shape[0]
        if out is None:
            out = torch.empty((B, self.d), dtype=torch.float64, device=Xd.device) if f64 else \
                torch.zeros((B, self.ldy), dtype=torch.float32, device=Xd.device)
        ydt = _lib.DT_F64 if out.dtype == torch.float64 else _lib.DT_F32
        args = (stream(), ptr(Xd), B, self.D, Xd.shape[1], ptr(self.Aq), self.ldk, ptr(self.scale), ptr(self.K),
                self.d, ptr(shift64), ptr(out), out.shape[1], ydt)
        if tiles is None:
            call("ofr_project_u8_exact", *args)
        else:
            call("ofr_project_u8_exact_range", *args, int(tiles[0]), int(tiles[1]))
        return out

    def tile_count(self, B):
        """Tiles of the projection grid for B faces (0: the B <= 4 GEMV, no tiles)."""
        return int(_lib.load().ofr_project_u8_exact_tiles(B, self.d))


def center_round(F64, shift64, ld, out=None):
    """fp64 rows [N][d] -> fp32 [N][ld] = rows - shift (pad columns zero), rounded once."""
    N, d = F64.shape
    if out is None:
        out = torch.zeros((N, ld), dtype=torch.float32, device=F64.device)
    call("ofr_center_round_f64", stream(), ptr(F64), N, d, F64.stride(0), ptr(shift64), ptr(out), out.shape[1])
    return out


# ---------------------------------------------------------------------------
# search  (classifier.py:76-129)
# ---------------------------------------------------------------------------
class Workspace:
    """Grow-only device scratch buffer (candidate lists of the search kernels)."""

    def __init__(self):
        self.buf = None

    def get(self, nbytes, device):
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != device:
            self.buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        return self.buf


class FloatGallery:
    """Device gallery for Euclidean / Cosine search.

    Euclidean: rows are stored CENTRED on a shift c (the gallery mean, fp64)
    and rounded to fp32 AFTER centring, so the stored values carry
    eps*|g - c| instead of eps*|g| of error (Fisherfaces features share a large
    common component); distances are translation invariant and queries are
    centred on the same c.  Cosine: raw rows (cosine is not translation
    invariant), shift None.
    """

    def __init__(self, feats, metric, device=None, shift64=None):
        """feats: host array [N][d] (any float type; used in fp64).  shift64 (Euclidean, fp64 [d]):
        centre on this vector instead of the rows' mean -- a sharded gallery centres every shard on
        the same one."""
        device = device or dev()
        self.metric = metric
        F = f64_dev(np.asarray(feats, np.float64), device=device) if not isinstance(feats, torch.Tensor) else \
            feats.to(device=device, dtype=torch.float64).contiguous()
        self.N, self.d = int(F.shape[0]), int(F.shape[1])
        self.ld = max(32, round_up(self.d, 32))
        self.shift64 = None
        if metric == _lib.METRIC_EUCLIDEAN and shift64 is not None:
            self.shift64 = f64_dev(shift64, device=device).reshape(-1).contiguous()
        elif metric == _lib.METRIC_EUCLIDEAN and self.N > 0:
            self.shift64 = col_mean_f64(F)
        self.G = center_round(F, self.shift64, self.ld)
        self._finish(device)

    @classmethod
    def from_device_rows(cls, G, d, metric, shift64=None):
        """Adopt fp32 rows [N][ld] that are already centred on shift64 (fp64 [d]) — e.g. written by Projection."""
        self = cls.__new__(cls)
        self.metric = metric
        self.G = G
        self.N, self.ld, self.d = int(G.shape[0]), int(G.shape[1]), int(d)
        self.shift64 = shift64
        self._finish(G.device)
        return self

    def _finish(self, device):
        self._Gbuf = self.G                      # rows [capacity][ld]; self.G = the first N
        self._auxbuf = torch.empty(max(self.N, 1), dtype=torch.float32, device=device)
        self.aux = self._auxbuf
        if self.N > 0:
            call("ofr_row_aux", stream(), self.metric, ptr(self.G), self.N, self.d, self.ld, ptr(self.aux))
        self.ws = Workspace()
        self.q8 = None
        self.bscale = None                       # fp6 tiers' column-block scales (block_scales)
        self._twin = None
        self.last_fallbacks = 0
        self.tier_failures = {}                  # tier -> recent uncertified fraction (start_tier)
        self._starts = 0

    def capacity(self):
        return int(self._Gbuf.shape[0])

    def append(self, feats):
        """Append gallery rows in place (NearestNeighbor.update, classifier.py:65-70): the new rows are
        centred on the EXISTING shift (any shift keeps distances exact; the first rows' mean keeps the
        fp32 rounding small), their aux terms and every built quantized tier are extended, the tier
        maxima recomputed.  Storage grows geometrically; a growth re-allocates and copies on the device
        and drops the quantized tiers (rebuilt on the next search).  Returns the new row count."""
        dev_ = self.G.device
        F = feats.to(device=dev_, dtype=torch.float64).contiguous() if isinstance(feats, torch.Tensor) else \
            f64_dev(np.asarray(feats, np.float64).reshape(-1, self.d), device=dev_)
        if F.ndim != 2 or F.shape[1] != self.d:
            raise ValueError(f"appended rows must have {self.d} features")
        n = int(F.shape[0])
        if n == 0:
            return self.N
        if self.N == 0:
            raise ValueError("append to an empty gallery: build it from the rows instead")
        N0, N1 = self.N, self.N + n
        if N1 > self.capacity():
            cap = max(N1, self.capacity() + self.capacity() // 2, 256)
            G = torch.zeros((cap, self.ld), dtype=torch.float32, device=dev_)
            G[:N0].copy_(self._Gbuf[:N0])
            aux = torch.empty(cap, dtype=torch.float32, device=dev_)
            aux[:N0].copy_(self._auxbuf[:N0])
            self._Gbuf, self._auxbuf, self.q8 = G, aux, None
        center_round(F, self.shift64, self.ld, out=self._Gbuf[N0:N1])
        call("ofr_row_aux", stream(), self.metric, ptr(self._Gbuf[N0:]), n, self.d, self.ld, ptr(self._auxbuf[N0:]))
        self.N, self.G, self.aux = N1, self._Gbuf[:N1], self._auxbuf[:N1]
        self.tier_failures = {}                    # new rows: the certificate statistics start over
        if self._twin is not None:                 # Cosine: the unit-row twin grows with it
            self._twin.append(self.unit_rows(self.G[N0:N1])[:, :self.d])
        for tier, g in (self.q8 or {}).items():     # "f6" before "f6x2": insertion order
            # the fp6 tiers keep the column-block scales they were built with (any scales are exact)
            if tier == "f6":
                call("ofr_f6_quantize_rows_at", stream(), ptr(self.G[N0:]), n, self.d, self.ld, N0, ptr(g["Gs"]),
                     g["Gs"].numel(), ptr(g["scale"]), ptr(g["stats"]), ptr(self.bscale))
                self._sample_rows(g, N0, N1)
            elif tier == "f6p":                        # its own compact tiles + the prefix terms (the row sample:
                call("ofr_row_aux", stream(), _lib.METRIC_EUCLIDEAN, ptr(self._Gbuf[N0:]), n, g["pdim"], self.ld,
                     ptr(g["paux"][N0:]))              # the f6 tier's, extended above)
                call("ofr_f6p_quantize_rows_at", stream(), ptr(self.G[N0:]), n, self.d, self.ld, N0, g["pst"],
                     ptr(g["Gs"]), g["Gs"].numel(), ptr(g["scale"]), ptr(g["stats"]), ptr(self.bscale))
                g["spaux"] = self._prefix_sample_aux(g["paux"], N1)
                g6 = self.q8["f6"]
                g["St"], g["sscale"] = g6["St"], g6["sscale"]
                call("ofr_q8_maxima", stream(), ptr(g["stats"]), ptr(g["paux"]), N1, ptr(g["gmax"]))
                continue
            elif tier == "f6x2":                       # the first slice is the f6 tier's, extended above
                call("ofr_f6x2_quantize_rows_at", stream(), ptr(self.G[N0:]), n, self.d, self.ld, N0, None,
                     ptr(g["Gs2"]), g["Gs2"].numel(), ptr(g["scale"]), ptr(g["stats"]), ptr(self.bscale))
                self._sample_rows2(g, N0, N1)
            else:
                call("ofr_q8_quantize_rows", stream(), tier, ptr(self.G[N0:]), n, self.d, self.ld, ptr(g["Gs"][N0:]),
                     g["ld"], ptr(g["scale"][N0:]), ptr(g["stats"][N0:]), None, None)
            call("ofr_q8_maxima", stream(), ptr(g["stats"]), ptr(self.aux), N1, ptr(g["gmax"]))
        return self.N

    # -- certified quantized coarse passes (Euclidean, B > 32) -------------------------------------
    # Tier "f6": one fp6 (e2m3) slice per row with an fp32 row scale (x~ = s v), fp6 MFMA at twice
    # the int8 rate.  Tier "f6x2", for the queries tier "f6" could not certify (crowded galleries):
    # two fp6 slices (x~ = s (v1 + v2/2^4), residual ~1/20 of f6's) in three fp6 MFMA segments.
    # Tier 1: one int8 slice (x~ = s x1; the first tier of OFR_SEARCH=q8).  Tier 2: two int8 slices
    # (x~ = s (x1 + x2/2^7)).  Last: the fp32 path.  Every tier ends in the exact fp64 re-rank; the
    # quantized tiers only answer where the certificate proves the result exact.
    # OFR_SEARCH picks the first tier: auto (= f6), q8 (tier 1), q8x2 (tier 2) or fp32.  NEXT: the
    # stage after each tier (f6x2 is finer than int8 x1, so its failures go on to int8 x2).
    # Tier "f6p" (prefix tier, before f6 when the gallery has one -- prefix_stages): the f6 tiles and
    # queries, scored on their first pstages 128-feature stages only.  Every squared distance is at least
    # its prefix part, so a query certifies as in f6 (merge_kernel's prefix bound); one that does not
    # runs the full f6 pass next.
    TIER_CHAIN = ("f6p", "f6", "f6x2", 1, 2, "fp32")
    NEXT = {"f6p": "f6", "f6": "f6x2", "f6x2": 2, 1: 2, 2: "fp32"}
    F6_TIERS = ("f6p", "f6", "f6x2")

    @classmethod
    def tier_path(cls, first):
        """The stages a query starting at tier `first` can pass through, in order (ends with fp32)."""
        path = [first]
        while path[-1] != "fp32":
            path.append(cls.NEXT[path[-1]])
        return tuple(path)

    # -- certified Cosine search: Euclidean tiers on the unit rows, then the reference formula ----------
    def unit_rows(self, X, shift64=None, out=None):
        """fp32 rows [n][>= d] -> fp32(x / ||x|| - shift) [n][ld] (fp64, rounded once)."""
        if out is None:
            out = torch.empty((X.shape[0], self.ld), dtype=torch.float32, device=X.device)
        call("ofr_normalize_rows_f32", stream(), ptr(X), X.shape[0], self.d, X.shape[1], ptr(shift64), ptr(out),
             self.ld)
        return out

    def _cos_twin(self):
        """Euclidean gallery of the unit rows, centred on their mean (Euclidean distances are translation
        invariant; features share a large common direction, and centring keeps the fp6 / int8
        quantization relative to the spread of the unit rows instead).  Built once, grown by append."""
        if self._twin is None:
            U = self.unit_rows(self.G)
            shift = torch.empty(self.d, dtype=torch.float64, device=U.device)
            call("ofr_col_mean", stream(), ptr(U), self.N, self.d, self.ld, ptr(shift))
            self.unit_rows(self.G, shift, out=U)     # centred, one rounding
            self._twin = FloatGallery.from_device_rows(U, self.d, _lib.METRIC_EUCLIDEAN, shift64=shift)
        return self._twin

    def use_cos_cert(self, B, k):
        """Certified Cosine path: not for galleries with a zero row (its distance is NaN, which the fp32
        path ranks last like the reference; a unit-row twin cannot represent it)."""
        if (os.environ.get("OFR_SEARCH", "auto") == "fp32" or self.metric != _lib.METRIC_COSINE or self.N == 0
                or B == 0 or k > Q8_MAX_K):
            return False
        if getattr(self, "_cos_ok", None) is None or self._cos_ok[0] != self.N:
            self._cos_ok = (self.N, not bool(torch.isinf(self.aux[:self.N]).any()))
        return self._cos_ok[1]

    def _search_cosine(self, Qd, k, index_base=0):
        """Cosine top-k = Euclidean top-k of the unit vectors (certified chain on the twin; ranks agree
        up to the fp32 rounding of the unit rows, ~1e-7 relative), distances by the reference formula."""
        tw = self._cos_twin()
        d_, i_ = tw.search(self.unit_rows(Qd, tw.shift64), k)
        self.last_fallbacks = tw.last_fallbacks
        call("ofr_cosine_pairs", stream(), ptr(Qd), Qd.shape[0], Qd.shape[1], ptr(self.G), self.N, self.ld, self.d,
             k, ptr(d_), ptr(i_))
        if index_base:
            i_ = torch.where(i_ >= 0, i_ + index_base, i_)
        # a zero query has no unit vector (every reference distance is NaN, distance.py:77): the fp32
        # path ranks it exactly as for any other NaN row set
        zero = torch.nonzero(Qd[:, :self.d].abs().amax(1) == 0).reshape(-1)
        if zero.numel():
            d2, i2 = self._search_f32(Qd.index_select(0, zero).contiguous(), k, index_base)
            d_.index_copy_(0, zero, d2)
            i_.index_copy_(0, zero, i2)
        return d_, i_

    def use_q8(self, B, k):
        mode = os.environ.get("OFR_SEARCH", "auto")
        return (mode != "fp32" and self.metric == _lib.METRIC_EUCLIDEAN and self.N > 0 and B > 0
                and k <= Q8_MAX_K)

    def next_tier(self, tier, nrows):
        """Stage after `tier` for `nrows` uncertified queries.  The int8 tiers run 256-query tiles
        over 10-30 GB of slices: for <= 32 queries the exact fp32 streaming pass is as cheap, so
        small sets go straight to it (and a small-batch workload never builds the int8 slices)."""
        nxt = self.NEXT[tier]
        return "fp32" if nxt != "fp32" and nrows <= SMALL_BATCH else nxt

    @staticmethod
    def first_tier():
        return {"q8": 1, "q8x2": 2}.get(os.environ.get("OFR_SEARCH", "auto"), "f6")

    # Adaptive start tier (serving, one device).  On a crowded gallery nearly every query fails the
    # fp6 certificate and pays the fp6 pass for nothing before the f6x2 pass rescues it.  start_tier
    # skips a quantized tier while its recent uncertified fraction (tier_failures: the latest batch of
    # >= ADAPT_MIN_BATCH queries, averaged with the one before) is >= SKIP_FAIL, never skipping to
    # the fp32 pass, and returns the configured first tier every REPROBE-th batch so a gallery that
    # stops being crowded is noticed.  A routing choice only: every stage certifies or hands on, the
    # results do not depend on it (tests/test_gpu_pipeline.py).  OFR_ADAPTIVE_TIER=0 disables it.
    SKIP_FAIL = 0.9
    REPROBE = 16
    ADAPT_MIN_BATCH = 256

    def start_tier(self, B):
        """First tier for a batch of B queries (see above); counts the batch."""
        first = self.first_tier()
        if first == "f6" and self.prefix_stages():
            first = "f6p"
        if B < self.ADAPT_MIN_BATCH or os.environ.get("OFR_ADAPTIVE_TIER", "1") != "1":
            return first
        self._starts += 1
        if self._starts % self.REPROBE == 0:
            return first
        t = first
        while self.tier_failures.get(t, 0.0) >= self.SKIP_FAIL and self.NEXT.get(t, "fp32") != "fp32":
            t = self.NEXT[t]
        return t

    def note_failures(self, tier, B, failed):
        """Record that `failed` of B queries that ran tier `tier` (from its start) stayed uncertified."""
        if B >= self.ADAPT_MIN_BATCH and tier != "fp32":
            f = failed / B
            prev = self.tier_failures.get(tier)
            self.tier_failures[tier] = f if prev is None else 0.5 * (prev + f)

    # -- column-block scales of the fp6 tiers (ofr_f6_block_scales) -------------------
    # One E8M0 byte per 32 features, shared by the gallery's fp6 tiles and every query batch: feature k
    # is quantized as x_k / 2^e with e = rint(log2(rms of its block / the largest block rms)), so the
    # row scale no longer lets the few high-variance columns of a trained Fisherfaces W (LDA eigenvalue
    # order) crush the rest into a handful of fp6 steps.  Any scales are exact for the certificate
    # (the stats are of the values stored); they only decide how tight it is.  OFR_F6_BLOCK_SCALES=0:
    # unit scales (the round-1..4 quantization).
    def block_sums(self):
        """Per-32-feature-block sums of squares of the gallery rows (fp64 device [ceil(d / 32)]): what a
        sharded gallery all-reduces before set_block_scales, so every rank quantizes alike."""
        sums = torch.zeros(-(-self.d // 32), dtype=torch.float64, device=self.G.device)
        call("ofr_f6_block_sumsq", stream(), ptr(self.G), self.N, self.d, self.ld, ptr(sums))
        return sums

    def set_block_scales(self, sums):
        """Column-block scales from block sums of squares (block_sums, possibly all-reduced); before the
        fp6 tiers are built (they keep the scales they were quantized with).  The same sums choose the
        prefix tier's length (prefix_stages), so the ranks of a sharded gallery agree on it too."""
        if self.q8 and any(t in self.q8 for t in self.F6_TIERS):
            raise RuntimeError("set_block_scales: the fp6 tiers are already built with other scales")
        self._pst = self.choose_prefix(sums.cpu().numpy(), self.d, self.N)
        if os.environ.get("OFR_F6_BLOCK_SCALES", "1") == "0":
            self.bscale = None
            return None
        nbytes = 4 * -(-self.d // 128)
        self.bscale = torch.empty(nbytes, dtype=torch.uint8, device=self.G.device)
        call("ofr_f6_block_scales", stream(), ptr(sums), self.d, ptr(self.bscale))
        return self.bscale

    def _block_scales(self):
        """The fp6 tiers' column-block scales, made from this gallery's rows on first use."""
        if self.bscale is None and not getattr(self, "_bscale_done", False):
            self._bscale_done = True
            if self.N > 0:
                self.set_block_scales(self.block_sums())
        return self.bscale

    # -- prefix tier f6p (ofr_knn_f6p_sampled) ------------------------------------------
    # Fisherfaces / Eigenfaces features come in eigenvalue order: the discriminating variance sits in
    # the leading columns (the trained W of the headline: 6 blocks of rms 54-272 against 11 for the other
    # 307).  A block is "leading" when its mean square is >= PREFIX_RATIO x the median block's; the
    # prefix covers the stages up to the last leading block, when that is at most 1/PREFIX_MAX_FRAC of
    # the stages and holds >= PREFIX_MIN_SHARE of the total variance; then the shortest prefix that still
    # holds PREFIX_SHORTEN of that share (the pass's cost grows with its stages, the bound's strength with
    # the share: on the headline's W one stage holds 0.74 against two stages' 0.83 and keeps as many
    # candidates, every query certified, 1.22M -> 1.28M queries/s, profiles/r05_prefix_len_ab.txt).
    # Isotropic features (a random W) have no prefix, and a gallery whose prefix certifies badly is
    # skipped by start_tier like any tier.  OFR_F6_PREFIX: auto (default), 0 (off) or a stage count.
    PREFIX_RATIO = 8.0
    PREFIX_MAX_FRAC = 4
    PREFIX_MIN_SHARE = 0.5
    PREFIX_SHORTEN = 0.85

    @classmethod
    def choose_prefix(cls, sums, d, N):
        """Prefix stages (0: no prefix tier) from the per-32-feature block sums of squares of the rows."""
        env = os.environ.get("OFR_F6_PREFIX", "auto").strip()
        nst = -(-d // 128)
        if env != "auto":
            if not env.isdigit():
                raise ValueError(f"OFR_F6_PREFIX must be 'auto' or a stage count (0: off), not {env!r}")
            return min(int(env), nst)
        if N < 1 or nst < cls.PREFIX_MAX_FRAC or os.environ.get("OFR_SIEVE_SAMPLE", "rows") == "panels":
            return 0
        width = np.minimum(32, d - 32 * np.arange(len(sums)))
        ms = np.asarray(sums, np.float64) / (N * width)
        med = float(np.median(ms))
        lead = np.nonzero(ms >= cls.PREFIX_RATIO * med)[0] if med > 0 else np.zeros(0, np.int64)
        if not len(lead):
            return 0
        pst = -(-32 * (int(lead[-1]) + 1) // 128)
        nb = 4 * pst                                     # the 32-feature blocks of pst stages
        share = float(ms[:nb].dot(width[:nb]) / ms.dot(width))
        if pst * cls.PREFIX_MAX_FRAC > nst or share < cls.PREFIX_MIN_SHARE:
            return 0
        for p in range(1, pst):
            if float(ms[:4 * p].dot(width[:4 * p]) / ms.dot(width)) >= cls.PREFIX_SHORTEN * share:
                return p
        return pst

    def prefix_stages(self):
        """Stages of the prefix tier for this gallery (0: none); Euclidean galleries, decided with the
        block scales (set_block_scales)."""
        if getattr(self, "_pst", None) is not None:
            return self._pst
        if self.metric != _lib.METRIC_EUCLIDEAN or self.N == 0:
            return 0
        if getattr(self, "_pst", None) is None:
            if self.bscale is None and not getattr(self, "_bscale_done", False):
                self._block_scales()
            if getattr(self, "_pst", None) is None:     # block scales were off or set elsewhere
                self._pst = self.choose_prefix(self.block_sums().cpu().numpy(), self.d, self.N)
        return self._pst

    def _prefix_sample_aux(self, paux, N):
        """Prefix terms of the row sample (rows 0, 64, 128, ...): saux[j] = paux[64 j]."""
        return paux[:N:_lib.load().ofr_f6_sample_step()].contiguous()

    @staticmethod
    def _q8_ld(d, slices):
        return round_up(d, 128) if slices == 1 else 2 * round_up(d, 64)

    def _tier_gallery(self, tier="f6"):
        """Quantized gallery rows of one tier (built once, kept on the device)."""
        if self.q8 is None:
            self.q8 = {}
        if tier not in self.q8:
            dev_ = self.G.device
            cap = self.capacity()                 # sized for the row storage (append fills in place)
            gs = torch.empty(cap, dtype=torch.float32, device=dev_)
            st = torch.empty((cap, 3), dtype=torch.float64, device=dev_)
            gmax = torch.empty(4, dtype=torch.float64, device=dev_)
            extra = {}
            if tier == "f6p":
                # its own compact tiles of the first pst stages (ofr_f6p_quantize_rows: power-of-two row scales,
                # prefix stats, maxima of those and of the prefix terms) and the f6 tier's row sample (St, sscale)
                # for the thresholds; built after f6, so append extends the sample first
                g6 = self._tier_gallery("f6")
                pst = self.prefix_stages()
                pdim = min(self.d, 128 * pst)
                if pdim < 1:
                    raise RuntimeError("f6p: this gallery has no prefix tier (prefix_stages() == 0)")
                paux = torch.empty(cap, dtype=torch.float32, device=dev_)
                call("ofr_row_aux", stream(), _lib.METRIC_EUCLIDEAN, ptr(self.G), self.N, pdim, self.ld, ptr(paux))
                nbytes = _lib.load().ofr_f6p_tiles_bytes(cap, pst)
                Gp = torch.empty(nbytes, dtype=torch.uint8, device=dev_)
                call("ofr_f6p_quantize_rows", stream(), ptr(self.G), self.N, self.d, self.ld, pst, ptr(Gp), nbytes,
                     ptr(gs), ptr(st), ptr(paux), ptr(gmax), ptr(self._block_scales()))
                self.q8[tier] = dict(Gs=Gp, scale=gs, stats=st, gmax=gmax, ld=0, paux=paux, pdim=pdim, pst=pst,
                                     spaux=self._prefix_sample_aux(paux, self.N), St=g6["St"], sscale=g6["sscale"])
                return self.q8[tier]
            if tier == "f6":
                lib = _lib.load()
                nbytes = lib.ofr_f6_tiles_bytes(cap, self.d)
                Gs = torch.empty(nbytes, dtype=torch.uint8, device=dev_)
                call("ofr_f6_quantize_rows", stream(), ptr(self.G), self.N, self.d, self.ld, ptr(Gs), nbytes,
                     ptr(gs), ptr(st), ptr(self.aux), ptr(gmax), ptr(self._block_scales()))
                # the sieve's row sample (ofr_knn_f6_sampled): rows 0, 64, 128, ... in their own tiles
                ns = -(-cap // lib.ofr_f6_sample_step())
                sbytes = lib.ofr_f6_tiles_bytes(ns, self.d)
                extra = dict(St=torch.empty(sbytes, dtype=torch.uint8, device=dev_),
                             sscale=torch.empty(ns, dtype=torch.float32, device=dev_),
                             sstats=torch.empty((ns, 3), dtype=torch.float64, device=dev_),
                             saux=torch.empty(ns, dtype=torch.float32, device=dev_))
                self._sample_rows(extra, 0, self.N)
                ld = 0
            elif tier == "f6x2":                  # first slice = the f6 tier's tiles (same codes and scale)
                Gs = self._tier_gallery("f6")["Gs"]
                nbytes = _lib.load().ofr_f6_tiles_bytes(cap, self.d)
                Gs2 = torch.empty(nbytes, dtype=torch.uint8, device=dev_)
                call("ofr_f6x2_quantize_rows", stream(), ptr(self.G), self.N, self.d, self.ld, None, ptr(Gs2),
                     nbytes, ptr(gs), ptr(st), ptr(self.aux), ptr(gmax), ptr(self._block_scales()))
                # second slices of the f6 tier's row sample (ofr_knn_f6x2_sampled)
                s1 = self._tier_gallery("f6")
                ns = int(s1["sscale"].numel())
                extra = dict(Gs2=Gs2, St2=torch.empty(_lib.load().ofr_f6_tiles_bytes(ns, self.d), dtype=torch.uint8,
                                                      device=dev_),
                             sscale2=torch.empty(ns, dtype=torch.float32, device=dev_),
                             sstats2=torch.empty((ns, 3), dtype=torch.float64, device=dev_))
                self._sample_rows2(extra, 0, self.N)
                ld = 0
            else:
                ld = self._q8_ld(self.d, tier)
                Gs = torch.empty((cap, ld), dtype=torch.int8, device=dev_)
                call("ofr_q8_quantize_rows", stream(), tier, ptr(self.G), self.N, self.d, self.ld, ptr(Gs), ld,
                     ptr(gs), ptr(st), ptr(self.aux), ptr(gmax))
            self.q8[tier] = dict(Gs=Gs, scale=gs, stats=st, gmax=gmax, ld=ld, **extra)
        return self.q8[tier]

    def _sample_rows(self, g, N0, N1):
        """Extend the f6 tier's row sample over gallery rows [N0, N1) (ofr_f6_sample_rows)."""
        step = _lib.load().ofr_f6_sample_step()
        j0, j1 = -(-N0 // step), -(-N1 // step)
        call("ofr_f6_sample_rows", stream(), ptr(self._Gbuf), N1, self.ld, self.d, j0, j1, ptr(self._auxbuf),
             ptr(g["St"]), g["St"].numel(), ptr(g["sscale"]), ptr(g["sstats"]), ptr(g["saux"]), ptr(self.bscale))

    def _sample_rows2(self, g, N0, N1):
        """Extend the f6x2 tier's second-slice row sample over gallery rows [N0, N1) (ofr_f6x2_sample_rows)."""
        step = _lib.load().ofr_f6_sample_step()
        j0, j1 = -(-N0 // step), -(-N1 // step)
        call("ofr_f6x2_sample_rows", stream(), ptr(self._Gbuf), N1, self.ld, self.d, j0, j1, ptr(g["St2"]),
             g["St2"].numel(), ptr(g["sscale2"]), ptr(g["sstats2"]), ptr(self.bscale))

    @staticmethod
    def row_sample():
        """The fp6 sieve's thresholds from the row sample (default) or, OFR_SIEVE_SAMPLE=panels, from every
        64th 256-row panel (ofr_knn_f6; probe / A-B)."""
        return os.environ.get("OFR_SIEVE_SAMPLE", "rows") != "panels"

    def quantize_queries(self, Qd, out=None, tier="f6"):
        """Centred fp32 query rows -> the tier's quantized rows, scales and stats (device)."""
        B = Qd.shape[0]
        dev_ = Qd.device
        if out is None or out["B"] != B or out["tier"] != tier:
            extra = {}
            if tier in self.F6_TIERS:
                nb = max(1, _lib.load().ofr_f6_tiles_bytes(B, self.d))
                Qs = torch.empty(nb, dtype=torch.uint8, device=dev_)
                if tier == "f6x2":
                    extra = dict(Qs2=torch.empty(nb, dtype=torch.uint8, device=dev_))
            else:
                Qs = torch.empty((B, self._q8_ld(self.d, tier)), dtype=torch.int8, device=dev_)
            out = dict(Qs=Qs, scale=torch.empty(B, dtype=torch.float32, device=dev_),
                       stats=torch.empty((B, 3), dtype=torch.float64, device=dev_),
                       cert=torch.empty(B, dtype=torch.int32, device=dev_),
                       bound=torch.empty(B, dtype=torch.float64, device=dev_), tier=tier, B=B, **extra)
        if tier == "f6p":                          # the prefix stages only (ofr_f6_quantize_rows_prefix)
            call("ofr_f6_quantize_rows_prefix", stream(), ptr(Qd), B, self.d, Qd.shape[1], self.prefix_stages(),
                 ptr(out["Qs"]), out["Qs"].numel(), ptr(out["scale"]), ptr(out["stats"]), ptr(self._block_scales()))
        elif tier == "f6":
            call("ofr_f6_quantize_rows", stream(), ptr(Qd), B, self.d, Qd.shape[1], ptr(out["Qs"]),
                 out["Qs"].numel(), ptr(out["scale"]), ptr(out["stats"]), None, None, ptr(self._block_scales()))
        elif tier == "f6x2":
            call("ofr_f6x2_quantize_rows", stream(), ptr(Qd), B, self.d, Qd.shape[1], ptr(out["Qs"]), ptr(out["Qs2"]),
                 out["Qs"].numel(), ptr(out["scale"]), ptr(out["stats"]), None, None, ptr(self._block_scales()))
        else:
            call("ofr_q8_quantize_rows", stream(), tier, ptr(Qd), B, self.d, Qd.shape[1], ptr(out["Qs"]),
                 out["Qs"].shape[1], ptr(out["scale"]), ptr(out["stats"]), None, None)
        return out

    def gather_queries(self, qq, group=None):
        """Quantized query rows of this rank's block of the batch -> the whole batch (all-gather over
        the ranks, rank-major).  The fp6 tiles concatenate only whole 256-row panels: every rank's
        block must be a multiple of 256 rows (int8 tiers: any equal split)."""
        from .parallel import gather_rows
        if qq["tier"] in self.F6_TIERS and qq["B"] % 256:
            raise ValueError("fp6 query tiles gather whole 256-row panels: rows per rank must be a multiple of 256")
        # scales (fp32, exact in fp64) and stats travel as one [rows][4] fp64 block: two collectives, not three
        side = gather_rows(torch.cat([qq["scale"].to(torch.float64).reshape(-1, 1), qq["stats"]], 1).contiguous(), group)
        B = side.shape[0]
        extra = {"Qs2": gather_rows(qq["Qs2"], group)} if qq["tier"] == "f6x2" else {}
        return dict(Qs=gather_rows(qq["Qs"], group), scale=side[:, 0].to(torch.float32).contiguous(),
                    stats=side[:, 1:].contiguous(), cert=torch.empty(B, dtype=torch.int32, device=side.device),
                    bound=torch.empty(B, dtype=torch.float64, device=side.device), tier=qq["tier"], B=B, **extra)

    def search_q8_phase(self, phases, Qd, qq, k, index_base=0, out=None, workspace=None):
        """phases 1 = quantized tiles, 2 = merge + exact re-rank + certificate (cert in qq["cert"]), 3 = both.
        The fp6 tiers split phase 1 (ofr_knn_f6): 4 = sample pass + thresholds, 8 = the sieve pass; the
        int8 tiers run all of phase 1 under bit 4 and nothing under bit 8.
        workspace: a Workspace of the caller's instead of the gallery's."""
        tier = qq["tier"]
        if tier not in self.F6_TIERS and phases & 12:
            phases = (phases & 3) | (1 if phases & 4 else 0)
            if phases == 0:
                return out
        g = self._tier_gallery(tier)
        B = Qd.shape[0]
        if out is None:
            out = (torch.empty((B, k), dtype=torch.float64, device=Qd.device),
                   torch.empty((B, k), dtype=torch.int64, device=Qd.device))
        lib = _lib.load()
        nbytes = (lib.ofr_knn_f6_workspace_bytes(B, self.N) if tier in self.F6_TIERS
                  else lib.ofr_knn_q8_workspace_bytes(B, self.N))
        ws = (workspace or self.ws).get(nbytes, Qd.device)
        if tier == "f6p":
            ns = -(-self.N // lib.ofr_f6_sample_step())
            call("ofr_knn_f6p_sampled", stream(), phases, ptr(Qd), B, Qd.shape[1], ptr(qq["Qs"]), ptr(qq["scale"]),
                 ptr(qq["stats"]), ptr(self.G), self.N, self.ld, self.d, ptr(g["Gs"]), ptr(g["scale"]),
                 ptr(g["paux"]), ptr(g["gmax"]), k, index_base, ptr(out[0]), ptr(out[1]), ptr(qq["cert"]),
                 ptr(qq["bound"]), ptr(g["St"]), ns, ptr(g["sscale"]), ptr(g["spaux"]), ptr(ws), ws.numel(),
                 ptr(self.bscale), g["pst"])
        elif tier == "f6x2" and self.row_sample():
            s1 = self._tier_gallery("f6")
            ns = -(-self.N // lib.ofr_f6_sample_step())
            # the sample's row scales: the f6x2 builder's own (sscale2), equal to the f6 tier's by construction
            # (quantize_f6_kernel<true> makes the same per-row scale; test_row_sample_extended_by_append pins it)
            call("ofr_knn_f6x2_sampled", stream(), phases, ptr(Qd), B, Qd.shape[1], ptr(qq["Qs"]), ptr(qq["Qs2"]),
                 ptr(qq["scale"]), ptr(qq["stats"]), ptr(self.G), self.N, self.ld, self.d, ptr(g["Gs"]),
                 ptr(g["Gs2"]), ptr(g["scale"]), ptr(self.aux), ptr(g["gmax"]), k, index_base, ptr(out[0]),
                 ptr(out[1]), ptr(qq["cert"]), ptr(qq["bound"]), ptr(s1["St"]), ptr(g["St2"]), ns,
                 ptr(g["sscale2"]), ptr(s1["saux"]), ptr(ws), ws.numel(), ptr(self.bscale))
        elif tier == "f6x2":
            call("ofr_knn_f6x2", stream(), phases, ptr(Qd), B, Qd.shape[1], ptr(qq["Qs"]), ptr(qq["Qs2"]),
                 ptr(qq["scale"]), ptr(qq["stats"]), ptr(self.G), self.N, self.ld, self.d, ptr(g["Gs"]),
                 ptr(g["Gs2"]), ptr(g["scale"]), ptr(self.aux), ptr(g["gmax"]), k, index_base, ptr(out[0]),
                 ptr(out[1]), ptr(qq["cert"]), ptr(qq["bound"]), ptr(ws), ws.numel(), ptr(self.bscale))
        elif tier == "f6" and self.row_sample():
            ns = -(-self.N // lib.ofr_f6_sample_step())
            call("ofr_knn_f6_sampled", stream(), phases, ptr(Qd), B, Qd.shape[1], ptr(qq["Qs"]), ptr(qq["scale"]),
                 ptr(qq["stats"]), ptr(self.G), self.N, self.ld, self.d, ptr(g["Gs"]), ptr(g["scale"]),
                 ptr(self.aux), ptr(g["gmax"]), k, index_base, ptr(out[0]), ptr(out[1]), ptr(qq["cert"]),
                 ptr(qq["bound"]), ptr(g["St"]), ns, ptr(g["sscale"]), ptr(g["saux"]), ptr(ws), ws.numel(),
                 ptr(self.bscale))
        elif tier == "f6":
            call("ofr_knn_f6", stream(), phases, ptr(Qd), B, Qd.shape[1], ptr(qq["Qs"]), ptr(qq["scale"]),
                 ptr(qq["stats"]), ptr(self.G), self.N, self.ld, self.d, ptr(g["Gs"]), ptr(g["scale"]),
                 ptr(self.aux), ptr(g["gmax"]), k, index_base, ptr(out[0]), ptr(out[1]), ptr(qq["cert"]),
                 ptr(qq["bound"]), ptr(ws), ws.numel(), ptr(self.bscale))
        else:
            call("ofr_knn_q8", stream(), phases, tier, ptr(Qd), B, Qd.shape[1], ptr(qq["Qs"]), ptr(qq["scale"]),
                 ptr(qq["stats"]), ptr(self.G), self.N, self.ld, self.d, ptr(g["Gs"]), g["ld"],
                 ptr(g["scale"]), ptr(self.aux), ptr(g["gmax"]), k, index_base, ptr(out[0]), ptr(out[1]),
                 ptr(qq["cert"]), ptr(qq["bound"]), ptr(ws), ws.numel())
        return out

    def merge_pruned(self, stage, Qd, qq, k, ub, index_base=0, out=None, workspace=None):
        """The split fp6 merge of a sharded gallery (ofr_knn_f6_merge_pruned, after phase 1 on the same
        workspace -- the gallery's, or the caller's): stage 1 writes ub [B][k] (this shard's upper
        bounds), stage 2 re-ranks pruned by ub [B] (the global bound) into out / qq["cert"] / qq["bound"].
        Tier f6p (round 6, ofr_knn_f6p_merge_pruned): stage 1's bounds are the exact squared distances of
        each query's first k candidates (a prefix key bounds nothing from above)."""
        tier = qq["tier"]
        g = self._tier_gallery(tier)
        B = Qd.shape[0]
        lib = _lib.load()
        ws = (workspace or self.ws).get(lib.ofr_knn_f6_workspace_bytes(B, self.N), Qd.device)
        o = out if out is not None else (None, None)
        args = [stream(), stage, ptr(Qd), B, Qd.shape[1], ptr(qq["Qs"]), ptr(qq["scale"]), ptr(qq["stats"]),
                ptr(self.G), self.N, self.ld, self.d, ptr(g["Gs"]), ptr(g["scale"]),
                ptr(g["paux"] if tier == "f6p" else self.aux), ptr(g["gmax"]), k, index_base, ptr(o[0]), ptr(o[1]),
                ptr(qq["cert"]), ptr(qq["bound"]), ptr(ub), ptr(ws), ws.numel()]
        if tier == "f6p":
            call("ofr_knn_f6p_merge_pruned", *args, g["pst"])
        else:
            call("ofr_knn_f6_merge_pruned", *args)
        return out

    def sieve_counts(self, B, workspace=None):
        """Rows kept per query by the last fp6 sieve pass of a B-query batch on `workspace` (the
        gallery's by default; int32 device view, valid until the next search on it), or None when
        B <= 32 (no sieve)."""
        off = _lib.load().ofr_knn_f6_sieve_counts_offset(B, self.N)
        w = workspace or self.ws
        if off == ctypes.c_size_t(-1).value or w.buf is None:
            return None
        return w.buf[off:off + 4 * B].view(torch.int32)

    def merge_evals(self, B, workspace=None):
        """Candidates each query of the last fp6-tier merge (phase 2) of a B-query batch on `workspace`
        re-ranked exactly (int32 device view [B]; its bytes: evals x d x 4 of fp32 rows)."""
        off = _lib.load().ofr_knn_f6_merge_evals_offset(B, self.N)
        w = workspace or self.ws
        if w.buf is None:
            return None
        return w.buf[off:off + 4 * B].view(torch.int32)

    SIEVE_CAP = 32768          # q8s::SIEVE_CAP: bucket slots per query

    def sieve_state(self, B, workspace=None):
        """The last fp6 sieve pass's per-query state on `workspace` (device views, B > 32): thresholds
        theta (uint32 order keys as int32 [B]; the kernel keeps a row iff !(score > key_float(theta |
        0xff))), counts [B] (rows that passed; > cap = overflow) and buckets [B][cap] of (truncated
        score fp32, row int32) pairs.  Layout of ofr_knn_f6's workspace (theta, count, bucket regions,
        each 256-byte aligned)."""
        off = _lib.load().ofr_knn_f6_sieve_counts_offset(B, self.N)
        w = workspace or self.ws
        if off == ctypes.c_size_t(-1).value or w.buf is None:
            return None
        step = round_up(4 * B, 256)
        theta = w.buf[off - step:off - step + 4 * B].view(torch.int32)
        count = w.buf[off:off + 4 * B].view(torch.int32)
        raw = w.buf[off + step:off + step + B * self.SIEVE_CAP * 8].view(torch.int32).view(B, self.SIEVE_CAP, 2)
        return theta, count, raw[:, :, 0].view(torch.float32), raw[:, :, 1]

    def fallback(self, Qd, qq, k, out, index_base=0, timings=None):
        """Re-run the queries the first tier left uncertified down the tier chain (then fp32).
        Returns the number of first-tier failures (host sync); self.last_fallbacks = the number of
        uncertified queries after each quantized tier that ran.  timings (a list, optional)
        receives (tier, queries, ms) per stage that ran (HIP events on the current stream)."""
        bad = open_rows(qq["cert"])
        if qq["tier"] == "f6" and 0 < int(bad.numel()) <= self.resieve_max() and self.resieve_enabled():
            bad = self._resieve(Qd, bad, k, out, index_base, qq)   # round 6: part of the fp6 tier
        counts = [int(bad.numel())]
        self.note_failures(qq["tier"], int(qq["B"]), counts[0])
        pending = {}                    # tier -> indices into the original batch waiting for it
        self.last_skipped = {}
        self._route(qq["tier"], bad, Qd, qq["stats"].index_select(0, bad), qq["bound"].index_select(0, bad), out, k,
                    pending)
        for tier in self.tier_path(qq["tier"])[1:]:
            rows = pending.pop(tier, None)
            if rows is None or not rows.numel():
                continue
            if tier != "fp32" and int(rows.numel()) <= SMALL_BATCH:   # see next_tier
                self._queue(pending, "fp32", rows)
                continue
            if timings is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            sub = Qd.index_select(0, rows).contiguous()
            if tier == "fp32":
                d2, i2 = self._search_f32(sub, k, index_base)
                out[0].index_copy_(0, rows, d2)
                out[1].index_copy_(0, rows, i2)
            else:
                q2 = self.quantize_queries(sub, tier=tier)
                d2, i2 = self.search_q8_phase(3, sub, q2, k, index_base)
                out[0].index_copy_(0, rows, d2)
                out[1].index_copy_(0, rows, i2)
                still = open_rows(q2["cert"])
                counts.append(int(still.numel()))
                self.note_failures(tier, int(rows.numel()), counts[-1])
                self._route(tier, rows.index_select(0, still), Qd, q2["stats"].index_select(0, still),
                            q2["bound"].index_select(0, still), out, k, pending)
            if timings is not None:
                ev[1].record()
                ev[1].synchronize()
                timings.append((str(tier), int(rows.numel()), ev[0].elapsed_time(ev[1])))
        self.last_fallbacks = tuple(counts)
        return counts[0]

    # the fp6 tier's second sieve pass for the queries it left open (round 6): at most this many
    RESIEVE_MAX = 256

    @classmethod
    def resieve_max(cls):
        return int(os.environ.get("OFR_RESIEVE_MAX", cls.RESIEVE_MAX))

    @staticmethod
    def resieve_enabled():
        """OFR_RESIEVE=0 turns the fp6 tier's second sieve pass off (then also off when the merge's deep
        continuation is: the second pass keeps rows for it to re-rank)."""
        return os.environ.get("OFR_RESIEVE", "1") != "0" and os.environ.get("OFR_MERGE_DEEP", "32") != "0"

    def _resieve(self, Qd, rows, k, out, index_base, qq):
        """The fp6 tier again for the queries it left open (rows of the batch), keeping every gallery row
        whose coarse score could still beat the query's k-th exact distance so far: smax = d_k^2 - |q|^2 + dS
        (merge_kernel's d2_lower inverted, with 1e-9 of slack), set by ofr_knn_f6_set_thresholds instead of
        the sample pass; the merge's deep continuation re-ranks the kept rows in key order until the
        certificate holds.  A query whose sieve bucket overflows (32768 rows) stays open.  The batch is padded
        to 33 rows (the sieve runs for B > 32; the pads repeat the first row).  Writes the results of the
        queries it certifies into out and qq["cert"] / qq["bound"]; returns the rows still open."""
        n = int(rows.numel())
        pad = max(0, 33 - n)
        prow = torch.cat([rows, rows[:1].expand(pad)]) if pad else rows
        sub = Qd.index_select(0, prow).contiguous()
        q2 = self.quantize_queries(sub, tier="f6")
        dk = out[0].index_select(0, prow)[:, k - 1].double()
        qn = (sub[:, : self.d].double() ** 2).sum(1)
        dS = self._dS("f6", q2["stats"]) * (1.0 + 1e-6)
        smax = (dk * dk - qn + dS) * (1.0 + 1e-9) + 1e-9 * (dk * dk + qn + dS)
        smax = torch.where(torch.isfinite(smax), smax, torch.full_like(smax, float("inf")))
        B2 = int(prow.numel())
        lib = _lib.load()
        ws = self.ws.get(lib.ofr_knn_f6_workspace_bytes(B2, self.N), Qd.device)
        call("ofr_knn_f6_set_thresholds", stream(), ptr(smax), B2, self.N, ptr(ws), ws.numel())
        d2, i2 = self.search_q8_phase(8 | 2, sub, q2, k, index_base, workspace=None)
        ok = q2["cert"][:n] != 0
        done = rows[ok]
        out[0].index_copy_(0, done, d2[:n][ok])
        out[1].index_copy_(0, done, i2[:n][ok])
        qq["cert"].index_fill_(0, done, 1)
        qq["bound"].index_copy_(0, done, q2["bound"][:n][ok])
        return rows[~ok]

    # the k-th distance must clear the next tier's predicted bound by this factor of the bound's gain
    ROUTE_SLACK = 1.5

    def _dS(self, tier, stats):
        """|S - S~| bound of the tier per query (merge_kernel's dS), stats [n][3] fp64."""
        gm = self._tier_gallery(tier)["gmax"]
        A, E, T, aux = gm[0], gm[1], gm[2], gm[3]
        a, e, t = stats[:, 0], stats[:, 1], stats[:, 2]
        nseg = {"f6p": 1, "f6": 1, "f6x2": 3}.get(tier, 0)
        gamma = (2 * nseg * -(-self.d // 128) + 64) * 2.0 ** -23 if nseg else 0.0
        return 2.0 * (a * E + e * A + e * E + t * T) + 2.0 ** -20 * (aux + 2.0 * a * A) + 2.0 * gamma * a * A

    def _route(self, tier, rows, Qd, stats, bound, out, k, pending):
        """Queue the queries `tier` left uncertified (rows; their stats and bounds in that tier) for the
        next stage.  A query whose k-th distance misses even the bound the next quantized tier would
        give it -- this tier's bound moved by the drop in dS, the candidate order assumed unchanged,
        with ROUTE_SLACK to spare -- skips that tier (from f6: a query f6x2 cannot rescue goes straight
        to int8 x2 instead of paying a three-segment pass for nothing).  Only a routing choice:
        every stage still certifies or hands on, so the results do not depend on it."""
        if not rows.numel():
            return
        nxt = self.NEXT[tier]
        after = self.NEXT.get(nxt)
        # from the prefix tier: its bound is of the prefix distance, which predicts nothing of f6's
        if tier == "f6p" or after is None or after == "fp32" or int(rows.numel()) <= SMALL_BATCH:
            self._queue(pending, nxt, rows)
            return
        sub = Qd.index_select(0, rows).contiguous()
        st_next = self.quantize_queries(sub, tier=nxt)["stats"]
        gain = self._dS(tier, stats) - self._dS(nxt, st_next)
        kth = out[0].index_select(0, rows)[:, k - 1]
        # -inf bound (sieve overflow): no information, try the next tier
        hopeless = torch.isfinite(bound) & (kth * kth >= bound + self.ROUTE_SLACK * gain)
        skip = rows[hopeless]
        keep = rows[~hopeless]
        self.last_skipped[str(nxt)] = int(skip.numel())
        self._queue(pending, nxt, keep)
        self._queue(pending, after, skip)

    @staticmethod
    def _queue(pending, tier, rows):
        if rows.numel():
            pending[tier] = rows if tier not in pending else torch.cat([pending[tier], rows])

    def query_rows(self, Q64):
        """Host or device fp64 query features [B][d] -> centred fp32 search rows [B][ld]."""
        Q = Q64 if isinstance(Q64, torch.Tensor) else f64_dev(np.asarray(Q64, np.float64), device=self.G.device)
        return center_round(Q.to(torch.float64).contiguous(), self.shift64, self.ld)

    def search_phase(self, phase, Qd, k, index_base=0, out=None, workspace=None):
        """One pass of the search: phase "tiles" (MFMA pass) or "merge" (merge + exact re-rank), both
        on the same workspace (the gallery's, or the caller's)."""
        B = Qd.shape[0]
        if out is None:
            out = (torch.empty((B, k), dtype=torch.float64, device=Qd.device),
                   torch.empty((B, k), dtype=torch.int64, device=Qd.device))
        lib = _lib.load()
        ws = (workspace or self.ws).get(lib.ofr_knn_workspace_bytes(B, self.N, k), Qd.device)
        name = "ofr_knn_tiles_f32" if phase == "tiles" else "ofr_knn_merge_f32"
        call(name, stream(), self.metric, ptr(Qd), B, Qd.shape[1], ptr(self.G), self.N, self.ld, self.d,
             ptr(self.aux), k, index_base, ptr(out[0]), ptr(out[1]), ptr(ws), ws.numel())
        return out

    def search(self, Qd, k, index_base=0):
        """Qd: centred fp32 search rows [B][ld] (see query_rows / Projection.project with shift64)."""
        if Qd.shape[1] != self.ld:
            raise ValueError(f"query row stride {Qd.shape[1]} != gallery stride {self.ld}")
        B = Qd.shape[0]
        if self.use_cos_cert(B, k):
            return self._search_cosine(Qd, k, index_base)
        if self.use_q8(B, k):
            self.last_start_tier = self.start_tier(B)
            qq = self.quantize_queries(Qd, tier=self.last_start_tier)
            out = self.search_q8_phase(3, Qd, qq, k, index_base)
            self.fallback(Qd, qq, k, out, index_base)
            return out
        return self._search_f32(Qd, k, index_base)

    def _search_f32(self, Qd, k, index_base=0):
        if k > _lib.MAX_K:
            return search_deep(self.metric, Qd, _lib.DT_F32, self.G, _lib.DT_F32, self.d, 1.0, k, index_base,
                               workspace=self.ws)
        B = Qd.shape[0]
        out_d = torch.empty((B, k), dtype=torch.float64, device=Qd.device)
        out_i = torch.empty((B, k), dtype=torch.int64, device=Qd.device)
        lib = _lib.load()
        nbytes = lib.ofr_knn_workspace_bytes(B, self.N, k)
        ws = self.ws.get(nbytes, Qd.device)
        call("ofr_knn_f32", stream(), self.metric, ptr(Qd), B, Qd.shape[1], ptr(self.G), self.N, self.ld, self.d,
             ptr(self.aux), k, index_base, ptr(out_d), ptr(out_i), ptr(ws), ws.numel())
        return out_d, out_i


_COUNT_DT = {1: (_lib.DT_U8, torch.uint8, np.uint8, 255), 2: (_lib.DT_U16, torch.int16, np.uint16, 65535),
             4: (_lib.DT_U32, torch.int32, np.uint32, 2 ** 32 - 1)}


def counts_of(F, denom, count_bytes=None):
    """Float rows F [n][nbins] that are EXACTLY integer counts / denom (the SpatialHistogram values,
    feature.py:298-299) -> (uint counts host array, bytes per count); None when they are not."""
    F = np.asarray(F, np.float64)
    if F.size and not np.isfinite(F).all():
        return None
    C = np.rint(F * denom)
    if F.size and (C.min() < 0 or not np.array_equal(C / denom, F)):
        return None
    top = C.max() if C.size else 0
    cb = count_bytes or next((b for b in (1, 2, 4) if top <= _COUNT_DT[b][3]), None)
    if cb is None or top > _COUNT_DT[cb][3]:       # wider than 32-bit counts: not a counts gallery
        return None
    return C.astype(_COUNT_DT[cb][2]), cb


def infer_count_denom(F):
    """The cell pixel count of LBP spatial histograms F (floats = count / cell): 1 / the smallest
    positive value when that divides every value exactly, else None (not a count histogram)."""
    F = np.asarray(F, np.float64)
    pos = F[F > 0]
    if not pos.size:
        return None
    denom = float(np.rint(1.0 / pos.min()))
    return denom if denom >= 1 and counts_of(F, denom) is not None else None


class Chi2Gallery:
    """Device gallery for ChiSquare search: fp32 values, or integer counts with a denominator
    (the LBP spatial histograms: count / cell, held as the counts -- exact and 4x smaller)."""

    def __init__(self, rows, dtype=_lib.DT_F32, denom=1.0, nbins=None, device=None):
        device = device or dev()
        self.dtype = dtype
        self.denom = float(denom)
        if isinstance(rows, torch.Tensor):
            self.G = rows.to(device).contiguous()
            self.nbins = int(nbins or rows.shape[1])
        else:
            arr = np.asarray(rows, np.float64)
            self.nbins = int(arr.shape[1])
            self.G = f32_rows(arr, ld=max(4, round_up(self.nbins, 4)), device=device)
        self.N = int(self.G.shape[0])
        self._Gbuf = self.G
        self.ws = Workspace()
        self.last_fallbacks = ()

    @classmethod
    def from_counts(cls, C, count_bytes, denom, device=None):
        """Host or device counts [n][nbins] (uint8 / uint16 / uint32 values) -> a counts gallery."""
        dt, tdt, ndt, _ = _COUNT_DT[count_bytes]
        device = device or dev()
        if not isinstance(C, torch.Tensor):
            C = torch.from_numpy(np.ascontiguousarray(np.asarray(C).astype(ndt).view(
                {1: np.uint8, 2: np.int16, 4: np.int32}[count_bytes])))
        nbins = int(C.shape[1])
        ld = round_up(max(nbins, 1), 16 // count_bytes)      # 16-byte rows for the tile kernel's loads
        G = C.to(device=device, dtype=tdt)
        if ld != nbins:
            Gp = torch.zeros((G.shape[0], ld), dtype=tdt, device=device)
            Gp[:, :nbins] = G
            G = Gp
        return cls(G, dtype=dt, denom=denom, nbins=nbins, device=device)

    @property
    def count_bytes(self):
        return {_lib.DT_U8: 1, _lib.DT_U16: 2, _lib.DT_U32: 4}.get(self.dtype)

    def counts_rows(self, arr):
        """Host float rows -> device counts rows of this (counts) gallery, or None when the rows are not
        exactly counts / denom in range (the caller then uses a float gallery)."""
        cb = self.count_bytes
        got = counts_of(np.asarray(arr, np.float64).reshape(-1, self.nbins), self.denom, cb) if cb else None
        if got is None:
            return None
        C = torch.from_numpy(np.ascontiguousarray(got[0].view({1: np.uint8, 2: np.int16, 4: np.int32}[cb])))
        out = torch.zeros((C.shape[0], self.G.shape[1]), dtype=self.G.dtype, device=self.G.device)
        out[:, :self.nbins] = C.to(self.G.device)
        return out

    def append(self, rows):
        """Append rows in place (NearestNeighbor.update): host float rows (for a counts gallery they must
        be exact counts / denom, else TypeError) or a device tensor of the gallery's element type;
        geometric growth.  Returns the new row count."""
        if isinstance(rows, torch.Tensor) and rows.dtype == self._Gbuf.dtype:
            new = torch.zeros((rows.shape[0], self._Gbuf.shape[1]), dtype=rows.dtype, device=self._Gbuf.device)
            new[:, :rows.shape[1]] = rows.to(self._Gbuf.device)
        elif self.dtype == _lib.DT_F32:
            new = f32_rows(np.asarray(rows, np.float64).reshape(-1, self.nbins), ld=self._Gbuf.shape[1],
                           device=self._Gbuf.device)
        else:
            new = None if isinstance(rows, torch.Tensor) else self.counts_rows(rows)
            if new is None:
                raise TypeError("append to a count gallery takes counts / denom rows or a device tensor of its "
                                "element type")
        n = int(new.shape[0])
        N0, N1 = self.N, self.N + n
        if N1 > self._Gbuf.shape[0]:
            cap = max(N1, self._Gbuf.shape[0] + self._Gbuf.shape[0] // 2, 256)
            G = torch.zeros((cap, self._Gbuf.shape[1]), dtype=self._Gbuf.dtype, device=self._Gbuf.device)
            G[:N0].copy_(self._Gbuf[:N0])
            self._Gbuf = G
        self._Gbuf[N0:N1].copy_(new)
        self.N, self.G = N1, self._Gbuf[:N1]
        return self.N

    def search(self, Qd, k, index_base=0):
        """Certified ChiSquare top-k: the fp32 VALU pass with its error bound; the queries it cannot
        certify are re-run with fp64 per-term arithmetic (ofr_chi2_knn_exact).  self.last_fallbacks
        = (uncertified after the fp32 pass, uncertified after the exact pass: near-ties at fp32 key
        resolution, 2^-23 relative).  k > 16: the exact any-k pass (search_deep)."""
        B = Qd.shape[0]
        if k > _lib.MAX_K:
            self.last_fallbacks = (0,)
            return search_deep(_lib.METRIC_CHISQUARE, Qd, self.dtype, self.G, self.dtype, self.nbins, self.denom, k,
                               index_base, workspace=self.ws)
        out_d = torch.empty((B, k), dtype=torch.float64, device=Qd.device)
        out_i = torch.empty((B, k), dtype=torch.int64, device=Qd.device)
        cert = torch.empty(B, dtype=torch.int32, device=Qd.device)
        lib = _lib.load()
        ws = self.ws.get(lib.ofr_chi2_workspace_bytes(B, self.N, k), Qd.device)
        call("ofr_chi2_knn", stream(), self.dtype, ptr(Qd), B, Qd.shape[1], ptr(self.G), self.N, self.G.shape[1],
             self.nbins, self.denom, k, index_base, ptr(out_d), ptr(out_i), ptr(ws), ws.numel(), ptr(cert))
        rows = open_rows(cert)
        counts = [int(rows.numel())]
        if rows.numel():
            sub = Qd.index_select(0, rows).contiguous()
            n = sub.shape[0]
            d2 = torch.empty((n, k), dtype=torch.float64, device=Qd.device)
            i2 = torch.empty((n, k), dtype=torch.int64, device=Qd.device)
            c2 = torch.empty(n, dtype=torch.int32, device=Qd.device)
            ws2 = self.ws.get(lib.ofr_chi2_workspace_bytes(n, self.N, k), Qd.device)
            call("ofr_chi2_knn_exact", stream(), self.dtype, ptr(sub), n, sub.shape[1], ptr(self.G), self.N,
                 self.G.shape[1], self.nbins, self.denom, k, index_base, ptr(d2), ptr(i2), ptr(ws2), ws2.numel(),
                 ptr(c2))
            out_d.index_copy_(0, rows, d2)
            out_i.index_copy_(0, rows, i2)
            counts.append(int((c2 == 0).sum()))
        self.last_fallbacks = tuple(counts)
        return out_d, out_i

    def query_rows(self, arr):
        """Host float query rows -> device rows of this gallery's element type; None for a counts
        gallery when the rows are not counts / denom."""
        if self.dtype != _lib.DT_F32:
            return self.counts_rows(arr)
        return f32_rows(np.asarray(arr, np.float64), ld=self.G.shape[1])


def search_deep(metric, Q, qdtype, G, gdtype, d, denom, k, index_base=0, workspace=None):
    """Any k (> 16 in practice): the reference's distance of every (query, row) pair in fp64 and the k
    smallest per query by (distance, row), NaN last (ofr_knn_deep; classifier.py:104-119, distance.py).
    Q [B][>= d], G [N][>= d] device rows of the given OFR dtypes (counts: value = count / denom).
    workspace: a Workspace to reuse (the gallery's own; its distance block can reach 2 GiB).
    Returns (fp64 [B][k], int64 [B][k]); entries past N are (+inf, -1)."""
    B, N = int(Q.shape[0]), int(G.shape[0]) if G is not None else 0
    out_d = torch.empty((B, k), dtype=torch.float64, device=Q.device)
    out_i = torch.empty((B, k), dtype=torch.int64, device=Q.device)
    ws = ((workspace or Workspace()).get(_lib.load().ofr_knn_deep_workspace_bytes(B, N), Q.device)
          if N else None)
    call("ofr_knn_deep", stream(), metric, ptr(Q), B, Q.shape[1], qdtype, ptr(G), N, G.shape[1] if N else d, gdtype,
         d, float(denom), int(k), index_base, ptr(out_d), ptr(out_i), ptr(ws), 0 if ws is None else ws.numel())
    return out_d, out_i


def topk_pack(d, i, bound=None):
    """(B x k) distances, indices and the per-query bound -> one [B][2k+1] fp64 block (ofr_topk_pack)."""
    B, k = d.shape
    out = torch.empty((B, 2 * k + 1), dtype=torch.float64, device=d.device)
    call("ofr_topk_pack", stream(), ptr(d.contiguous()), ptr(i.contiguous()),
         None if bound is None else ptr(bound.contiguous()), B, k, ptr(out))
    return out


def topk_merge_certify(lists, P, B, k, certify=True):
    """Gathered blocks [P][B][2k+1] -> (best k distances, indices, certificate int32 or None)
    (ofr_topk_merge_certify)."""
    out_d = torch.empty((B, k), dtype=torch.float64, device=lists.device)
    out_i = torch.empty((B, k), dtype=torch.int64, device=lists.device)
    cert = torch.empty(B, dtype=torch.int32, device=lists.device) if certify else None
    call("ofr_topk_merge_certify", stream(), ptr(lists.contiguous()), P, B, k, ptr(out_d), ptr(out_i), ptr(cert))
    return out_d, out_i, cert


def kth_bound(allb, P, B, k):
    """[P][B][k] ascending upper bounds -> [B] k-th smallest over the P*k (ofr_kth_bound)."""
    ub = torch.empty(B, dtype=torch.float64, device=allb.device)
    call("ofr_kth_bound", stream(), ptr(allb.contiguous()), P, B, k, ptr(ub))
    return ub


def open_rows(cert):
    """int32 certificate [B] -> int64 device indices of the uncertified queries, ascending
    (ofr_open_rows; one host read of their count)."""
    B = cert.shape[0]
    rows = torch.empty(max(B, 1), dtype=torch.int64, device=cert.device)
    cnt = torch.empty(1, dtype=torch.int32, device=cert.device)
    call("ofr_open_rows", stream(), ptr(cert.contiguous()), B, ptr(rows), ptr(cnt))
    return rows[:int(cnt.item())]


def topk_merge(in_d, in_i, P, kin, k):
    B = in_d.shape[0]
    out_d = torch.empty((B, k), dtype=torch.float64, device=in_d.device)
    out_i = torch.empty((B, k), dtype=torch.int64, device=in_d.device)
    call("ofr_topk_merge", stream(), ptr(in_d), ptr(in_i), B, P, kin, k, ptr(out_d), ptr(out_i))
    return out_d, out_i


# ---------------------------------------------------------------------------
# LBP  (lbp.py:80-130, feature.py:286-302)
# ---------------------------------------------------------------------------
def elbp_codes(imgs_u8, geom):
    """imgs: uint8 [n][H][W] device tensor; geom: lbp geometry tuple -> uint32 codes as int64 [n][dy][dx]."""
    (oy, ox), (by, bx), offs, wts = geom
    n, H, W = imgs_u8.shape
    dy, dx = H - by + 1, W - bx + 1
    out = torch.empty((n, max(dy, 0), max(dx, 0)), dtype=torch.int32, device=imgs_u8.device)
    offs32 = np.ascontiguousarray(offs, dtype=np.int32)
    w64 = np.ascontiguousarray(wts, dtype=np.float64)
    call("ofr_elbp_codes", stream(), ptr(imgs_u8), n, H, W, len(offs32), offs32.ctypes.data_as(_lib.c_vp),
         w64.ctypes.data_as(_lib.c_vp), oy, ox, by, bx, ptr(out))
    return out  # int32 storage of uint32 codes (reinterpret on host)


def elbp_hist(imgs_u8, geom, grid, count_bytes=None):
    """-> (counts device tensor [n][gr*gc][2^P] of uint8/int16/int32 storage, cell pixel count)."""
    (oy, ox), (by, bx), offs, wts = geom
    n, H, W = imgs_u8.shape
    P = len(offs)
    gr, gc = grid
    dy, dx = H - by + 1, W - bx + 1
    py = dy // gr if dy > 0 else 0
    px = dx // gc if dx > 0 else 0
    cell = py * px
    if count_bytes is None:
        count_bytes = 1 if cell <= 255 else (2 if cell <= 65535 else 4)
    tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[count_bytes]
    out = torch.empty((n, gr * gc, 1 << P), dtype=tdt, device=imgs_u8.device)
    offs32 = np.ascontiguousarray(offs, dtype=np.int32)
    w64 = np.ascontiguousarray(wts, dtype=np.float64)
    call("ofr_elbp_hist_geom", stream(), ptr(imgs_u8), n, H, W, P, offs32.ctypes.data_as(_lib.c_vp),
         w64.ctypes.data_as(_lib.c_vp), oy, ox, by, bx, gr, gc, ptr(out), count_bytes)
    return out, cell, count_bytes


# ---------------------------------------------------------------------------
# training products  (feature.py:91-94, 162-168, 229)
# ---------------------------------------------------------------------------
def gemm_f64(A, B, transA=False, transB=False, alpha=1.0):
    """op(A) @ op(B) in fp64 on the MFMA; A, B contiguous fp64 device tensors."""
    M = A.shape[1] if transA else A.shape[0]
    K = A.shape[0] if transA else A.shape[1]
    N = B.shape[0] if transB else B.shape[1]
    Kb = B.shape[1] if transB else B.shape[0]
    if K != Kb:
        raise ValueError(f"gemm_f64: inner dimensions {K} != {Kb}")
    C = torch.empty((M, N), dtype=torch.float64, device=A.device)
    call("ofr_gemm_f64", stream(), int(transA), int(transB), M, N, K, float(alpha), ptr(A), A.shape[1], ptr(B),
         B.shape[1], 0.0, ptr(C), N)
    return C


def _eig_call(name, mats, m):
    n = int(mats[0].shape[0])
    m = max(0, min(int(m), n))
    for A in mats:
        if A.dtype != torch.float64 or tuple(A.shape) != (n, n) or not A.is_contiguous():
            raise ValueError(f"{name}: needs contiguous square fp64 device matrices")
    lib = _lib.load()
    nbytes = lib.ofr_eig_workspace_bytes(n, m)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=mats[0].device)
    evals = torch.empty(max(m, 1), dtype=torch.float64, device=mats[0].device)
    evecs = torch.empty((n, max(m, 1)), dtype=torch.float64, device=mats[0].device)
    call(name, stream(), n, *[ptr(A) for A in mats], m, ptr(evals), ptr(evecs), evecs.shape[1], ptr(ws), nbytes)
    return evals[:m], evecs[:, :m]


def eigh_desc_f64(A, m, overwrite=False):
    """The m largest eigenpairs of a symmetric fp64 device matrix, descending, eigenvectors as the
    columns of a device [n][m] (rocSOLVER dsyevd, ofr_eigh_f64)."""
    return _eig_call("ofr_eigh_f64", [A if overwrite else A.clone()], m)


def sygv_desc_f64(Sb, Sw, m, overwrite=False):
    """The m largest eigenpairs of Sb v = lambda Sw v (Sw positive definite), descending, columns at
    unit 2-norm (rocSOLVER dsygvd, ofr_sygv_f64).  OfrError(code E_NUMERIC) when Sw is not
    positive definite."""
    return _eig_call("ofr_sygv_f64", [Sb if overwrite else Sb.clone(), Sw if overwrite else Sw.clone()], m)


def col_mean_u8(Xd, D):
    mean = torch.empty(D, dtype=torch.float64, device=Xd.device)
    call("ofr_col_mean_u8", stream(), ptr(Xd), Xd.shape[0], D, Xd.shape[1], ptr(mean))
    return mean


def col_mean_f64(F):
    mean = torch.empty(F.shape[1], dtype=torch.float64, device=F.device)
    call("ofr_col_mean_f64", stream(), ptr(F), F.shape[0], F.shape[1], F.shape[1], ptr(mean))
    return mean


def center_u8_f64(Xd, D, mean):
    out = torch.empty((Xd.shape[0], D), dtype=torch.float64, device=Xd.device)
    call("ofr_center_u8_f64", stream(), ptr(Xd), Xd.shape[0], D, Xd.shape[1], ptr(mean), ptr(out), D)
    return out


def center_f64(X, mean):
    out = torch.empty_like(X)
    call("ofr_sub_mean_f64", stream(), ptr(X), X.shape[0], X.shape[1], X.shape[1], ptr(mean), ptr(out), X.shape[1])
    return out


def normalize_columns(U):
    U = U.contiguous()
    call("ofr_normalize_cols_f64", stream(), ptr(U), U.shape[0], U.shape[1], U.shape[1])
    return U


def counts_numpy(counts, count_bytes):
    """Device count tensor (uint8 / int16 / int32 storage) -> unsigned numpy array."""
    a = counts.cpu().numpy()
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32}[count_bytes])


def class_center_f64(F, y):
    """F: fp64 [N][d] device; y: int labels 0..c-1 (host) -> (means [c][d], Fc [N][d], Mc, Mc_n [c][d])."""
    y = np.asarray(y).astype(np.int64)
    N, d = F.shape
    c = int(y.max()) + 1 if len(y) else 0
    perm = np.argsort(y, kind="stable")
    counts = np.bincount(y, minlength=c)
    offsets = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    perm_d = torch.from_numpy(perm.astype(np.int64)).to(F.device)
    off_d = torch.from_numpy(offsets).to(F.device)
    total = col_mean_f64(F)
    means = torch.empty((c, d), dtype=torch.float64, device=F.device)
    Fc = torch.empty((N, d), dtype=torch.float64, device=F.device)
    Mc = torch.empty((c, d), dtype=torch.float64, device=F.device)
    Mc_n = torch.empty((c, d), dtype=torch.float64, device=F.device)
    call("ofr_class_center_f64", stream(), ptr(F), N, d, F.shape[1], ptr(perm_d), ptr(off_d), c, ptr(total),
         ptr(means), ptr(Fc), ptr(Mc), ptr(Mc_n))
    return total, means, Fc, Mc, Mc_n
