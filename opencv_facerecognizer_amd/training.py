"""Device pipeline of Fisherfaces / PCA training on uint8 faces.

Reference: ``Fisherfaces.compute`` (feature.py:211-235) = ``PCA(n - c)`` (feature.py:83-108:
centre, ``svd``, keep the leading n - c left singular vectors) chained into ``LDA(c - 1)``
(feature.py:147-182: class scatter Sw, Sb; ``eig(inv(Sw) Sb)``; float32 eigenvectors), then
W = P . L (feature.py:229) and the features W^T x (feature.py:231-235).

What the pixels being integers buys (csrc/ofr_gram.hip): with x' = x - 128 every Gram or scatter
product of the data is an EXACT int8-MFMA integer matrix plus centring terms made of exact column
/ class sums; the reference forms the same matrices from float64 ``X - mean`` whose elements are
already rounded.  Three regimes, by what PCA keeps (k = its number of components, n images of
D pixels, c classes):

* ``pixel``  k = D (n - c >= D and n >= D; BASELINE configs[4]): P is a square orthogonal matrix,
  i.e. PCA only rotates the space, and LDA's eigenproblem is similar to the same problem in pixel
  space: inv(P^T Sw P) P^T Sb P = P^T inv(Sw) Sb P, so L = P^T V and W = P L = V.  W is computed
  directly from the pixel-space Sw = X'^T X' - sum_i s_i s_i^T / n_i and
  Sb = sum_i s_i s_i^T / n_i - s s^T / n (s_i: class sums of x'), no SVD and no PCA projection.
  (The reference rounds L to float32 in PCA coordinates, which has no pixel-space equivalent: W
  differs from it by that rounding, <= 2^-24 relative per element of L.)
* ``gram``   n <= D (the bundled model, small training sets): the n x n Gram of the centred
  images, G = X' X'^T - (r 1^T + 1 r^T) / n + (s.s) / n^2 (r = X' s), device ``eigh`` (as the
  reference's ``svd``: sigma^2 = eigenvalues); PCA features are V_k Sigma_k (= U_k^T (x - mean)
  exactly), LDA runs on them, and W = U_k L = XC^T (V_k Sigma_k^-1 L) -- one exact uint8 x fp64
  product on the int8-slice projection engine, minus the rank-one mean term.
* ``cov``    n > D and k < D: the D x D covariance X'^T X' - s s^T / n, device ``eigh``, P = its
  leading k eigenvectors; features XC P on the projection engine (shift mean^T P); LDA on them;
  W = P L on the fp64 MFMA.

Multi-GPU: every exact piece is a sum over images, so rank r computes them over its
own rows and one all-reduce (sum) combines them -- exactly, in any order, because they are
integer-valued below 2^53 (``parallel.allreduce_exact``): the trained model does not depend on
the number of GPUs.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _device
from ._lib import call, ptr, stream


def finite(stage, *ts):
    """Raise OfrError naming the stage when a device intermediate holds a NaN / inf (one reduction
    and one host read per tensor: training only)."""
    from ._lib import OfrError
    for t in ts:
        if not bool(torch.isfinite(t).all()):
            raise OfrError(f"Fisherfaces training: non-finite values after {stage}")
    return ts[0] if len(ts) == 1 else ts


def _i64(t, device):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(t, dtype=np.int64))).to(device)


# ---------------------------------------------------------------------------
# exact pieces
# ---------------------------------------------------------------------------
def padded(Xd, n, D, transpose=False):
    """uint8 rows [n][>= D] -> [rows][ld] (X or X^T), ld % 128 == 0, pad columns 128 (x' = 0)."""
    rows, K = (D, n) if transpose else (n, D)
    ld = _device.round_up(max(K, 1), 128)
    out = torch.empty((rows, ld), dtype=torch.uint8, device=Xd.device)
    call("ofr_pad_u8", stream(), ptr(Xd), n, D, Xd.shape[1], int(transpose), ptr(out), ld)
    return out, K


def gram(Xp, R, K):
    """C [R][R] = X' X'^T over the K columns of the padded uint8 rows Xp (exact)."""
    C = torch.empty((R, R), dtype=torch.float64, device=Xp.device)
    call("ofr_gram_u8", stream(), ptr(Xp), R, K, Xp.shape[1], ptr(C), R)
    return C


class Layout:
    """Rows grouped by class label (labels must be 0..c-1, feature.py:164-165 iterates range(c))."""

    def __init__(self, y, device, c=None):
        """c: the number of classes when this is one shard of a larger set (its labels may miss some)."""
        y = np.asarray(y).astype(np.int64).reshape(-1)
        if c is None:
            c = len(np.unique(y))
            if len(y) and (y.min() < 0 or y.max() != c - 1):
                raise ValueError("LDA: labels must be the integers 0..c-1 (feature.py:164-165 iterates range(c))")
        elif len(y) and (y.min() < 0 or y.max() >= c):
            raise ValueError("labels must lie in 0..c-1")
        self.y, self.c, self.n = y, c, len(y)
        self.counts = np.bincount(y, minlength=c)
        perm = np.argsort(y, kind="stable")
        self.perm = _i64(perm, device)
        self.offsets = _i64(np.concatenate([[0], np.cumsum(self.counts)]), device)
        self.all_perm = _i64(np.arange(len(y)), device)
        self.all_offsets = _i64([0, len(y)], device)


def class_sums(Xd, D, lay, shift=128, means=False):
    """Per-class column sums of x - shift [c][D] (exact) and, optionally, the class means."""
    S = torch.empty((lay.c, D), dtype=torch.float64, device=Xd.device)
    M = torch.empty_like(S) if means else None
    call("ofr_class_sums_u8", stream(), ptr(Xd), D, Xd.shape[1], ptr(lay.perm), ptr(lay.offsets), lay.c, shift,
         ptr(S), ptr(M))
    return S, M


def column_sums(Xd, D, lay, shift=128):
    """Column sums of x - shift over all rows [D] (exact) and the column means (rounded once)."""
    s = torch.empty((1, D), dtype=torch.float64, device=Xd.device)
    m = torch.empty_like(s)
    call("ofr_class_sums_u8", stream(), ptr(Xd), D, Xd.shape[1], ptr(lay.all_perm), ptr(lay.all_offsets), 1, shift,
         ptr(s), ptr(m))
    return s.reshape(-1), m.reshape(-1)


def pixel_pieces(Xd, D, lay):
    """The additive exact pieces of pixel-space statistics over this process's rows:
    G = X'^T X' [D][D], class sums of x' [c][D], column sums of x' [D] (all integer-valued)."""
    Xt, _ = padded(Xd, lay.n, D, transpose=True)
    G = gram(Xt, D, lay.n)
    del Xt
    S, _ = class_sums(Xd, D, lay)
    s, _ = column_sums(Xd, D, lay)
    return {"G": G, "S": S, "s": s}


def pixel_scatter(pieces, counts, n):
    """Sw, Sb [D][D] (feature.py:160-168 over pixels) from the exact pieces:
    T = sum_i m_i s_i^T (m_i = s_i / n_i, rounded once), Sw = G - T, Sb = T - s s^T / n."""
    G, S, s = pieces["G"], pieces["S"], pieces["s"]
    D = G.shape[0]
    nd = torch.from_numpy(np.asarray(counts, np.float64)).to(G.device)
    M = torch.empty_like(S)
    call("ofr_row_div_f64", stream(), ptr(S), S.shape[0], D, D, ptr(nd), ptr(M), D)      # m_i = s_i / n_i
    T = _device.gemm_f64(M, S, transA=True)
    Sw = torch.empty_like(G)
    Sb = torch.empty_like(G)
    call("ofr_scatter_combine_f64", stream(), ptr(G), ptr(T), ptr(s), 1.0 / n, D, D, ptr(Sw), ptr(Sb))
    return Sw, Sb


def covariance(pieces, n):
    """XC^T XC [D][D] = X'^T X' - s s^T / n (PCA of n > D images, feature.py:91-94)."""
    G, s = pieces["G"], pieces["s"]
    D = G.shape[0]
    C = torch.empty_like(G)
    call("ofr_scatter_combine_f64", stream(), ptr(G), ptr(G), ptr(s), 1.0 / n, D, D, None, ptr(C))
    return C


def centred_gram(Xd, D, lay):
    """XC XC^T [n][n] of n images (PCA of n <= D images): X' X'^T - (r 1^T + 1 r^T) / n + s.s / n^2."""
    n = lay.n
    Xp, _ = padded(Xd, n, D)
    G = gram(Xp, n, D)
    del Xp
    s, _ = column_sums(Xd, D, lay)
    r = torch.empty(n, dtype=torch.float64, device=Xd.device)
    call("ofr_row_dot_u8", stream(), ptr(Xd), n, D, Xd.shape[1], ptr(s), ptr(r))
    sh = s.cpu().numpy()
    call("ofr_center_gram_f64", stream(), ptr(G), n, n, ptr(r), -1.0 / n, float(sh @ sh) / (float(n) * n))
    return G


def eigh_desc(C, m):
    """The m largest eigenpairs of a symmetric device matrix, descending (the reference's svd order),
    on the device (``ofr_eigh_f64``, rocSOLVER dsyevd; C is overwritten).  Returns device tensors
    (evals [m], V [n][m])."""
    return _device.eigh_desc_f64(C, m, overwrite=True)


def mean_image(Xd, D, lay):
    """Column means of the uint8 images, sum / n rounded once (= numpy's mean, feature.py:91)."""
    return column_sums(Xd, D, lay, shift=0)[1]


def feature_scatter(Fd, y):
    """Sw, Sb [k][k] (feature.py:160-168) of fp64 device features [n][k] on the fp64 MFMA."""
    _, _, Fc, Mc, Mc_n = _device.class_center_f64(Fd, y)
    return _device.gemm_f64(Fc, Fc, transA=True), _device.gemm_f64(Mc, Mc_n, transA=True)


def feature_scatter_sharded(Fd, lay, counts, n, allreduce):
    """Sw, Sb [k][k] (feature.py:160-168) of fp64 features [n_r][k] sharded over ranks: the class sums of
    every rank's rows are all-reduced into the global class means (``allreduce``: sums a list of
    device tensors in place over the ranks), each rank centres its own rows on them and the
    Fc^T Fc products are all-reduced into Sw; Sb = Mc^T (n_i Mc) from the global means, the same on
    every rank.  counts: the global class sizes (device fp64 [c]), n their sum.  Equal to
    feature_scatter of all the rows up to the order of the fp64 sums."""
    k, c, dev_ = Fd.shape[1], lay.c, Fd.device
    sums = torch.empty((c, k), dtype=torch.float64, device=dev_)
    call("ofr_class_sums_f64", stream(), ptr(Fd), k, Fd.shape[1], ptr(lay.perm), ptr(lay.offsets), c, ptr(sums))
    allreduce([sums])
    tot = _col_sums_f64(sums).reshape(1, k).contiguous()
    nd = torch.tensor([float(n)], dtype=torch.float64, device=dev_)
    total = torch.empty_like(tot)
    call("ofr_row_div_f64", stream(), ptr(tot), 1, k, k, ptr(nd), ptr(total), k)
    means, Mc, Mc_n = (torch.empty((c, k), dtype=torch.float64, device=dev_) for _ in range(3))
    call("ofr_class_between_f64", stream(), ptr(sums), ptr(counts), c, k, ptr(total), ptr(means), ptr(Mc), ptr(Mc_n))
    Fc = torch.empty((Fd.shape[0], k), dtype=torch.float64, device=dev_)
    call("ofr_class_sub_f64", stream(), ptr(Fd), Fd.shape[0], k, Fd.shape[1], ptr(lay.perm), ptr(lay.offsets), c,
         ptr(means), ptr(Fc))
    Sw = _device.gemm_f64(Fc, Fc, transA=True)
    del Fc
    allreduce([Sw])
    return Sw, _device.gemm_f64(Mc, Mc_n, transA=True)


def fisher_gram(Xd, D, lay, y, k, m):
    """The gram regime of Fisherfaces.compute (n <= D): PCA(k) through the n x n Gram of the centred
    faces, LDA(m) on its features V_k Sigma_k, W = XC^T (V_k Sigma_k^-1 L) -> (LDA eigenvalues, W
    [D][m] device fp64)."""
    from .facerec.feature import lda_eigen
    lam, V = finite("eigh_desc", *eigh_desc(finite("centred_gram", centred_gram(Xd, D, lay)), k))
    sig = lam.clamp_min(0.0).sqrt()
    Sw, Sb = finite("feature_scatter", *feature_scatter((V * sig).contiguous(), y))
    evals, L = lda_eigen(Sw, Sb, m)
    L32 = _device.f64_dev(np.asarray(L, dtype=np.float32).astype(np.float64))   # feature.py:176
    inv = torch.where(sig > 0, 1.0 / sig, torch.zeros_like(sig))
    M = _device.gemm_f64((V * inv).contiguous(), L32)                       # V_k Sigma^-1 L
    return evals, xct_times(Xd, D, lay, M, mean_image(Xd, D, lay))


def xct_times(Xd, D, lay, M, mean):
    """XC^T M [D][m] for uint8 images X [n][D] and an fp64 device matrix M [n][m]:
    sum_n x_n[p] M[n][j] exactly on the int8-slice projection engine (X^T as the face rows, M as
    the weights), minus the rank-one mean term mean[p] * colsum(M)[j] in fp64."""
    n = lay.n
    Xt, _ = padded(Xd, n, D, transpose=True)           # [D][round_up(n, 128)] uint8
    Pm = _device.Projection(Wt_device=M.t().contiguous(), D=n)
    Y = Pm.project(Xt, f64=True)                        # [D][m]
    del Xt, Pm
    colsum = _col_sums_f64(M)
    call("ofr_rank1_f64", stream(), ptr(Y), D, Y.shape[1], Y.shape[1], ptr(mean), ptr(colsum), -1.0)
    return Y


def _col_sums_f64(M):
    ones = torch.ones((1, M.shape[0]), dtype=torch.float64, device=M.device)
    return _device.gemm_f64(ones, M).reshape(-1)
