"""Feature extraction (reference ``src/ocvfacerec/facerec/feature.py``).

Same classes, constructor arguments, attributes (pickled state), return types
and errors as the reference:

* ``PCA`` (feature.py:78-139): ``_num_components``, ``_mean`` (np.matrix D x 1),
  ``_eigenvectors`` (np.matrix D x k), ``_eigenvalues`` (k,).
* ``LDA`` (feature.py:142-203): float32 ``_eigenvectors`` / ``_eigenvalues``.
* ``Fisherfaces`` (feature.py:206-260): ``_eigenvectors`` W (np.matrix D x d,
  float64), ``_eigenvalues``, ``_num_components``; ``extract`` is W^T x with
  NO mean subtraction (feature.py:237-242).
* ``SpatialHistogram`` (feature.py:266-305).

What moves to the GPU: the centring and Gram/covariance products of PCA
(the SVD of the centred data, feature.py:91-94, becomes an exact int8-MFMA
Gram matrix of the uint8 faces + a device ``eigh``, see training.py), the
scatter matrices of LDA (feature.py:160-168), the LDA eigenproblem (:170: the
reference's host ``inv`` + ``eig`` for small orders, the symmetric-definite
pencil on the device above ``AUTO_DEVICE_MIN``, see ``lda_eigen``), W = P.L
(:229), every projection loop (:104-108, :178-182, :231-235 and ``extract``)
on the exact int8-slice projection engine, and the LBP + per-cell histograms
(:286-302).

Eigenvector signs: an eigensolver may return any column sign; distances and
the Fisherfaces W are invariant to PCA column signs, and the LDA/Fisherfaces
column signs are as arbitrary in the reference as here.
"""
from __future__ import annotations

import os
import warnings

import numpy as np
import torch

from .. import _device


class AbstractFeature(object):
    """feature.py:38-52."""

    def compute(self, X, y):
        raise NotImplementedError("Every AbstractFeature must implement the compute method.")

    def extract(self, X):
        raise NotImplementedError("Every AbstractFeature must implement the extract method.")

    def save(self):
        raise NotImplementedError("Not implemented yet (TODO).")

    def load(self):
        raise NotImplementedError("Not implemented yet (TODO).")

    def __repr__(self):
        return "AbstractFeature"


class Identity(AbstractFeature):
    """feature.py:55-71 (forwards the data)."""

    def __init__(self):
        AbstractFeature.__init__(self)

    def compute(self, X, y):
        return X

    def extract(self, X):
        return X

    def __repr__(self):
        return "Identity"


from .operators import ChainOperator  # noqa: E402  (feature.py:74-75 import order)
from .util import as_column_matrix  # noqa: E402,F401


def _stack_rows(X):
    """List of equally-shaped items -> 2-D host array [N][D] (the rows of the reference's column matrix)."""
    return np.stack([np.asarray(x).reshape(-1) for x in X])


def _device_rows(X):
    """Items -> (device rows, D, kind): uint8 images use the u8 layout, everything else fp64."""
    if isinstance(X, (list, tuple)):
        Xd = _device.upload_u8_items(X)             # a host list of uint8 faces: pinned, overlapped upload
        if Xd is not None:
            return Xd, int(np.asarray(X[0]).size), "u8"
    A = _stack_rows(X)
    if A.dtype == np.uint8:
        return _device.u8_rows(A), A.shape[1], "u8"
    return _device.f64_dev(A.astype(np.float64)), A.shape[1], "f64"


class _DeviceProjMixin:
    """Cached device projection (derived state; dropped from pickles).

    uint8 inputs (faces) use the exact int8-slice MFMA kernel; any other input
    dtype uses the fp64 MFMA GEMM.  Both give fp64-accurate W^T x - shift.
    """

    def _proj_matrix(self):  # -> (W D x d, own shift (fp64 [d] host array) or None)
        raise NotImplementedError

    def _proj(self):
        W, shift = self._proj_matrix()
        src = self._eigenvectors
        cache = self.__dict__.get("_dev_proj")
        if cache is None or cache[0] is not src or cache[1] is not shift:
            P = _device.Projection(W)
            P.W_host = W
            P.own_shift = None if shift is None else _device.f64_dev(np.asarray(shift, np.float64).reshape(-1))
            cache = (src, shift, P)   # holds src/shift so that the identity check stays valid
            self.__dict__["_dev_proj"] = cache
        return cache[2]

    def _prime_proj(self, W_dev):
        """Seed the projection cache from the device copy of W [D][d] fp64 that training just
        produced (the host W in self._eigenvectors is its copy): no upload of W back to the device."""
        P = _device.Projection(Wt_device=W_dev.t().contiguous(), D=int(W_dev.shape[0]))
        P.W_host = None
        P._W64 = W_dev
        P.own_shift = None
        self.__dict__["_dev_proj"] = (self._eigenvectors, None, P)

    @staticmethod
    def _w64(P):
        """fp64 W on the device (the GEMM path of non-uint8 inputs), uploaded on first use."""
        if getattr(P, "_W64", None) is None:
            P._W64 = _device.f64_dev(np.asarray(P.W_host, np.float64))
        return P._W64

    def _shift(self, P, extra):
        """Own shift (PCA mean term) plus an extra centring shift (search layout), fp64 device or None."""
        if P.own_shift is None:
            return extra
        return P.own_shift if extra is None else P.own_shift + extra

    def project_device(self, X, shift64=None, f64=False, ld=None):
        """Batch of items -> (W^T x - own shift - shift64): fp32 search rows [B][ldy] or fp64 [B][d]."""
        P = self._proj()
        sh = self._shift(P, shift64)
        if hasattr(X, "data_ptr"):      # device uint8 faces [B][H][W] / [B][D] (e.g. ingest.faces): no host trip
            if X.dtype != torch.uint8:
                raise TypeError("device face batches must be uint8")
            return P.project(_device.u8_rows(X), shift64=sh, f64=f64)
        if isinstance(X, (list, tuple)):
            Xd = _device.upload_u8_items(X)         # a host list of uint8 faces: pinned, overlapped upload
            if Xd is not None:
                return P.project(Xd, shift64=sh, f64=f64)
        A = X if isinstance(X, np.ndarray) and X.ndim == 2 and not isinstance(X, np.matrix) else _stack_rows(X)
        if A.dtype == np.uint8:
            return P.project(_device.u8_rows(A), shift64=sh, f64=f64)
        Y = _device.gemm_f64(_device.f64_dev(A.astype(np.float64)), self._w64(P))
        if sh is not None:
            Y = _device.center_f64(Y, sh)
        return Y if f64 else _device.center_round(Y, None, P.ldy)

    def _project_host(self, X):
        """Batch -> list of (d,1) float64 np.matrix features (reference return type)."""
        Y = self.project_device(X, f64=True).cpu().numpy()
        return [np.asmatrix(r.reshape(-1, 1)) for r in Y]

    def __getstate__(self):
        st = dict(self.__dict__)
        for key in ("_dev_proj", "_dev_features", "_regime"):   # derived state, never pickled
            st.pop(key, None)
        return st


class PCA(_DeviceProjMixin, AbstractFeature):
    """feature.py:78-139."""

    def __init__(self, num_components=0):
        AbstractFeature.__init__(self)
        self._num_components = num_components

    def compute(self, X, y):
        Xd, D, kind = _device_rows(X)
        y = np.asarray(y)
        n = Xd.shape[0]
        if self._num_components <= 0 or (self._num_components > n - 1):     # feature.py:88-89
            self._num_components = n - 1
        # centre the data on the device (feature.py:91-92)
        if kind == "u8":
            mean = _device.col_mean_u8(Xd, D)
            XC = _device.center_u8_f64(Xd, D, mean)
        else:
            mean = _device.col_mean_f64(Xd)
            XC = _device.center_f64(Xd, mean)
        # economy SVD of the D x N centred matrix (feature.py:94) via the smaller Gram matrix
        if n <= D:
            G = _device.gemm_f64(XC, XC, transB=True).cpu().numpy()            # N x N = XC XC^T (rows)
            lam, V = np.linalg.eigh(G)
            order = np.argsort(-lam, kind="stable")
            lam, V = lam[order], V[:, order]
            U = _device.gemm_f64(XC, _device.f64_dev(V), transA=True)          # D x N, columns ~ sigma_i u_i
            U = _device.normalize_columns(U)
        else:
            C = _device.gemm_f64(XC, XC, transA=True).cpu().numpy()            # D x D covariance * N
            lam, V = np.linalg.eigh(C)
            order = np.argsort(-lam, kind="stable")
            lam, V = lam[order], V[:, order]
            U = _device.f64_dev(V)
        k = min(self._num_components, U.shape[1])
        lam = np.maximum(lam[:k], 0.0)
        Ud = U[:, :k].contiguous()
        self._eigenvectors = np.asmatrix(Ud.cpu().numpy())                      # feature.py:99
        self._eigenvalues = lam / n                                              # feature.py:102 (sigma^2 / N)
        self._mean = np.asmatrix(mean.cpu().numpy().reshape(-1, 1))              # feature.py:91
        # features = U^T (x - mean) for every sample (feature.py:104-108): XC @ U on the MFMA
        F = _device.gemm_f64(XC, Ud).cpu().numpy()
        return [np.asmatrix(f.reshape(-1, 1)) for f in F]

    def extract(self, X):
        """feature.py:110-112."""
        return self._project_host([np.asarray(X).reshape(-1)])[0]

    def project(self, X):
        """feature.py:114-116: U^T (X - mean) for a column (D,1)."""
        return self._project_host([np.asarray(X).reshape(-1)])[0]

    def _proj_matrix(self):
        W = np.asarray(self._eigenvectors)
        shift = self.__dict__.get("_shift_cache")
        if shift is None or shift[0] is not self._mean or shift[1] is not self._eigenvectors:
            mu = _device.f64_dev(np.asarray(self._mean).reshape(-1, 1))
            s = _device.gemm_f64(_device.f64_dev(W), mu, transA=True).cpu().numpy().reshape(-1)   # U^T mu (fp64)
            shift = (self._mean, self._eigenvectors, s)
            self.__dict__["_shift_cache"] = shift
        return W, shift[2]

    def reconstruct(self, X):
        return np.dot(self._eigenvectors, X) + self._mean

    def __getstate__(self):
        st = _DeviceProjMixin.__getstate__(self)
        st.pop("_shift_cache", None)
        return st

    @property
    def num_components(self):
        return self._num_components

    @property
    def eigenvalues(self):
        return self._eigenvalues

    @property
    def eigenvectors(self):
        return self._eigenvectors

    @property
    def mean(self):
        return self._mean

    def __repr__(self):
        return "PCA (num_components=%d)" % (self._num_components)


# "auto": matrices up to this order keep the reference's own host inv + eig (well under a second);
# larger ones go to the device pencil solver (configs[4], d = 10,000: 2.1 s against minutes of eig)
AUTO_DEVICE_MIN = 1024


def lda_eigen(Sw, Sb, num_components, solver=None, device_out=False):
    """Leading eigenpairs of inv(Sw) Sb, sorted by eigenvalue (feature.py:170-176).

    Sw, Sb: float64 host arrays or device tensors.  solver (or OFR_LDA_SOLVER):
    * "eig": exactly the reference's ``np.linalg.eig(np.linalg.inv(Sw) * Sb)``, real parts, descending;
    * "eigh": the symmetric-definite pencil Sb v = lambda Sw v on host LAPACK (sygvx for a few of
      the largest, sygvd when most are kept);
    * "device": the same pencil on the device (rocSOLVER dsygvd, ``ofr_sygv_f64``);
    * "auto" (default): "eig" up to order AUTO_DEVICE_MIN, "device" above.
    The pencil solvers scale columns to unit 2-norm like eig's -- the same eigenpairs up to
    column sign for distinct eigenvalues, in O(d^3) symmetric work instead of a general eig of a
    d x d matrix (minutes at d = 10000) -- and fall back to "eig" when Sw is not positive
    definite.  Returns (float64 (m,), float64 (d, m)) host arrays; with device_out the eigenvectors
    come back as a device tensor (no round trip when the device solver ran).
    """
    solver = solver or os.environ.get("OFR_LDA_SOLVER", "auto")
    if solver not in ("eig", "eigh", "device", "auto"):
        raise ValueError("OFR_LDA_SOLVER must be 'eig', 'eigh', 'device' or 'auto'")
    n = Sw.shape[0]
    m = max(0, min(int(num_components), n))
    if solver == "auto":
        solver = "device" if n > AUTO_DEVICE_MIN else "eig"
    if solver == "device" and m > 0:
        from .._lib import E_NUMERIC, OfrError
        Swd = Sw if isinstance(Sw, torch.Tensor) else _device.f64_dev(np.ascontiguousarray(Sw, np.float64))
        Sbd = Sb if isinstance(Sb, torch.Tensor) else _device.f64_dev(np.ascontiguousarray(Sb, np.float64))
        try:
            lam, V = _device.sygv_desc_f64(Sbd.contiguous(), Swd.contiguous(), m)
        except OfrError as e:
            if e.code != E_NUMERIC:
                raise
            warnings.warn("LDA: Sw is not positive definite (%s); using the general eig" % e)
        else:
            return lam.cpu().numpy(), (V.contiguous() if device_out else V.cpu().numpy())
    if isinstance(Sw, torch.Tensor):
        Sw, Sb = Sw.cpu().numpy(), Sb.cpu().numpy()
    if solver == "eigh" and m > 0:
        import scipy.linalg
        try:
            if 4 * m < n:   # a few eigenpairs: bisection + inverse iteration on the reduced problem
                lam, V = scipy.linalg.eigh(Sb, Sw, subset_by_index=[n - m, n - 1], driver="gvx")
            else:           # most of them: divide and conquer, all pairs
                lam, V = scipy.linalg.eigh(Sb, Sw, driver="gvd")
        except (np.linalg.LinAlgError, ValueError) as e:
            warnings.warn("LDA: Sw is not positive definite (%s); using the general eig" % e)
        else:
            order = np.argsort(-lam, kind="stable")[:m]
            V = V[:, order]
            V = V / np.linalg.norm(V, axis=0)
            return lam[order], (_device.f64_dev(np.ascontiguousarray(V)) if device_out else V)
    try:
        iSw = None if _numerically_singular(Sw) else np.linalg.inv(Sw)
    except np.linalg.LinAlgError:
        iSw = None
    if iSw is None:
        lam, V = _lda_singular_sw(Sw, Sb, m)
    else:
        evals, evecs = np.linalg.eig(iSw @ Sb)
        idx = np.argsort(-evals.real)
        lam, V = evals[idx][:m].real, evecs[:, idx][:, :m].real
    return lam, (_device.f64_dev(np.ascontiguousarray(V)) if device_out else V)


def _numerically_singular(Sw):
    """sigma_min(Sw) <= 16 n eps sigma_max(Sw): inv(Sw) is then rounding noise (2-norm condition
    beyond 1 / (16 n eps))."""
    sv = np.linalg.svd(np.asarray(Sw, np.float64), compute_uv=False)
    return sv.size > 0 and not (sv[-1] > 16 * sv.size * np.finfo(np.float64).eps * sv[0])


def _lda_singular_sw(Sw, Sb, m):
    """feature.py:170 when Sw is singular to working precision (``_numerically_singular``, or inv(Sw)
    meets an exactly zero pivot).

    Sw is singular whenever the within-class deviations span fewer than the PCA(n - c) dimensions
    it lives in -- e.g. two identical images in one class: the bundled data set holds one such pair
    (steve_crop0.jpg == steve_crop5.jpg), so the reference's own inv(Sw) there inverts rounding noise
    (its last LU pivot is ~1 ulp of the matrix): its non-dominant columns are set by that noise, and
    whether the noise is exactly zero (inv raises) depends on the last bits of the PCA features.  The reference's result with a vanishing POSITIVE pivot is
    the generalized problem Sb v = lambda Sw v: the null directions of Sw come first with an
    infinite eigenvalue, the rest are the finite generalized eigenpairs -- the same columns the
    reference's inv + eig converge to.  Solved by QZ (scipy.linalg.eig(Sb, Sw), LAPACK dggev);
    |beta| below 1e3 n eps ||Sw|| counts as zero (infinite eigenvalue, ranked first).  Columns at
    unit 2-norm like numpy's eig."""
    import scipy.linalg
    Sw = np.asarray(Sw, np.float64)
    Sb = np.asarray(Sb, np.float64)
    n = Sw.shape[0]
    (alpha, beta), V = scipy.linalg.eig(Sb, Sw, homogeneous_eigvals=True)
    tol = 1e3 * n * np.finfo(np.float64).eps * max(np.linalg.norm(Sw), np.finfo(np.float64).tiny)
    inf = np.abs(beta) <= tol
    with np.errstate(divide="ignore", invalid="ignore"):
        lam = np.where(inf, np.inf, (alpha / np.where(inf, 1.0, beta)).real)
    idx = np.argsort(-lam, kind="stable")[:m]
    V = V[:, idx].real
    nrm = np.linalg.norm(V, axis=0)
    V = V / np.where(nrm > 0, nrm, 1.0)
    warnings.warn("LDA: Sw is singular to working precision (feature.py:170); %d null direction(s) of Sw ranked "
                  "first (generalized eigenproblem, QZ)" % int(inf.sum()))
    return lam[idx], V


class LDA(_DeviceProjMixin, AbstractFeature):
    """feature.py:142-203."""

    def __init__(self, num_components=0):
        AbstractFeature.__init__(self)
        self._num_components = num_components

    @staticmethod
    def scatter(X, y):
        """Sw, Sb (float64 host arrays) of the items X with labels y (feature.py:160-168), on the device."""
        F = _device.f64_dev(_stack_rows(X).astype(np.float64))
        y = np.asarray(y)
        c = len(np.unique(y))
        if len(y) and (y.min() < 0 or y.max() != c - 1):
            raise ValueError("LDA: labels must be the integers 0..c-1 (feature.py:164-165 iterates range(c))")
        total, means, Fc, Mc, Mc_n = _device.class_center_f64(F, y)
        Sw = _device.gemm_f64(Fc, Fc, transA=True)           # sum_i (Xi - mi)(Xi - mi)^T
        Sb = _device.gemm_f64(Mc, Mc_n, transA=True)         # sum_i n_i (mi - m)(mi - m)^T
        return Sw.cpu().numpy(), Sb.cpu().numpy(), F

    def compute(self, X, y):
        y = np.asarray(y)
        c = len(np.unique(y))
        if self._num_components <= 0:                          # feature.py:155-158
            self._num_components = c - 1
        elif self._num_components > (c - 1):
            self._num_components = c - 1
        Sw, Sb, F = self.scatter(X, y)
        # eigenvalue problem of inv(Sw) Sb (feature.py:170-176), host LAPACK
        evals, evecs = lda_eigen(Sw, Sb, self._num_components)
        self._eigenvalues = np.array(evals, dtype=np.float32, copy=True)
        self._eigenvectors = np.matrix(evecs, dtype=np.float32, copy=True)
        # features = L^T x (feature.py:178-182) on the MFMA
        L = _device.f64_dev(np.asarray(self._eigenvectors, dtype=np.float64))
        Y = _device.gemm_f64(F, L).cpu().numpy()
        return [np.asmatrix(r.reshape(-1, 1)) for r in Y]

    def extract(self, X):
        return self.project(X)

    def project(self, X):
        """feature.py:184-185."""
        return self._project_host([np.asarray(X).reshape(-1)])[0]

    def _proj_matrix(self):
        return np.asarray(self._eigenvectors, dtype=np.float64), None

    def reconstruct(self, X):
        return np.dot(self._eigenvectors, X)

    @property
    def num_components(self):
        return self._num_components

    @property
    def eigenvectors(self):
        return self._eigenvectors

    @property
    def eigenvalues(self):
        return self._eigenvalues

    def __repr__(self):
        return "LDA (num_components=%d)" % (self._num_components)


def fisherfaces_device(Xd, D, y, num_components=0):
    """The device pipeline of ``Fisherfaces.compute`` (feature.py:211-229) on resident uint8 faces
    Xd [n][>= D] with labels y (0..c-1): PCA(n - c) then LDA(num_components), W = P . L.  Returns
    (LDA eigenvalues fp64 host [m], W device fp64 [D][m], m, regime); nothing of the faces or of W
    leaves the device.  Regimes by what PCA keeps (training.py): pixel / gram / cov."""
    from .. import training
    y = np.asarray(y)
    lay = training.Layout(y, Xd.device)
    n, c = lay.n, lay.c
    k = n - c                                              # PCA(n - c), feature.py:219 / :88-89
    if k <= 0 or k > n - 1:
        k = n - 1
    k = min(k, D, n)                                       # columns of the economy SVD
    m = num_components                                     # LDA(num_components), feature.py:155-158
    if m <= 0 or m > c - 1:
        m = c - 1
    if k >= D:
        # PCA keeps every pixel dimension (a rotation): LDA in pixel space, W = V directly
        regime = "pixel"
        Sw, Sb = training.finite("pixel_scatter", *training.pixel_scatter(training.pixel_pieces(Xd, D, lay),
                                                                          lay.counts, n))
        evals, Wd = lda_eigen(Sw, Sb, m, device_out=True)
        del Sw, Sb
    elif n <= D:
        # n x n Gram of the centred faces: U_k = XC^T V_k / sigma_k, features V_k sigma_k
        regime = "gram"
        evals, Wd = training.fisher_gram(Xd, D, lay, y, k, m)
    else:
        # D x D covariance: P = leading k eigenvectors, features XC P, W = P L
        regime = "cov"
        pieces = training.pixel_pieces(Xd, D, lay)
        lam, Pd = training.finite("eigh_desc", *training.eigh_desc(
            training.finite("covariance", training.covariance(pieces, n)), k))
        del pieces
        Pd = Pd.contiguous()
        mu = training.mean_image(Xd, D, lay)
        shift = _device.gemm_f64(mu.reshape(1, -1).contiguous(), Pd).reshape(-1)
        Fd = _device.Projection(Wt_device=Pd.t().contiguous(), D=D).project(Xd, shift64=shift, f64=True)
        Sw, Sb = training.finite("feature_scatter", *training.feature_scatter(Fd, y))
        del Fd
        evals, L = lda_eigen(Sw, Sb, m)
        L32 = np.asarray(L, dtype=np.float32).astype(np.float64)          # feature.py:176
        Wd = _device.gemm_f64(Pd, _device.f64_dev(L32))                      # feature.py:229
    return evals, Wd, m, regime


class Fisherfaces(_DeviceProjMixin, AbstractFeature):
    """feature.py:206-260."""

    def __init__(self, num_components=0):
        AbstractFeature.__init__(self)
        self._num_components = num_components

    def compute(self, X, y):
        """feature.py:211-235.  uint8 faces take the exact device pipeline (training.py): PCA(n - c)
        then LDA(num_components), W = P . L, features W^T x; any other input dtype takes the
        ChainOperator(PCA, LDA) path on fp64 device GEMMs."""
        y = np.asarray(y)
        Xd, D, kind = _device_rows(X)
        if kind != "u8":
            return self._compute_chain(X, y)
        evals, Wd, m, self._regime = fisherfaces_device(Xd, D, y, self._num_components)
        self._eigenvalues = np.array(evals, dtype=np.float32, copy=True)      # :226-227 (LDA's, float32)
        self._num_components = m
        self._eigenvectors = np.asmatrix(Wd.cpu().numpy())
        self._prime_proj(Wd.contiguous())
        # features of the training set (:231-235): one batched exact projection of the resident faces
        Fd = self.project_device(Xd, f64=True)
        feats = [np.asmatrix(r.reshape(-1, 1)) for r in Fd.cpu().numpy()]
        self.__dict__["_dev_features"] = (id(feats), Fd)      # handed to the classifier's gallery
        return feats

    def _compute_chain(self, X, y):
        """feature.py:211-235 for non-uint8 inputs: ChainOperator(PCA, LDA) on fp64 device GEMMs."""
        n = len(y)                                             # feature.py:216-217
        c = len(np.unique(y))
        pca = PCA(num_components=(n - c))                      # :219-224
        lda = LDA(num_components=self._num_components)
        model = ChainOperator(pca, lda)
        model.compute(X, y)
        self._eigenvalues = lda.eigenvalues                    # :226-227
        self._num_components = lda.num_components
        # W = P . L (:229) on the fp64 MFMA
        P = _device.f64_dev(np.asarray(pca.eigenvectors))
        L = _device.f64_dev(np.asarray(lda.eigenvectors, dtype=np.float64))
        self._eigenvectors = np.asmatrix(_device.gemm_f64(P, L).cpu().numpy())
        self.__dict__.pop("_dev_proj", None)
        # features of the training set (:231-235): one batched projection
        return self._project_host(X)

    def extract(self, X):
        """feature.py:237-239."""
        return self._project_host([np.asarray(X).reshape(-1)])[0]

    def project(self, X):
        """feature.py:241-242: W^T X, no mean subtraction."""
        return self._project_host([np.asarray(X).reshape(-1)])[0]

    def extract_batch(self, X):
        """Batch version of extract: list of (d,1) float64 matrices."""
        return self._project_host(X)

    def _proj_matrix(self):
        return np.asarray(self._eigenvectors), None

    def reconstruct(self, X):
        return np.dot(self._eigenvectors, X)

    @property
    def num_components(self):
        return self._num_components

    @property
    def eigenvalues(self):
        return self._eigenvalues

    @property
    def eigenvectors(self):
        return self._eigenvectors

    def __repr__(self):
        return "Fisherfaces (num_components=%s)" % (self.num_components)


from .lbp import ExtendedLBP, LocalDescriptor  # noqa: E402  (feature.py:263)


class SpatialHistogram(AbstractFeature):
    """feature.py:266-305: per-cell LBP histograms, concatenated row-major over the grid.

    The histograms are integer counts on the device (one ``ofr_elbp_hist`` launch per batch of
    same-sized faces); the float64 histograms the reference API returns are count / (py * px),
    which is exactly what numpy's ``np.histogram(..., density=True)`` gives for one cell
    (feature.py:298-299).  ``compute`` leaves the device counts for the classifier
    (``PredictableModel.compute``): the LBPH gallery stays resident as counts, never rebuilt from
    the float64 list."""

    def __init__(self, lbp_operator=ExtendedLBP(), sz=(8, 8)):
        AbstractFeature.__init__(self)
        if not isinstance(lbp_operator, LocalDescriptor):
            raise TypeError("Only an operator of type facerec.lbp.LocalDescriptor is a valid lbp_operator.")
        self.lbp_operator = lbp_operator
        self.sz = sz

    def compute(self, X, y):
        feats, dev = self._histograms(X, keep_device=True)
        if dev is not None:      # one face size: the counts go to the classifier's device gallery
            self.__dict__["_dev_features"] = (id(feats), dev)
        return feats

    def extract(self, X):
        return self.histograms([X])[0]

    def spatially_enhanced_histogram(self, X):
        return self.histograms([X])[0]

    def counts_device(self, imgs):
        """uint8 image stack (n,H,W) (host or device) -> (counts device tensor [n][cells][2^P], cell pixels, bytes)."""
        if not isinstance(self.lbp_operator, ExtendedLBP):
            raise NotImplementedError("SpatialHistogram (MI355X build) runs ExtendedLBP operators only")
        from .lbp import as_u8_images
        if not hasattr(imgs, "device"):
            imgs = as_u8_images(np.ascontiguousarray(imgs) if isinstance(imgs, np.ndarray) and imgs.ndim == 3
                                else np.stack([np.asarray(x) for x in imgs]))
        counts, cell, cb = _device.elbp_hist(_device.u8_images(imgs), self.lbp_operator.geometry(), tuple(self.sz))
        return counts, cell, cb

    def counts_batch(self, X):
        """Faces of one size (list, array [n][H][W] or a uint8 device tensor such as ``ingest.faces``
        returns) -> (counts [n][cells * 2^P] device tensor, cell pixel count, bytes per count), one
        launch.  The histogram of face i is counts[i] / cell."""
        counts, cell, cb = self.counts_device(X if hasattr(X, "device") or (isinstance(X, np.ndarray) and X.ndim == 3)
                                              else list(X))
        return counts.reshape(counts.shape[0], -1), cell, cb

    def histograms(self, X):
        """List of images -> list of float64 histograms = count/(py*px) (np.histogram density, :298-299)."""
        return self._histograms(X)[0]

    def _histograms(self, X, keep_device=False):
        if hasattr(X, "device"):          # a device face batch [n][H][W]
            X = X.cpu().numpy()
        if len(X) == 0:
            return [], None
        shapes = {np.asarray(x).shape for x in X}
        out = [None] * len(X)
        dev = None
        for shp in shapes:   # images of one size per launch
            sel = [i for i, x in enumerate(X) if np.asarray(x).shape == shp]
            counts, cell, cb = self.counts_device([X[i] for i in sel])
            c = _device.counts_numpy(counts, cb).astype(np.int64).reshape(len(sel), -1)
            with np.errstate(invalid="ignore", divide="ignore"):
                h = c.astype(np.float64) / float(cell)
            for j, i in enumerate(sel):
                out[i] = h[j]
            if keep_device and len(shapes) == 1 and cell > 0:
                dev = ("counts", counts.reshape(len(sel), -1), cell, cb)
        return out, dev

    def __getstate__(self):
        st = dict(self.__dict__)
        st.pop("_dev_features", None)      # derived device state, never pickled
        return st

    def __repr__(self):
        return "SpatialHistogram (operator=%s, grid=%s)" % (repr(self.lbp_operator), str(self.sz))


for _c in (AbstractFeature, Identity, PCA, LDA, Fisherfaces, SpatialHistogram):
    _c.__module__ = "ocvfacerec.facerec.feature"
