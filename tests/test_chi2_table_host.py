"""The chi-square MFMA coarse pass's table and error bound, re-derived on the host (no GPU).

ofr_chi2_knn runs uint8 counts through a low-rank form of distance.py:112-116: per bin
(a - c)^2 / (a + c) = a + c - 4 F(a, c), F(a, c) = a c / (a + c) ~= sum_r U[a][r] U[c][r] with an fp16
table U [256][8].  The certificate of that pass uses |S - S~| <= ofr_chi2_mfma_bound(nbins) (Tq + Tg);
here the table is read back and the bound's ingredients (eta: the table's worst error per bin relative
to a + c; kappa: the worst sum |products| per bin relative to a + c) are recomputed exactly in fp64."""
import ctypes

import numpy as np

from opencv_facerecognizer_amd import _lib


def _table():
    buf = np.zeros(256 * 8, np.uint16)
    _lib.load().ofr_chi2_table(buf.ctypes.data_as(ctypes.c_void_p))
    return buf.view(np.float16).astype(np.float64).reshape(256, 8)


def test_table_error_bound_holds_for_every_count_pair():
    U = _table()
    assert np.all(U[0] == 0)                              # F(0, c) = 0 exactly
    a = np.arange(256, dtype=np.float64)[:, None]
    c = np.arange(256, dtype=np.float64)[None, :]
    s = a + c
    F = np.where(s > 0, a * c / np.where(s > 0, s, 1), 0.0)
    A = U @ U.T
    P = np.abs(U)[:, None, :] * np.abs(U)[None, :, :]
    m = s > 0
    eta = (np.abs(A - F)[m] / s[m]).max()
    kappa = (P.sum(2)[m] / s[m]).max()
    for nbins in (64, 4096, 16384, 65536):
        gamma = (nbins // 4 + 64) * 2.0 ** -23
        need = 4 * (eta + gamma * kappa) + 2.0 ** -22
        got = _lib.load().ofr_chi2_mfma_bound(nbins)
        assert got >= need and got <= need * (1 + 1e-6) + 1e-12, (nbins, got, need)
    assert eta < 1e-3 and kappa < 0.3                     # what makes the pass certify


def test_low_rank_chi2_close_on_histograms():
    """On LBP-like counts the table's chi^2 is within the bound of the exact one (count units)."""
    U = _table()
    r = np.random.default_rng(5)
    q = r.poisson(0.9, (20, 4096)).clip(0, 255)
    g = r.poisson(0.9, (30, 4096)).clip(0, 255)
    exact = np.array([[np.sum(np.where(x + y > 0, (x - y) ** 2 / np.maximum(x + y, 1), 0.0)) for y in g] for x in q])
    approx = q.sum(1)[:, None] + g.sum(1)[None, :] - 4 * np.einsum("bkr,nkr->bn", U[q], U[g])
    bound = _lib.load().ofr_chi2_mfma_bound(4096) * (q.sum(1)[:, None] + g.sum(1)[None, :])
    assert np.all(np.abs(exact - approx) <= bound)
