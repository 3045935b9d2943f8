"""LDA eigensolvers (host, no GPU): the reference's eig(inv(Sw) Sb) and the symmetric-definite
eigh(Sb, Sw) selected by OFR_LDA_SOLVER=eigh (opencv_facerecognizer_amd/facerec/feature.py
lda_eigen; reference feature.py:170-176) give the same eigenpairs up to column sign."""
import numpy as np
import pytest

import facerec_oracle as O


def _scatter(n, d, c, seed):
    r = np.random.default_rng(seed)
    means = r.normal(0, 3, (c, d))
    y = np.arange(n) % c
    X = (means[y] + r.normal(0, 1, (n, d))).T        # d x n, as feature.py holds it
    _, Sw, Sb = O.lda_scatter(X, y)
    return np.asarray(Sw), np.asarray(Sb)


@pytest.mark.parametrize("n,d,c", [(31, 27, 4), (400, 120, 40), (300, 250, 10)])
def test_lda_eigh_matches_reference_eig(n, d, c):
    from opencv_facerecognizer_amd.facerec.feature import lda_eigen
    Sw, Sb = _scatter(n, d, c, n + d)
    l0, V0 = lda_eigen(Sw, Sb, c - 1, solver="eig")
    l1, V1 = lda_eigen(Sw, Sb, c - 1, solver="eigh")
    assert V0.shape == V1.shape == (d, c - 1)
    np.testing.assert_allclose(l1, l0, rtol=1e-7, atol=1e-9 * abs(l0).max())
    np.testing.assert_allclose(np.linalg.norm(V1, axis=0), 1.0, rtol=1e-12)
    cos = np.abs(np.sum(V0 * V1, axis=0))
    assert cos.min() > 1 - 1e-7, cos


def test_lda_eigh_falls_back_on_indefinite_sw():
    from opencv_facerecognizer_amd.facerec.feature import lda_eigen
    Sw, Sb = _scatter(31, 27, 4, 5)
    Sw = Sw - (np.linalg.eigvalsh(Sw)[0] + 1.0) * np.eye(27)   # invertible, not positive definite
    with pytest.warns(UserWarning):
        l1, _ = lda_eigen(Sw, Sb, 3, solver="eigh")
    l0, _ = lda_eigen(Sw, Sb, 3, solver="eig")
    np.testing.assert_array_equal(l1, l0)


def test_lda_solver_env_rejects_unknown(monkeypatch):
    from opencv_facerecognizer_amd.facerec.feature import lda_eigen
    monkeypatch.setenv("OFR_LDA_SOLVER", "svd")
    Sw, Sb = _scatter(31, 27, 4, 6)
    with pytest.raises(ValueError):
        lda_eigen(Sw, Sb, 3)
