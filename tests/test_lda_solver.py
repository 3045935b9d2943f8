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


def test_lda_singular_sw_takes_the_pencil_limit():
    """inv(Sw) with an exactly zero pivot (feature.py:170 would raise): the null direction of Sw comes
    first with an infinite eigenvalue, the other columns solve Sb v = lambda Sw v."""
    from opencv_facerecognizer_amd.facerec.feature import lda_eigen
    Sw, Sb = _scatter(31, 27, 4, 8)
    Sw[-1, :] = 0.0
    Sw[:, -1] = 0.0                                  # exactly singular: LU meets a zero pivot
    with pytest.raises(np.linalg.LinAlgError):
        np.linalg.inv(Sw)
    with pytest.warns(UserWarning, match="singular"):
        lam, V = lda_eigen(Sw, Sb, 3, solver="eig")
    assert np.isinf(lam[0]) and lam[0] > 0 and np.all(np.isfinite(lam[1:]))
    assert abs(abs(V[-1, 0]) - 1.0) < 1e-12          # the null direction e_27
    np.testing.assert_allclose(np.linalg.norm(V, axis=0), 1.0, rtol=1e-12)
    for j in (1, 2):
        r = Sb @ V[:, j] - lam[j] * (Sw @ V[:, j])
        assert np.linalg.norm(r) < 1e-9 * np.linalg.norm(Sb), (j, np.linalg.norm(r))


def test_lda_singular_sw_reproduces_the_reference_on_bundled_faces(golden):
    """The bundled faces hold two identical images of one class (steve_crop0 == steve_crop5), so Sw of
    PCA(n - c) is singular in exact arithmetic and the reference's inv(Sw) inverted rounding noise (its
    golden dominant eigenvalue 2.9e16).  The pencil limit gives the reference's golden LDA columns."""
    from opencv_facerecognizer_amd.facerec.feature import _lda_singular_sw
    f = golden("individuals_faces.npz")
    X = f["X"].reshape(31, -1)
    dup = [(i, j) for i in range(31) for j in range(i + 1, 31) if np.array_equal(X[i], X[j])]
    assert dup == [(23, 28)] and f["y"][23] == f["y"][28]
    _, Sw, Sb = O.lda_scatter(f["pca_features"].T, f["y"])
    with pytest.warns(UserWarning):
        lam, V = _lda_singular_sw(np.asarray(Sw), np.asarray(Sb), 3)
    L = np.asarray(f["lda_eigenvectors"], np.float64)
    cos = np.abs(np.sum(L * V, 0)) / np.linalg.norm(L, axis=0)
    assert cos[0] > 1 - 1e-9 and cos[1] > 1 - 1e-6 and cos[2] > 0.999, cos
    assert np.isinf(lam[0]) and f["lda_eigenvalues"][0] > 1e15
    np.testing.assert_allclose(lam[1:], f["lda_eigenvalues"][1:], rtol=5e-3)
