"""The context-based C ABI of SURVEY §8b (ofr_ctx_create / ofr_project_u8 / ofr_gram / ofr_scatter /
ofr_knn), called through ctypes on plain row-major device buffers of odd sizes, against the
float64 oracle (the reference's numpy formulas: feature.py:91-94, 114-116, 160-168, 241-242;
distance.py:57-60, 74-77, 112-116)."""
import ctypes

import numpy as np
import pytest
import torch

import facerec_oracle as O
from test_gpu_parity import _check_search, _rng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from opencv_facerecognizer_amd import _lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    torch.cuda.set_device(0)
    _lib.device()
    h = ctypes.c_void_p()
    _lib.call("ofr_ctx_create", 0, ctypes.byref(h))
    yield h
    _lib.call("ofr_ctx_destroy", h)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("D,d,B", [(1000, 53, 37), (4096, 64, 300)])
def test_project_u8(ctx, D, d, B):
    from opencv_facerecognizer_amd._lib import call, ptr, stream, OFR_FP64_ACC, OFR_PROJ_REUSE_W
    r = _rng(61)
    X = r.integers(0, 256, (B, D), dtype=np.uint8)
    W = r.normal(0, 1, (D, d)).astype(np.float32)
    mu = r.uniform(0, 255, D)
    Xd, Wd, mud = _dev(X), _dev(W), _dev(mu)
    Y = torch.empty((B, d), dtype=torch.float32, device="cuda")
    ref0 = X.astype(np.float64) @ W.astype(np.float64)                    # Fisherfaces.project (no mean)
    ref1 = (X.astype(np.float64) - mu) @ W.astype(np.float64)             # PCA.project
    for flags, m, ref in ((0, None, ref0), (OFR_PROJ_REUSE_W | OFR_FP64_ACC, mud, ref1), (OFR_PROJ_REUSE_W, None, ref0)):
        call("ofr_project_u8", ctx, stream(), ptr(Xd), B, D, ptr(Wd), d, ptr(m), ptr(Y), flags)
        got = Y.cpu().numpy().astype(np.float64)
        rel = np.linalg.norm(got - ref, axis=1) / np.linalg.norm(ref, axis=1)
        assert rel.max() < 1e-6, rel.max()


@pytest.mark.parametrize("side", [0, 1])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_gram(ctx, side, prec):
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._lib import call, ptr, stream
    r = _rng(62)
    A = r.normal(0, 1, (300, 129)).astype(np.float32)
    A64 = A.astype(np.float64)
    ref = A64.T @ A64 if side == 0 else A64 @ A64.T
    n = ref.shape[0]
    dt = torch.float64 if prec == "f64" else torch.float32
    G = torch.empty((n, n), dtype=dt, device="cuda")
    Ad = _dev(A)                       # held: a temporary's memory could be reused before the kernels run
    call("ofr_gram", ctx, stream(), ptr(Ad), 300, 129, side, _lib.DT_F64 if prec == "f64" else _lib.DT_F32, ptr(G))
    got = G.cpu().numpy().astype(np.float64)
    tol = 1e-12 if prec == "f64" else 2 ** -23
    assert np.abs(got - ref).max() <= tol * np.abs(ref).max() * 4


def test_scatter(ctx):
    from opencv_facerecognizer_amd._lib import call, ptr, stream
    r = _rng(63)
    N, d, c = 500, 40, 9
    y = r.integers(0, c, N).astype(np.int32)
    F = (r.normal(0, 1, (N, d)) + 3.0 * r.normal(0, 1, (c, d))[y]).astype(np.float32)
    Sw = torch.empty((d, d), dtype=torch.float64, device="cuda")
    Sb = torch.empty_like(Sw)
    M = torch.empty((c, d), dtype=torch.float64, device="cuda")
    Fd, yd, y1 = _dev(F), _dev(y), _dev((y + 1).astype(np.int32))
    call("ofr_scatter", ctx, stream(), ptr(Fd), ptr(yd), N, d, c, ptr(Sw), ptr(Sb), ptr(M))
    _, Sw0, Sb0 = O.lda_scatter(F.astype(np.float64).T, y)
    assert np.allclose(Sw.cpu().numpy(), Sw0, rtol=1e-10, atol=1e-10 * np.abs(Sw0).max())
    assert np.allclose(Sb.cpu().numpy(), Sb0, rtol=1e-10, atol=1e-10 * np.abs(Sb0).max())
    means = np.stack([F[y == i].astype(np.float64).mean(0) for i in range(c)])
    assert np.allclose(M.cpu().numpy(), means, rtol=1e-12, atol=1e-12)
    # labels outside 0..c-1 are rejected like the reference's range(c) loop would mis-handle them
    from opencv_facerecognizer_amd._lib import OfrError
    with pytest.raises(OfrError):
        call("ofr_scatter", ctx, stream(), ptr(Fd), ptr(y1), N, d, c, ptr(Sw), ptr(Sb), None)


@pytest.mark.parametrize("metric", ["EuclideanDistance", "CosineDistance", "ChiSquareDistance"])
def test_knn(ctx, metric):
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._lib import call, ptr, stream
    r = _rng(64)
    N, B, d, k = 1500, 70, 45, 3
    if metric == "ChiSquareDistance":
        G = r.integers(0, 6, (N, d)) / 225.0
        Q = np.concatenate([G[r.integers(0, N, B // 2)], r.integers(0, 6, (B - B // 2, d)) / 225.0])
        G[7] = G[8]                                  # an exact duplicate pair
    else:
        protos = r.normal(0, 5, (60, d))
        G = protos[np.arange(N) % 60] + r.normal(0, 1, (N, d))
        Q = protos[r.integers(0, 60, B)] + r.normal(0, 1, (B, d))
    G = G.astype(np.float32).astype(np.float64)
    Q = Q.astype(np.float32).astype(np.float64)
    m = {"EuclideanDistance": _lib.METRIC_EUCLIDEAN, "CosineDistance": _lib.METRIC_COSINE,
         "ChiSquareDistance": _lib.METRIC_CHISQUARE}[metric]
    od = torch.empty((B, k), dtype=torch.float32, device="cuda")
    oi = torch.empty((B, k), dtype=torch.int64, device="cuda")
    Qd, Gd = _dev(Q.astype(np.float32)), _dev(G.astype(np.float32))
    call("ofr_knn", ctx, stream(), m, ptr(Qd), B, ptr(Gd), None, N, d, k, 0, ptr(od), ptr(oi))
    _check_search(metric, Q, G, od.cpu().numpy().astype(np.float64), oi.cpu().numpy(), k, near_rel=2e-4)


@pytest.mark.parametrize("r,P,grid,shape", [(1, 8, (8, 8), (128, 128)), (2, 8, (4, 5), (61, 93)), (3, 4, (7, 7), (70, 70))])
def test_elbp_hist(ctx, r, P, grid, shape):
    """SURVEY §8b's ofr_elbp_hist(ctx, stream, imgs, n, H, W, w[P][4], off[P][4], P, gr, gc, counts): the sample
    offsets relative to the centre pixel (lbp.py:84-121 before the block origin is added), uint8 counts,
    bit-exact against the oracle's ExtendedLBP + per-cell histogram counts (feature.py:286-302)."""
    from opencv_facerecognizer_amd._lib import c_vp, call, ptr, stream
    from opencv_facerecognizer_amd.facerec.lbp import elbp_geometry
    (oy, ox), _, offs, wts = elbp_geometry(r, P)
    off_c = np.ascontiguousarray(offs - np.array([oy, ox, oy, ox], np.int32), dtype=np.int32)
    w = np.ascontiguousarray(wts, dtype=np.float64)
    g = _rng(63)
    imgs = g.integers(0, 256, (12,) + shape, dtype=np.uint8)
    imgs[:4] = (imgs[:4] // 64) * 64 + 31                   # tie-heavy
    gr, gc = grid
    out = torch.empty((12, gr * gc, 1 << P), dtype=torch.uint8, device="cuda")
    call("ofr_elbp_hist", ctx, stream(), ptr(_dev(imgs)), 12, shape[0], shape[1], w.ctypes.data_as(c_vp),
         off_c.ctypes.data_as(c_vp), P, gr, gc, ptr(out))
    got = out.cpu().numpy().astype(np.int64)
    for i in range(12):
        ref, _ = O.spatial_histogram_counts(O.elbp(imgs[i], r, P), P, grid)
        assert np.array_equal(got[i], ref), i
