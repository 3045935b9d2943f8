"""CPU oracle for the ocvfacerec recognition hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  It is an independent float64 numpy restatement of the reference
algorithms (bytefish facerec as vendored in ``src/ocvfacerec/facerec/``), each
function citing the reference file:line it follows (paths relative to
``/root/reference/src/ocvfacerec/facerec/``).

Parity pinning: the restatement is checked against golden vectors produced by
running the reference's own modules in this container
(``tests/golden/make_golden.py``; outputs in ``tests/golden/*.npz``) and
against the reference's bundled trained model ``data/individuals.pkl``.

Two evaluation modes are provided for the nearest-neighbour search:
* ``nn_predict_faithful`` mirrors the reference loop (one distance call per
  gallery item, ``classifier.py:104-108``) — the reference-faithful CPU
  baseline;
* ``nn_search_vectorized`` computes the same float64 distances with BLAS and
  a stable (lowest-index-first) ordering.
"""
from __future__ import annotations

import numpy as np

F64_EPS = np.finfo("float").eps  # distance.py:115 ``np.finfo('float').eps``


# ---------------------------------------------------------------------------
# util.py
# ---------------------------------------------------------------------------
def as_column_matrix(X):
    """util.py:70-84 — D x N matrix of the input dtype (columns = flattened items)."""
    if len(X) == 0:
        return np.array([])
    cols = [np.asarray(x).reshape(-1) for x in X]
    return np.asmatrix(np.stack(cols, axis=1).astype(np.asarray(X[0]).dtype, copy=False))


# ---------------------------------------------------------------------------
# feature.py: PCA / LDA / Fisherfaces
# ---------------------------------------------------------------------------
def pca_compute(X, y, num_components=0):
    """feature.py:83-108.  Returns dict(mean, eigenvectors, eigenvalues, features, num_components)."""
    XC = as_column_matrix(X)
    n = XC.shape[1]
    if num_components <= 0 or num_components > n - 1:          # :88-89
        num_components = n - 1
    mean = XC.mean(axis=1).reshape(-1, 1)                       # :91
    XC = XC - mean                                              # :92
    U, s, _ = np.linalg.svd(XC, full_matrices=False)            # :94
    idx = np.argsort(-s)                                        # :96
    s, U = s[idx], U[:, idx]                                    # :97
    U = U[:, :num_components].copy()                            # :99
    s = s[:num_components].copy()                               # :100
    ev = np.power(s, 2) / XC.shape[1]                           # :102
    feats = [np.dot(U.T, np.asarray(x).reshape(-1, 1) - mean) for x in X]   # :104-108, :114-116
    return dict(mean=mean, eigenvectors=U, eigenvalues=ev, features=feats, num_components=num_components)


def lda_scatter(F, y):
    """feature.py:160-168: total mean, Sw and Sb (float64) of column features F (d x N)."""
    F = np.asarray(F, dtype=np.float64)
    y = np.asarray(y)
    c = len(np.unique(y))
    d = F.shape[0]
    mean_total = F.mean(axis=1).reshape(-1, 1)
    Sw = np.zeros((d, d))
    Sb = np.zeros((d, d))
    for i in range(c):
        Xi = F[:, np.where(y == i)[0]]
        mi = Xi.mean(axis=1).reshape(-1, 1)
        Sw += np.dot(Xi - mi, (Xi - mi).T)
        Sb += Xi.shape[1] * np.dot(mi - mean_total, (mi - mean_total).T)
    return mean_total, Sw, Sb


def lda_compute(X, y, num_components=0):
    """feature.py:147-182.  X: list of (d,1) PCA features."""
    XC = as_column_matrix(X)
    y = np.asarray(y)
    c = len(np.unique(y))
    if num_components <= 0 or num_components > c - 1:          # :155-158
        num_components = c - 1
    _, Sw, Sb = lda_scatter(XC, y)                              # :160-168
    evals, evecs = np.linalg.eig(np.linalg.inv(Sw) @ Sb)        # :170 (np.matrix * == matmul)
    idx = np.argsort(-evals.real)                               # :172
    evals, evecs = evals[idx], evecs[:, idx]                    # :173
    evals = np.array(evals[:num_components].real, dtype=np.float32, copy=True)            # :175
    evecs = np.matrix(evecs[:, :num_components].real, dtype=np.float32, copy=True)        # :176
    feats = [np.dot(evecs.T, np.asarray(x).reshape(-1, 1)) for x in X]                     # :178-185
    return dict(eigenvectors=evecs, eigenvalues=evals, features=feats, num_components=num_components,
                Sw=Sw, Sb=Sb)


def fisherfaces_compute(X, y, num_components=0):
    """feature.py:211-235: PCA(n-c) -> LDA(num_components); W = P.L; features = W^T x."""
    y = np.asarray(y)
    n = len(y)
    c = len(np.unique(y))
    pca = pca_compute(X, y, n - c)                              # :219, operators.py:72-74
    lda = lda_compute(pca["features"], y, num_components)       # :220
    W = np.dot(pca["eigenvectors"], lda["eigenvectors"])        # :229
    feats = [fisherfaces_project(W, x) for x in X]              # :231-235
    return dict(W=np.asmatrix(W), eigenvalues=lda["eigenvalues"], num_components=lda["num_components"],
                features=feats, pca=pca, lda=lda)


def fisherfaces_project(W, x):
    """feature.py:237-242 — W^T x with NO mean subtraction."""
    return np.dot(np.asmatrix(W).T, np.asarray(x).reshape(-1, 1))


# ---------------------------------------------------------------------------
# lbp.py: ExtendedLBP ; feature.py: SpatialHistogram
# ---------------------------------------------------------------------------
def elbp_geometry(radius=1, neighbors=8):
    """lbp.py:84-121: per-point (fy, fx, cy, cx) integer offsets and fp64 weights (w1..w4).

    Returns (origin (oy, ox), block size (by, bx), offsets int64 [P,4] as
    (fy, fx, cy, cx), weights float64 [P,4]).
    """
    angles = 2 * np.pi / neighbors                                              # :84
    theta = np.arange(0, 2 * np.pi, angles)                                     # :85
    sp = np.array([-np.sin(theta), np.cos(theta)]).T                            # :87
    sp *= radius                                                                # :88
    miny, maxy = min(sp[:, 0]), max(sp[:, 0])                                   # :90-93
    minx, maxx = min(sp[:, 1]), max(sp[:, 1])
    by = np.ceil(max(maxy, 0)) - np.floor(min(miny, 0)) + 1                     # :95
    bx = np.ceil(max(maxx, 0)) - np.floor(min(minx, 0)) + 1                     # :96
    oy = 0 - np.floor(min(miny, 0))                                             # :98
    ox = 0 - np.floor(min(minx, 0))                                             # :99
    offs = np.zeros((len(sp), 4), np.int64)
    wts = np.zeros((len(sp), 4), np.float64)
    for i, p in enumerate(sp):
        y, x = p + (oy, ox)                                                     # :108
        fx, fy, cx, cy = np.floor(x), np.floor(y), np.ceil(x), np.ceil(y)       # :110-113
        ty, tx = y - fy, x - fx                                                 # :115-116
        wts[i] = [(1 - tx) * (1 - ty), tx * (1 - ty), (1 - tx) * ty, tx * ty]   # :118-121
        offs[i] = [fy, fx, cy, cx]
    return (int(oy), int(ox)), (int(by), int(bx)), offs, wts


def elbp(X, radius=1, neighbors=8):
    """lbp.py:80-130 — uint32 codes, evaluated in the reference's fp64 operation order (no FMA)."""
    X = np.asanyarray(X)
    ysize, xsize = X.shape
    (oy, ox), (by, bx), offs, wts = elbp_geometry(radius, neighbors)
    dx = xsize - bx + 1                                                         # :101
    dy = ysize - by + 1                                                         # :102
    C = np.asarray(X[oy:oy + dy, ox:ox + dx], dtype=np.uint8)                   # :104
    result = np.zeros((dy, dx), dtype=np.uint32)                                # :105
    for i in range(len(offs)):
        fy, fx, cy, cx = offs[i]
        w1, w2, w3, w4 = wts[i]
        N = w1 * X[fy:fy + dy, fx:fx + dx]                                      # :123
        N += w2 * X[fy:fy + dy, cx:cx + dx]                                     # :124
        N += w3 * X[cy:cy + dy, fx:fx + dx]                                     # :125
        N += w4 * X[cy:cy + dy, cx:cx + dx]                                     # :126
        result += np.uint32(1 << i) * (N >= C)                                  # :128-129
    return result


def spatial_histogram_counts(L, neighbors=8, sz=(8, 8)):
    """feature.py:286-302 as integer counts: (grid_rows*grid_cols, 2**P) int64, and the cell size."""
    lh, lw = L.shape
    gr, gc = sz
    py, px = int(np.floor(lh / gr)), int(np.floor(lw / gc))                     # :292-293
    nb = 2 ** neighbors
    out = np.zeros((gr * gc, nb), np.int64)
    for r in range(gr):
        for c in range(gc):
            C = L[r * py:(r + 1) * py, c * px:(c + 1) * px]                     # :297
            out[r * gc + c] = np.bincount(C.reshape(-1).astype(np.int64), minlength=nb)[:nb]
    return out, py * px


def spatial_histogram(X, radius=1, neighbors=8, sz=(8, 8)):
    """feature.py:286-302 — concatenated per-cell density histograms (float64)."""
    L = elbp(X, radius, neighbors)
    lh, lw = L.shape
    gr, gc = sz
    py, px = int(np.floor(lh / gr)), int(np.floor(lw / gc))
    nb = 2 ** neighbors
    E = []
    for r in range(gr):
        for c in range(gc):
            C = L[r * py:(r + 1) * py, c * px:(c + 1) * px]
            H = np.histogram(C, bins=nb, range=(0, nb), density=True)[0]        # :298-299
            E.extend(H)
    return np.asarray(E)


# ---------------------------------------------------------------------------
# distance.py
# ---------------------------------------------------------------------------
def euclidean(p, q):
    """distance.py:57-60."""
    p = np.asarray(p).flatten()
    q = np.asarray(q).flatten()
    return np.sqrt(np.sum(np.power((p - q), 2)))


def cosine(p, q):
    """distance.py:74-77 (negated cosine similarity)."""
    p = np.asarray(p).flatten()
    q = np.asarray(q).flatten()
    return -np.dot(p.T, q) / (np.sqrt(np.dot(p, p.T) * np.dot(q, q.T)))


def chisquare(p, q):
    """distance.py:112-116."""
    p = np.asarray(p).flatten()
    q = np.asarray(q).flatten()
    bin_dists = (p - q) ** 2 / (p + q + F64_EPS)
    return np.sum(bin_dists)


METRICS = {"EuclideanDistance": euclidean, "CosineDistance": cosine, "ChiSquareDistance": chisquare}


def pairwise(metric, Q, G):
    """All-pairs float64 distances [B, N] for the three metrics (vectorised)."""
    Q = np.asarray(Q, np.float64)
    G = np.asarray(G, np.float64)
    if metric == "EuclideanDistance":
        # direct-difference form, blocked to bound memory
        out = np.empty((Q.shape[0], G.shape[0]))
        for i in range(Q.shape[0]):
            dlt = G - Q[i]
            out[i] = np.sqrt(np.einsum("ij,ij->i", dlt, dlt))
        return out
    if metric == "CosineDistance":
        num = Q @ G.T
        return -num / np.sqrt(np.einsum("ij,ij->i", Q, Q)[:, None] * np.einsum("ij,ij->i", G, G)[None, :])
    if metric == "ChiSquareDistance":
        out = np.empty((Q.shape[0], G.shape[0]))
        for i in range(Q.shape[0]):
            out[i] = np.sum((G - Q[i]) ** 2 / (G + Q[i] + F64_EPS), axis=1)
        return out
    raise ValueError(metric)


# ---------------------------------------------------------------------------
# classifier.py: NearestNeighbor
# ---------------------------------------------------------------------------
def _vote(sorted_y):
    """classifier.py:121-123 — bincount vote, ties to the smallest label."""
    hist = dict((key, val) for key, val in enumerate(np.bincount(sorted_y)) if val)
    best = None
    for key, val in hist.items():
        if best is None or val > best[1]:
            best = (key, val)
    return best[0]


def nn_predict_faithful(X, y, q, metric="EuclideanDistance", k=1):
    """classifier.py:76-129, one metric call per gallery item (reference-faithful loop).

    Uses a stable argsort so exact ties resolve to the lowest gallery index
    (the reference's default quicksort leaves tie order unspecified).
    """
    fn = METRICS[metric]
    y = np.asarray(y)
    distances = []
    for xi in X:                                                                 # :104-108
        distances.append(fn(np.asarray(xi).reshape(-1, 1), q))
    if len(distances) > len(y):                                                  # :109-110
        raise Exception("More distances than classes. Is your distance metric correct?")
    distances = np.asarray(distances)
    idx = np.argsort(distances, kind="stable")                                   # :113
    sorted_y = y[idx][:k]                                                        # :115-118
    sorted_d = distances[idx][:k]                                                # :116-119
    return [_vote(sorted_y), {"labels": sorted_y, "distances": sorted_d}], idx[:k]


def nn_search_vectorized(metric, Q, G, k):
    """float64 all-pairs distances + stable top-k: returns (dist [B,k], idx [B,k])."""
    D = pairwise(metric, Q, G)
    idx = np.argsort(D, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(D, idx, 1), idx


def nn_search_blas(Q, G, k):
    """Vectorised float64 1-NN with BLAS: ||q||^2 + ||g||^2 - 2 Q G^T (CPU-baseline timing only; the
    GEMM form cancels, so parity checks use ``nn_search_vectorized``)."""
    Q = np.asarray(Q, np.float64)
    G = np.asarray(G, np.float64)
    D2 = np.einsum("ij,ij->i", Q, Q)[:, None] + np.einsum("ij,ij->i", G, G)[None, :] - 2.0 * (Q @ G.T)
    idx = np.argsort(D2, axis=1, kind="stable")[:, :k]
    return np.sqrt(np.maximum(np.take_along_axis(D2, idx, 1), 0)), idx


def near_tie_mask(metric, Q, G, rel=1e-4):
    """Queries whose best and second-best oracle distances are within ``rel``."""
    D = pairwise(metric, Q, G)
    part = np.sort(D, axis=1)[:, :2]
    d1, d2 = part[:, 0], part[:, 1]
    scale = np.maximum(np.abs(d1), 1e-300)
    return (d2 - d1) / scale <= rel


# ---------------------------------------------------------------------------
# validation.py: KFoldCrossValidation with Fisherfaces + NearestNeighbor
# ---------------------------------------------------------------------------
def kfold_fisherfaces_faithful(X, y, k=10, seed=0, metric="EuclideanDistance"):
    """validation.py:202-258 (shuffle :54-70 from random.seed(seed)), the model of
    thetrainer.py:120-124 (Fisherfaces + NearestNeighbor k=1), one predict per test face
    (:251-256).  Returns (true_positives, false_positives, k_used)."""
    import math
    import random
    random.seed(seed)
    idx = np.argsort([random.random() for _ in range(len(y))])
    y = np.asarray(y)[idx]
    X = [X[i] for i in idx]
    c = len(np.unique(y))
    folds = [np.where(y == i)[0].tolist() for i in range(c)]
    n = min(len(f) for f in folds)
    k = min(k, n)
    size = int(math.floor(n / k))
    tp = fp = 0
    for i in range(k):
        lo, hi = i * size, (i + 1) * size
        test = [folds[r][j] for j in range(lo, hi) for r in range(c)]
        train = [folds[r][j] for j in range(0, lo) for r in range(c)]
        train += [folds[r][j] for j in range(hi, n) for r in range(c)]
        m = fisherfaces_compute([X[t] for t in train], y[train])
        for j in test:
            q = fisherfaces_project(m["W"], X[j])
            pred = nn_predict_faithful(m["features"], y[train], q, metric, 1)[0][0]
            tp, fp = (tp + 1, fp) if pred == y[j] else (tp, fp + 1)
    return tp, fp, k



# ---------------------------------------------------------------------------
# Face-tensor ingestion: cv2.imread(GRAYSCALE) + cv2.resize
# (INTER_LINEAR) in TheTrainer.read_images (trainer/thetrainer.py:99-103), and
# the recognizers' crop + cv2.cvtColor(BGR2GRAY) + cv2.resize(INTER_CUBIC)
# (bin/ocvf_recognizer.py:64-66, ocvf_recognizer_ros.py:113-115).
#
# The arithmetic lives in OpenCV, a third-party dependency ABSENT from
# /root/reference and from this image (README.md:44-48 names Ubuntu 14.04's
# python-opencv, i.e. OpenCV 2.4.8).  Restated from OpenCV's published 8-bit
# fixed-point algorithm (imgproc resize.cpp resizeGeneric_ with
# INTER_RESIZE_COEF_BITS = 11; color.cpp RGB2Gray with yuv_shift = 14), scalar
# (non-SIMD) form.  Parity against cv2 itself is UNPINNED: OpenCV's SSE paths of
# the vertical pass round differently in the last bit on some pixels.  What
# pins it: the reference's pickled gallery (data/individuals.pkl) is reproduced
# from the bundled JPEGs to ~1e-3 (tests/test_gpu_ingest.py).
# ---------------------------------------------------------------------------
CV_COEF_BITS = 11
CV_COEF_SCALE = 1 << CV_COEF_BITS


def _cv_axis(dsize, ssize, interp):
    """Source taps [dsize][ksize] (clamped to the image) and int16 weights of one axis.

    resizeGeneric_: scale = 1 / (dsize / ssize); f = (float)((i + 0.5) * scale - 0.5); s = floor(f);
    f -= s; weights = saturate_cast<short>(rint(cbuf * 2048)) with cbuf = (1 - f, f) for
    INTER_LINEAR and interpolateCubic(f) (A = -0.75, float arithmetic) for INTER_CUBIC.  Linear
    columns past the edges use f = 0 (x only; rows keep their weights and clamp the row index)."""
    scale = 1.0 / (dsize / ssize)
    f = ((np.arange(dsize) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    one = np.float32(1.0)
    if interp == "linear":
        cbuf = np.stack([one - f, f], 1)
        first = s
    else:
        A = np.float32(-0.75)
        x = f
        c0 = ((A * (x + one) - np.float32(5) * A) * (x + one) + np.float32(8) * A) * (x + one) - np.float32(4) * A
        c1 = ((A + np.float32(2)) * x - (A + np.float32(3))) * x * x + one
        c2 = ((A + np.float32(2)) * (one - x) - (A + np.float32(3))) * (one - x) * (one - x) + one
        c3 = one - c0 - c1 - c2
        cbuf = np.stack([c0, c1, c2, c3], 1).astype(np.float32)
        first = s - 1
    w = np.clip(np.rint(cbuf * np.float32(CV_COEF_SCALE)), -32768, 32767).astype(np.int64)
    taps = np.clip(first[:, None] + np.arange(cbuf.shape[1])[None, :], 0, ssize - 1)
    return taps, w, s, f


def cv_resize_u8(img, size, interp="linear"):
    """cv2.resize(img, size=(width, height), interpolation) of a 2-D uint8 image, fixed point:
    H pass D[x] = sum_k S[tap_k] * alpha_k (int), V pass (sum_k D_k * beta_k + 2^21) >> 22,
    saturated to uint8; a resize to the same size is a copy (cv::resize shortcut)."""
    img = np.asarray(img, np.uint8)
    H, W = img.shape
    dw, dh = int(size[0]), int(size[1])
    if (dw, dh) == (W, H):
        return img.copy()
    xt, xw, xs, xf = _cv_axis(dw, W, interp)
    if interp == "linear":                       # x only: columns past either edge take (1, 0) at the edge pixel
        edge = (xs < 0) | (xs >= W - 1)
        xt[edge] = np.clip(xs[edge], 0, W - 1)[:, None]
        xw[edge] = np.array([CV_COEF_SCALE, 0])
    yt, yw, _, _ = _cv_axis(dh, H, interp)
    S = img.astype(np.int64)
    Dh = np.einsum("rxk,xk->rx", S[:, xt], xw)                 # [H][dw]
    V = np.einsum("ykx,yk->yx", Dh[yt], yw)                    # [dh][dw]
    return np.clip((V + (1 << (2 * CV_COEF_BITS - 1))) >> (2 * CV_COEF_BITS), 0, 255).astype(np.uint8)


def cv_bgr2gray(img):
    """cv2.cvtColor(img, COLOR_BGR2GRAY) for uint8 BGR (or BGRA): (1868 B + 9617 G + 4899 R + 2^13) >> 14."""
    a = np.asarray(img, np.uint8).astype(np.int64)
    return ((a[..., 0] * 1868 + a[..., 1] * 9617 + a[..., 2] * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def recognizer_face(frame_bgr, box, size):
    """ocvf_recognizer.py:64-66: crop img[y0:y1, x0:x1], BGR2GRAY, resize(size, INTER_CUBIC)."""
    x0, y0, x1, y1 = box
    return cv_resize_u8(cv_bgr2gray(frame_bgr[y0:y1, x0:x1]), size, "cubic")
