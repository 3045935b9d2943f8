"""The CPU oracle against the golden vectors produced by the reference's own code (tests/golden/make_golden.py)."""
import numpy as np
import pytest

import facerec_oracle as O


def _lbp_names(g):
    return sorted(k[4:] for k in g.files if k.startswith("img_"))


def test_oracle_lbp_codes_bit_exact(golden):
    g = golden("lbp_golden.npz")
    n = 0
    for nm in _lbp_names(g):
        im = g["img_" + nm]
        for r, P in ((1, 8), (2, 8), (2, 16), (3, 4)):
            ref = g[f"codes_{nm}_r{r}p{P}"]
            got = O.elbp(im, r, P)
            assert got.dtype == ref.dtype == np.uint32
            assert np.array_equal(got, ref), (nm, r, P)
            n += 1
    assert n == 40


def test_oracle_lbp_ties_differ_from_integer_lbp(golden):
    # the reference is NOT integer LBP: fp64 round-off in the bit-4/6 weights flips ties (SURVEY §7 hard part 1)
    im = golden("lbp_golden.npz")["img_lowent"].astype(int)
    codes = O.elbp(im.astype(np.uint8))
    C = im[1:-1, 1:-1]
    nb = [(0, 1), (-1, 1), (-1, 0), (-1, -1), (0, -1), (1, -1), (1, 0), (1, 1)]
    intl = sum(((im[1 + dy:127 + dy, 1 + dx:127 + dx] >= C).astype(np.uint32) << i) for i, (dy, dx) in enumerate(nb))
    assert (intl != codes).sum() > 1000


def test_oracle_spatial_histograms_bit_exact(golden):
    g = golden("lbp_golden.npz")
    for nm in _lbp_names(g):
        if f"hist_{nm}_r1p8_g8" not in g.files:
            continue
        im = g["img_" + nm]
        assert np.array_equal(O.spatial_histogram(im, 1, 8, (8, 8)), g[f"hist_{nm}_r1p8_g8"]), nm
        assert np.array_equal(O.spatial_histogram(im, 2, 8, (4, 5)), g[f"hist_{nm}_r2p8_g4x5"]), nm
        counts, cell = O.spatial_histogram_counts(O.elbp(im), 8, (8, 8))
        assert np.array_equal(counts.reshape(-1) / float(cell), g[f"hist_{nm}_r1p8_g8"])


@pytest.mark.parametrize("s", ["d3", "d99", "hist"])
def test_oracle_distances_and_nn(golden, s):
    d = golden("dist_golden.npz")
    for m in ("EuclideanDistance", "CosineDistance", "ChiSquareDistance"):
        key = f"{s}_{m}_D"
        if key not in d.files:
            continue
        D = O.pairwise(m, d[s + "_Q"], d[s + "_G"])
        np.testing.assert_allclose(D, d[key], rtol=1e-13, atol=1e-13)
        for k in (1, 3, 5):
            for qi, q in enumerate(d[s + "_Q"]):
                p, _ = O.nn_predict_faithful(list(d[s + "_G"]), d[s + "_y"], q, m, k)
                assert p[0] == d[f"{s}_{m}_k{k}_label"][qi]
                assert np.array_equal(p[1]["labels"], d[f"{s}_{m}_k{k}_labels"][qi])
                assert np.array_equal(p[1]["distances"], d[f"{s}_{m}_k{k}_dists"][qi])


def test_oracle_fisherfaces_bit_exact(golden):
    f = golden("individuals_faces.npz")
    r = O.fisherfaces_compute(list(f["X"]), f["y"])
    assert np.array_equal(np.asarray(r["W"]), f["W"])
    assert np.array_equal(r["eigenvalues"], f["eigenvalues"])
    feats = np.stack([np.asarray(x).ravel() for x in r["features"]])
    assert np.array_equal(feats, f["features"])
    assert np.array_equal(np.asarray(r["pca"]["mean"]).ravel(), f["pca_mean"])


def test_oracle_pickled_model_predictions(golden):
    f = golden("individuals_faces.npz")
    m = golden("individuals_model.npz")
    G = list(m["gallery"])
    for x, lab, dist in zip(f["X"], f["pkl_pred_labels"], f["pkl_pred_dist"]):
        q = O.fisherfaces_project(m["W"], x)
        p, _ = O.nn_predict_faithful(G, m["labels"], q, "EuclideanDistance", 1)
        assert p[0] == lab
        assert p[1]["distances"][0] == pytest.approx(dist, rel=1e-12)
