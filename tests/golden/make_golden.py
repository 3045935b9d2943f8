"""Generate the committed golden fixtures by running the REFERENCE's own code.

Run once in the build container (needs ``/root/reference``; never runs on the
GPU box):  ``python tests/golden/make_golden.py``

The reference is Python 2.7.  ``distance.py`` imports unmodified under
Python 3; the other hot-path modules need a handful of mechanical py2->py3
edits.  ``_RefImporter`` below reads each reference module's
source *from /root/reference at run time*, applies exactly those edits in
memory, and executes it as ``ocvfacerec.*`` — nothing of the reference is
written into this repository except the resulting numeric fixtures:

* ``individuals.pkl``      — the reference's bundled trained model (data file)
* ``individuals_model.npz`` — its contents (W, eigenvalues, gallery, labels)
  as read by the non-executing pickle parser
* ``individuals_faces.npz`` — the 31 bundled JPEGs decoded to 70x70 uint8
  (PIL Y-channel decode + half-pixel bilinear; NOT bit-identical to cv2,
  which is absent — these tensors are simply the fixed inputs) and the
  reference Fisherfaces.compute / predict outputs on them
* ``lbp_golden.npz``        — reference ExtendedLBP codes and SpatialHistogram
  outputs on 10 seeded images (uniform, tie-heavy, low-entropy, constant, ...)
* ``dist_golden.npz``       — reference distance.py matrices and
  NearestNeighbor.predict outputs on seeded vectors.
"""
from __future__ import annotations

import importlib.abc
import importlib.util
import os
import re
import shutil
import sys

import numpy as np

REF = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SEED = 20261015

# (module, literal-or-regex, replacement) — the py2->py3 compat edits of SURVEY.md §8c
_EDITS = {
    "ocvfacerec.facerec.util": [
        ("except IOError as (errno, strerror):", "except IOError:"),
        ('print "I/O error({0}): {1}".format(errno, strerror)', "pass"),
        ('print "Cannot open image."', "pass"),
        ("dtype=np.float)", "dtype=np.float64)"),
        ("xrange(", "range("),
    ],
    "ocvfacerec.facerec.lbp": [
        ("origy = 0 - np.floor(min(miny, 0))", "origy = int(0 - np.floor(min(miny, 0)))"),
        ("origx = 0 - np.floor(min(minx, 0))", "origx = int(0 - np.floor(min(minx, 0)))"),
        ("dx = xsize - blocksizex + 1", "dx = int(xsize - blocksizex + 1)"),
        ("dy = ysize - blocksizey + 1", "dy = int(ysize - blocksizey + 1)"),
        ("fx = np.floor(x)", "fx = int(np.floor(x))"),
        ("fy = np.floor(y)", "fy = int(np.floor(y))"),
        ("cx = np.ceil(x)", "cx = int(np.ceil(x))"),
        ("cy = np.ceil(y)", "cy = int(np.ceil(y))"),
        ("result += (1 << i) * D", "result += np.uint32(1 << i) * D"),
        ("np.float)", "np.float64)"),
    ],
    "ocvfacerec.facerec.feature": [("normed=True", "density=True")],
    "ocvfacerec.facerec.classifier": [
        ("hist.iteritems()", "hist.items()"),
        ("from StringIO import StringIO", "from io import StringIO"),
    ],
    "ocvfacerec.facerec.distance": [],
    "ocvfacerec.facerec.model": [],
    "ocvfacerec.facerec.operators": [],
}


class _RefImporter(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Serve ``ocvfacerec``, ``ocvfacerec.facerec`` and the hot-path modules from /root/reference."""

    def find_spec(self, fullname, path, target=None):
        if fullname in ("ocvfacerec", "ocvfacerec.facerec"):
            return importlib.util.spec_from_loader(fullname, self, is_package=True)
        if fullname in _EDITS:
            return importlib.util.spec_from_loader(fullname, self)
        return None

    def create_module(self, spec):
        return None

    def exec_module(self, module):
        name = module.__name__
        if name in ("ocvfacerec", "ocvfacerec.facerec"):
            module.__path__ = []
            return
        fn = os.path.join(REF, *name.split(".")) + ".py"
        src = open(fn).read()
        for a, b in _EDITS[name]:
            if a not in src:
                raise RuntimeError(f"compat edit not applicable in {fn}: {a!r}")
            src = src.replace(a, b)
        exec(compile(src, fn, "exec"), module.__dict__)


def load_reference():
    for k in list(sys.modules):
        if k == "ocvfacerec" or k.startswith("ocvfacerec."):
            del sys.modules[k]
    sys.meta_path.insert(0, _RefImporter())
    import ocvfacerec.facerec.classifier as classifier
    import ocvfacerec.facerec.distance as distance
    import ocvfacerec.facerec.feature as feature
    import ocvfacerec.facerec.lbp as lbp
    import ocvfacerec.facerec.model as model
    return dict(feature=feature, classifier=classifier, distance=distance, lbp=lbp, model=model)


# ---------------------------------------------------------------------------
def _bilinear_resize_u8(img, size):
    """Half-pixel-centre bilinear resize (cv2.INTER_LINEAR geometry, float arithmetic)."""
    w, h = size
    H, W = img.shape
    sy, sx = H / h, W / w
    ys = np.clip((np.arange(h) + 0.5) * sy - 0.5, 0, H - 1)
    xs = np.clip((np.arange(w) + 0.5) * sx - 0.5, 0, W - 1)
    y0 = np.floor(ys).astype(int)
    x0 = np.floor(xs).astype(int)
    y1 = np.minimum(y0 + 1, H - 1)
    x1 = np.minimum(x0 + 1, W - 1)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    a = img.astype(np.float64)
    top = a[y0][:, x0] * (1 - fx) + a[y0][:, x1] * fx
    bot = a[y1][:, x0] * (1 - fx) + a[y1][:, x1] * fx
    return np.clip(np.rint(top * (1 - fy) + bot * fy), 0, 255).astype(np.uint8)


def decode_faces(size=(70, 70)):
    from PIL import Image
    root = "/root/reference/data/individuals"
    names = ["dennis", "linus", "bill", "steve"]   # label order recorded in individuals.pkl
    X, y, files = [], [], []
    for c, nm in enumerate(names):
        for f in sorted(os.listdir(os.path.join(root, nm))):
            im = Image.open(os.path.join(root, nm, f))
            im.draft("L", im.size)
            g = np.asarray(im.convert("L"), dtype=np.uint8)
            X.append(_bilinear_resize_u8(g, size))
            y.append(c)
            files.append(f"{nm}/{f}")
    return np.stack(X), np.asarray(y, np.int64), names, files


def lbp_images():
    rng = np.random.Generator(np.random.PCG64(SEED))
    imgs = {}
    imgs["uniform0"] = rng.integers(0, 256, (128, 128), dtype=np.uint8)
    imgs["uniform1"] = rng.integers(0, 256, (128, 128), dtype=np.uint8)
    imgs["lowent"] = rng.integers(100, 102, (128, 128), dtype=np.uint8)          # ties everywhere
    imgs["ternary"] = (rng.integers(0, 3, (128, 128)) * 7 + 60).astype(np.uint8)
    imgs["constant"] = np.full((128, 128), 77, np.uint8)
    gy, gx = np.mgrid[0:128, 0:128]
    imgs["ramp"] = ((gx // 3 + gy // 5) % 256).astype(np.uint8)                   # plateaus + steps
    imgs["checker"] = (((gx + gy) % 2) * 255).astype(np.uint8)
    imgs["extremes"] = rng.choice(np.array([0, 255], np.uint8), (128, 128))
    imgs["odd37x53"] = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    imgs["tiny10"] = rng.integers(0, 256, (10, 10), dtype=np.uint8)
    return imgs


def main():
    sys.path.insert(0, REPO)
    from opencv_facerecognizer_amd.facerec import _safepickle

    os.makedirs(HERE, exist_ok=True)
    ref = load_reference()
    feature, classifier, distance, lbp, model = (ref[k] for k in ("feature", "classifier", "distance", "lbp", "model"))

    # ---- 1. bundled model ---------------------------------------------------
    pkl = "/root/reference/data/individuals.pkl"
    shutil.copyfile(pkl, os.path.join(HERE, "individuals.pkl"))
    Dummy = {n: type(n.rsplit(".", 1)[1], (object,), {}) for n in (
        "ocvfacerec.trainer.thetrainer.ExtendedPredictableModel", "ocvfacerec.facerec.feature.Fisherfaces",
        "ocvfacerec.facerec.classifier.NearestNeighbor", "ocvfacerec.facerec.distance.EuclideanDistance")}
    m = _safepickle.loads(open(pkl, "rb").read(), Dummy)
    W = np.asarray(m.feature._eigenvectors)
    G = np.stack([np.asarray(x).reshape(-1) for x in m.classifier.X])
    np.savez_compressed(os.path.join(HERE, "individuals_model.npz"), W=W, eigenvalues=m.feature._eigenvalues,
                        num_components=m.feature._num_components, gallery=G, labels=m.classifier.y,
                        k=m.classifier.k, image_size=np.asarray(m.image_size),
                        subject_names=np.asarray([m.subject_names[i] for i in range(len(m.subject_names))]))

    # reference objects rebuilt from the parsed state (no unpickling)
    fish = feature.Fisherfaces.__new__(feature.Fisherfaces)
    fish.__dict__.update(_eigenvectors=m.feature._eigenvectors, _eigenvalues=m.feature._eigenvalues,
                         _num_components=m.feature._num_components)
    nn = classifier.NearestNeighbor(dist_metric=distance.EuclideanDistance(), k=1)
    nn.X, nn.y = list(m.classifier.X), np.asarray(m.classifier.y)
    pkl_model = model.PredictableModel(fish, nn)

    # ---- 2. bundled faces: compute + predict -------------------------------
    X, y, names, files = decode_faces((70, 70))
    pk_labels, pk_dists = [], []
    for x in X:
        p = pkl_model.predict(x)
        pk_labels.append(p[0])
        pk_dists.append(p[1]["distances"][0])
    fm = model.PredictableModel(feature.Fisherfaces(), classifier.NearestNeighbor(distance.EuclideanDistance(), k=1))
    fm.compute(list(X), list(y))
    # the chained PCA/LDA of the reference are locals of Fisherfaces.compute: re-run them to expose them
    pca = feature.PCA(len(y) - len(np.unique(y)))
    pfeat = pca.compute(list(X), y)
    lda = feature.LDA(0)
    lda.compute(pfeat, y)
    res_labels, res_d1, res_d3, res_l3 = [], [], [], []
    for x in X:
        p = fm.predict(x)
        res_labels.append(p[0])
        res_d1.append(p[1]["distances"][0])
    fm.classifier.k = 3
    for x in X:
        p = fm.predict(x)
        res_l3.append(p[1]["labels"])
        res_d3.append(p[1]["distances"])
    np.savez_compressed(
        os.path.join(HERE, "individuals_faces.npz"), X=X, y=y, names=np.asarray(names), files=np.asarray(files),
        pkl_pred_labels=np.asarray(pk_labels), pkl_pred_dist=np.asarray(pk_dists),
        W=np.asarray(fm.feature._eigenvectors), eigenvalues=fm.feature._eigenvalues,
        num_components=fm.feature._num_components,
        features=np.stack([np.asarray(f).reshape(-1) for f in fm.classifier.X]),
        pca_mean=np.asarray(pca.mean).reshape(-1), pca_eigenvalues=pca.eigenvalues,
        pca_eigenvectors=np.asarray(pca.eigenvectors), lda_eigenvectors=np.asarray(lda.eigenvectors),
        lda_eigenvalues=lda.eigenvalues,
        pca_features=np.stack([np.asarray(f).reshape(-1) for f in pfeat]),
        resub_labels=np.asarray(res_labels), resub_dist1=np.asarray(res_d1),
        resub_labels_k3=np.asarray(res_l3), resub_dist_k3=np.asarray(res_d3))

    # ---- 3. LBP ----------------------------------------------------------------
    out = {}
    for nm, im in lbp_images().items():
        out[f"img_{nm}"] = im
        for (r, P) in ((1, 8), (2, 8), (2, 16), (3, 4)):
            out[f"codes_{nm}_r{r}p{P}"] = lbp.ExtendedLBP(radius=r, neighbors=P)(im)
        if min(im.shape) >= 18:
            out[f"hist_{nm}_r1p8_g8"] = feature.SpatialHistogram(lbp.ExtendedLBP(1, 8), (8, 8)).extract(im)
            out[f"hist_{nm}_r2p8_g4x5"] = feature.SpatialHistogram(lbp.ExtendedLBP(2, 8), (4, 5)).extract(im)
    np.savez_compressed(os.path.join(HERE, "lbp_golden.npz"), **out)

    # ---- 4. distances + NearestNeighbor --------------------------------------
    rng = np.random.Generator(np.random.PCG64(SEED + 1))
    sets = {}
    sets["d3"] = (rng.normal(0, 300, (6, 3)), rng.normal(0, 300, (40, 3)))
    Gq = rng.normal(50, 20, (60, 99))
    Gq[17] = Gq[5]                                   # exact duplicate gallery rows -> distance ties
    Qq = rng.normal(50, 20, (5, 99))
    Qq[0] = Gq[5]                                    # zero-distance query
    sets["d99"] = (Qq, Gq)
    hs = [out[f"hist_{n}_r1p8_g8"] for n in ("uniform0", "uniform1", "lowent", "ternary", "constant", "ramp",
                                             "checker", "extremes")]
    Hg = np.stack(hs + [h[::-1] for h in hs])
    sets["hist"] = (Hg[:4].copy(), Hg)
    dres = {}
    metric_cls = {"EuclideanDistance": distance.EuclideanDistance, "CosineDistance": distance.CosineDistance,
                  "ChiSquareDistance": distance.ChiSquareDistance}
    labels_all = {}
    for sname, (Q, Gs) in sets.items():
        dres[f"{sname}_Q"] = Q
        dres[f"{sname}_G"] = Gs
        y_s = np.arange(len(Gs)) % 4
        labels_all[sname] = y_s
        dres[f"{sname}_y"] = y_s
        for mname, cls in metric_cls.items():
            if sname != "hist" and mname == "ChiSquareDistance":
                continue
            met = cls()
            dres[f"{sname}_{mname}_D"] = np.array([[met(g.reshape(-1, 1), q.reshape(-1, 1)) for g in Gs] for q in Q])
            for k in (1, 3, 5):
                c = classifier.NearestNeighbor(dist_metric=met, k=k)
                c.compute([g.reshape(-1, 1) for g in Gs], y_s)
                preds = [c.predict(q.reshape(-1, 1)) for q in Q]
                dres[f"{sname}_{mname}_k{k}_label"] = np.asarray([p[0] for p in preds])
                dres[f"{sname}_{mname}_k{k}_labels"] = np.stack([p[1]["labels"] for p in preds])
                dres[f"{sname}_{mname}_k{k}_dists"] = np.stack([p[1]["distances"] for p in preds])
    np.savez_compressed(os.path.join(HERE, "dist_golden.npz"), **dres)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
