"""Model persistence: the reference pickle loads through the non-executing reader; nothing else does."""
import io
import os
import pickle

import numpy as np
import pytest

from opencv_facerecognizer_amd.facerec import _safepickle
from ocvfacerec.facerec.serialization import load_model, loads_model, save_model

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_load_reference_pickle_layout(golden):
    m = load_model(os.path.join(GOLDEN, "individuals.pkl"))
    from ocvfacerec.trainer.thetrainer import ExtendedPredictableModel
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    assert isinstance(m, ExtendedPredictableModel)
    assert isinstance(m.feature, Fisherfaces) and isinstance(m.classifier, NearestNeighbor)
    assert isinstance(m.classifier.dist_metric, EuclideanDistance)
    ref = golden("individuals_model.npz")
    assert m.image_size == (70, 70)
    assert m.subject_names == {0: "dennis", 1: "linus", 2: "bill", 3: "steve"}
    assert isinstance(m.feature._eigenvectors, np.matrix) and m.feature._eigenvectors.dtype == np.float64
    assert np.array_equal(np.asarray(m.feature._eigenvectors), ref["W"])
    assert m.feature._eigenvalues.dtype == np.float32 and np.array_equal(m.feature._eigenvalues, ref["eigenvalues"])
    assert len(m.classifier.X) == 31 and all(isinstance(x, np.matrix) and x.shape == (3, 1) for x in m.classifier.X)
    assert np.array_equal(np.stack([np.asarray(x).ravel() for x in m.classifier.X]), ref["gallery"])
    assert np.array_equal(m.classifier.y, ref["labels"]) and m.classifier.k == 1
    assert repr(m.classifier.dist_metric) == "EuclideanDistance"


def test_save_load_roundtrip(tmp_path):
    m = load_model(os.path.join(GOLDEN, "individuals.pkl"))
    m.classifier.__dict__["_dev"] = ("not", "pickled")   # derived device state must be dropped
    p = tmp_path / "m.pkl"
    save_model(str(p), m)
    raw = p.read_bytes()
    assert b"ocvfacerec.trainer.thetrainer" in raw and b"_dev" not in raw
    m2 = load_model(str(p))
    assert np.array_equal(np.asarray(m2.feature._eigenvectors), np.asarray(m.feature._eigenvectors))
    assert m2.subject_names == m.subject_names and np.array_equal(m2.classifier.y, m.classifier.y)
    # the stdlib unpickler resolves the same classes through the ocvfacerec alias package
    m3 = pickle.loads(raw)
    assert type(m3) is type(m)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


@pytest.mark.parametrize("proto", [0, 2, 4])
def test_refuses_arbitrary_callables(proto):
    with pytest.raises(_safepickle.UnpicklingError):
        loads_model(pickle.dumps(_Evil(), protocol=proto))
    with pytest.raises(_safepickle.UnpicklingError):
        loads_model(pickle.dumps({"x": io.BytesIO}, protocol=proto))


def test_parse_numpy_payloads_all_protocols():
    obj = {"a": np.arange(6, dtype=np.float32).reshape(2, 3), "b": np.asmatrix(np.eye(2)), "c": [1, 2.5, "x"],
           "e": np.array([1, 2], dtype=">i4")}
    for proto in range(0, 6):
        r = _safepickle.loads(pickle.dumps(obj, protocol=proto), {})
        assert np.array_equal(r["a"], obj["a"]) and r["a"].dtype == np.float32
        assert isinstance(r["b"], np.matrix)
        assert r["c"] == obj["c"] and list(r["e"]) == [1, 2]


def _globals(raw):
    import pickletools
    return {tuple(a.split(" ", 1)) for op, a, _ in pickletools.genops(raw) if op.name == "GLOBAL"}


@pytest.mark.parametrize("proto", [0, 2])
def test_save_writes_numpy1_globals(tmp_path, proto):
    """A saved model names numpy the way the reference's individuals.pkl does (numpy 1.x / Python 2
    consumers cannot import numpy 2's numpy._core) and still loads here, safely and with pickle."""
    m = load_model(os.path.join(GOLDEN, "individuals.pkl"))
    p = tmp_path / "m.pkl"
    save_model(str(p), m, protocol=proto)
    raw = p.read_bytes()
    assert b"numpy._core" not in raw
    g = _globals(raw)
    assert ("numpy.core.multiarray", "_reconstruct") in g and ("numpy.matrixlib.defmatrix", "matrix") in g
    ref = open(os.path.join(GOLDEN, "individuals.pkl"), "rb").read()
    for mod, name in [("numpy.core.multiarray", "_reconstruct"), ("numpy.matrixlib.defmatrix", "matrix"),
                      ("ocvfacerec.facerec.feature", "Fisherfaces")]:
        assert f"c{mod}\n{name}\n".encode() in ref
    assert all(mod.split(".")[0] in ("numpy", "ocvfacerec", "copy_reg", "__builtin__", "_codecs") for mod, _ in g), g
    m2 = load_model(str(p))
    assert np.array_equal(np.asarray(m2.feature._eigenvectors), np.asarray(m.feature._eigenvectors))
    assert np.array_equal(np.stack([np.asarray(x).ravel() for x in m2.classifier.X]),
                          np.stack([np.asarray(x).ravel() for x in m.classifier.X]))
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)
        m3 = pickle.loads(raw)
    assert isinstance(m3.classifier.X[0], np.matrix)
