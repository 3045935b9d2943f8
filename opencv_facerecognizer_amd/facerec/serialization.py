"""Model persistence (reference ``src/ocvfacerec/facerec/serialization.py:38-49``).

``save_model`` pickles the model object as the reference does (the device
caches are dropped by ``__getstate__``; classes pickle under their reference
paths ``ocvfacerec.facerec.*`` / ``ocvfacerec.trainer.thetrainer``), so a
saved model has the reference's pickled layout.

Protocols 0-2 (the ones Python 2 reads) are written with the numpy globals of
the reference's file (``numpy.core.multiarray._reconstruct``,
``numpy.matrixlib.defmatrix.matrix``) instead of numpy 2's ``numpy._core``,
which numpy 1.x -- the recognizers' Python 2 stack -- cannot import.

``load_model`` reads reference pickles (Python-2 protocol 0, e.g. the bundled
``data/individuals.pkl``) and our own with the NON-EXECUTING reader in
``_safepickle``: nothing named in the file is imported or called; only the
facerec model classes below and numpy array/matrix/dtype payloads are built.
"""
from __future__ import annotations

import pickle
import pickletools

from . import _safepickle

# numpy-2 globals -> the names numpy 1.x (and the reference's individuals.pkl) use
_NUMPY1_GLOBALS = {("numpy", "matrix"): ("numpy.matrixlib.defmatrix", "matrix")}


def _numpy1_globals(data):
    """Rewrite the GLOBAL opcodes of a protocol 0-2 pickle that name numpy-2 modules."""
    out, last = [], 0
    for op, arg, pos in pickletools.genops(data):
        if op.name != "GLOBAL":
            continue
        mod, name = arg.split(" ", 1)
        new = _NUMPY1_GLOBALS.get((mod, name))
        if new is None and (mod == "numpy._core" or mod.startswith("numpy._core.")):
            new = ("numpy.core" + mod[len("numpy._core"):], name)
        if new is not None:
            out.append(data[last:pos])
            out.append(b"c" + new[0].encode() + b"\n" + new[1].encode() + b"\n")
            last = pos + 3 + len(mod.encode()) + len(name.encode())   # 'c' module '\n' name '\n'
    out.append(data[last:])
    return b"".join(out)


def _model_classes():
    from ..trainer.thetrainer import ExtendedPredictableModel
    from . import classifier, distance, feature, lbp, model, operators
    classes = {}
    for mod in (classifier, distance, feature, lbp, model, operators):
        for name in dir(mod):
            obj = getattr(mod, name)
            if isinstance(obj, type) and getattr(obj, "__module__", "").startswith("ocvfacerec."):
                classes[f"{obj.__module__}.{obj.__name__}"] = obj
    classes["ocvfacerec.trainer.thetrainer.ExtendedPredictableModel"] = ExtendedPredictableModel
    return classes


def dumps_model(model, protocol=2):
    data = pickle.dumps(model, protocol=protocol)
    return _numpy1_globals(data) if protocol <= 2 else data


def save_model(filename, model, protocol=2):
    """serialization.py:38-41 (protocol 2 instead of cPickle's default 0; both load under Python 2)."""
    data = dumps_model(model, protocol)
    with open(filename, "wb") as output:
        output.write(data)


def loads_model(data):
    return _safepickle.loads(data, _model_classes())


def load_model(filename):
    """serialization.py:44-49, without executing anything from the file."""
    with open(filename, "rb") as pkl_file:
        res = loads_model(pkl_file.read())
    print(">> New Model Loaded")
    return res
