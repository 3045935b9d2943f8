"""Model persistence (reference ``src/ocvfacerec/facerec/serialization.py:38-49``).

``save_model`` pickles the model object as the reference does (the device
caches are dropped by ``__getstate__``; classes pickle under their reference
paths ``ocvfacerec.facerec.*`` / ``ocvfacerec.trainer.thetrainer``), so a
saved model has the reference's pickled layout.

``load_model`` reads reference pickles (Python-2 protocol 0, e.g. the bundled
``data/individuals.pkl``) and our own with the NON-EXECUTING reader in
``_safepickle``: nothing named in the file is imported or called; only the
facerec model classes below and numpy array/matrix/dtype payloads are built.
"""
from __future__ import annotations

import pickle

from . import _safepickle


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


def save_model(filename, model, protocol=2):
    """serialization.py:38-41 (protocol 2 instead of cPickle's default 0)."""
    with open(filename, "wb") as output:
        pickle.dump(model, output, protocol=protocol)


def loads_model(data):
    return _safepickle.loads(data, _model_classes())


def load_model(filename):
    """serialization.py:44-49, without executing anything from the file."""
    with open(filename, "rb") as pkl_file:
        res = loads_model(pkl_file.read())
    print(">> New Model Loaded")
    return res
