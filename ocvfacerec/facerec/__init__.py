"""Alias: ocvfacerec.facerec.<mod> is opencv_facerecognizer_amd.facerec.<mod>."""
import importlib as _importlib
import sys as _sys

for _m in ("distance", "lbp", "feature", "operators", "classifier", "model", "util", "serialization", "validation"):
    _mod = _importlib.import_module("opencv_facerecognizer_amd.facerec." + _m)
    _sys.modules[__name__ + "." + _m] = _mod
    globals()[_m] = _mod
