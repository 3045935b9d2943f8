"""Alias: ocvfacerec.trainer.thetrainer is opencv_facerecognizer_amd.trainer.thetrainer."""
import importlib as _importlib
import sys as _sys

_mod = _importlib.import_module("opencv_facerecognizer_amd.trainer.thetrainer")
_sys.modules[__name__ + ".thetrainer"] = _mod
thetrainer = _mod
