"""opencv_facerecognizer_amd — MI355X (gfx950) implementation of the ocvfacerec
(bytefish facerec) recognition hot path.

The reference's module layout is mirrored under ``opencv_facerecognizer_amd.facerec``
and ``opencv_facerecognizer_amd.trainer``; the top-level ``ocvfacerec`` package
aliases them so reference callers (``from ocvfacerec.facerec.model import
PredictableModel``) and pickles (``ocvfacerec.facerec.feature.Fisherfaces``)
resolve to these classes.  Compute runs in libocvf_hip.so (include/ofr.h).
"""
__version__ = "0.1.0"
