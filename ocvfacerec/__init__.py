"""Alias of the reference package name: ``ocvfacerec.facerec.*`` and
``ocvfacerec.trainer.thetrainer`` resolve to the MI355X implementation in
``opencv_facerecognizer_amd`` (same module objects, so pickles written by either
name load into the same classes)."""
