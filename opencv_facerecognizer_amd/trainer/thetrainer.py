"""Training driver (reference ``src/ocvfacerec/trainer/thetrainer.py``).

``ExtendedPredictableModel`` (thetrainer.py:51-61) is the class every pickled model is an
instance of.  ``TheTrainer`` keeps the reference's constructor and methods, so
``bin/ocvf_recognizer*.py -t`` and the interactive trainer (ocvf_interactive_trainer.py:199-207)
run unchanged:

* ``read_images`` (:72-111): same walk (``os.walk`` order, one label per non-empty folder, files
  in ``os.listdir`` order), same return value ``[X, y, folder_names]`` and error handling.  Each
  file is decoded as ``cv2.imread(IMREAD_GRAYSCALE)`` would (``ingest.imread_gray``: cv2 when
  importable, else the libjpeg luma plane / OpenCV grey weights); the ``cv2.resize`` calls become
  ONE device launch over the whole dataset (``ingest.faces``, OpenCV's INTER_LINEAR fixed point).
* ``get_model`` (:113-124): Fisherfaces + 1-NN Euclidean.
* ``train`` (:142-179): dataset check, optional k-fold validation with the ``facerec`` logger on
  stdout, ``model.compute``, ``save_model``.
* ``train_arrays``: the compute + save part of ``train`` for already-decoded face tensors.
"""
from __future__ import annotations

import logging
import os
import sys

import numpy as np

from .. import ingest
from ..facerec.classifier import NearestNeighbor
from ..facerec.distance import EuclideanDistance
from ..facerec.feature import Fisherfaces
from ..facerec.model import PredictableModel
from ..facerec.serialization import save_model
from ..facerec.validation import KFoldCrossValidation


class ExtendedPredictableModel(PredictableModel):
    """thetrainer.py:51-61: PredictableModel + image_size + subject_names."""

    def __init__(self, feature, classifier, image_size, subject_names):
        PredictableModel.__init__(self, feature=feature, classifier=classifier)
        self.image_size = image_size
        self.subject_names = subject_names


class TheTrainer(object):
    def __init__(self, _data_set, _image_size, _model_filename, _numfolds=None):
        self.dataset = _data_set
        self.image_size = _image_size
        self.model_filename = _model_filename
        self.numfolds = _numfolds

    @staticmethod
    def read_images(path, image_size=None):
        """thetrainer.py:72-111 -> [X (list of uint8 (h, w) arrays), y (labels), folder_names]."""
        label = 0
        decoded, y, folder_names = [], [], []
        for dirname, dirnames, _ in os.walk(path):
            for subdirname in dirnames:
                subject_path = os.path.join(dirname, subdirname)
                if not os.listdir(subject_path):          # only folders that hold something
                    continue
                folder_names.append(subdirname)
                for filename in os.listdir(subject_path):
                    try:
                        decoded.append(ingest.imread_gray(os.path.join(subject_path, filename)))
                        y.append(label)
                    except IOError as e:                   # :105-106 (report, skip the file)
                        print(">> I/O error({0}): {1}".format(e.errno, e.strerror))
                    except Exception:                      # :107-109 (an undecodable file)
                        print(">> Unexpected error:", sys.exc_info()[0])
                        raise
                label += 1
        # the per-file cv2.resize / colour conversion of :99-103 as one device batch
        X = [g for g, _ in decoded]
        need = [i for i, (g, c) in enumerate(decoded) if c is not None or
                (image_size is not None and g.shape[::-1] != tuple(image_size))]
        if need:
            src = [decoded[i][0] if decoded[i][1] is None else decoded[i][1] for i in need]
            if image_size is not None:
                out = ingest.faces(src, image_size, ingest.INTER_LINEAR, host=True)
                for j, i in enumerate(need):
                    X[i] = out[j]
            else:   # colour images kept at their size: grey conversion only
                for j, i in enumerate(need):
                    X[i] = ingest.faces([src[j]], (src[j].shape[1], src[j].shape[0]), host=True)[0]
        return [[np.asarray(x, dtype=np.uint8) for x in X], y, folder_names]

    @staticmethod
    def get_model(image_size, subject_names):
        """thetrainer.py:113-124: Fisherfaces + 1-NN with Euclidean distance."""
        feature = Fisherfaces()
        classifier = NearestNeighbor(dist_metric=EuclideanDistance(), k=1)
        return ExtendedPredictableModel(feature=feature, classifier=classifier, image_size=image_size,
                                        subject_names=subject_names)

    def read_subject_names(path):
        """thetrainer.py:126-140 (declared without self in the reference; call it on the class)."""
        folder_names = []
        for _, dirnames, _ in os.walk(path):
            folder_names.extend(dirnames)
        return folder_names

    def train(self):
        """thetrainer.py:142-179."""
        if not os.path.exists(self.dataset):
            print(">> [Error] No Dataset Found at '%s'." % self.dataset)
            sys.exit(1)
        print(">> Loading Dataset <-- " + self.dataset)
        images, labels, subject_names = self.read_images(self.dataset, self.image_size)
        subject_dictionary = dict(zip(list(range(max(labels) + 1)), subject_names))
        model = self.get_model(image_size=self.image_size, subject_names=subject_dictionary)
        if self.numfolds is not None:
            print(">> Validating Model With %s Folds.." % self.numfolds)
            handler = logging.StreamHandler(sys.stdout)
            handler.setFormatter(logging.Formatter('%(asctime)s - %(name)s - %(levelname)s - %(message)s'))
            logger = logging.getLogger("facerec")
            logger.addHandler(handler)
            logger.setLevel(logging.DEBUG)
            crossval = KFoldCrossValidation(model, k=self.numfolds)
            crossval.validate(images, labels)
            crossval.print_results()
        print(">> Computing Model..")
        model.compute(images, labels)
        print(">> Saving Model..")
        save_model(self.model_filename, model)
        return model

    def train_arrays(self, images, labels, subject_names):
        """thetrainer.py:150-179 from decoded uint8 face tensors (labels 0..c-1)."""
        labels = list(labels)
        subject_dictionary = dict(zip(list(range(max(labels) + 1)), subject_names))
        model = self.get_model(image_size=self.image_size, subject_names=subject_dictionary)
        model.compute([np.asarray(x, dtype=np.uint8) for x in images], labels)
        save_model(self.model_filename, model)
        return model


ExtendedPredictableModel.__module__ = "ocvfacerec.trainer.thetrainer"
TheTrainer.__module__ = "ocvfacerec.trainer.thetrainer"
