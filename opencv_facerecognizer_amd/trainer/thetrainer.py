"""Training driver glue (reference ``src/ocvfacerec/trainer/thetrainer.py``).

Kept: ``ExtendedPredictableModel`` (thetrainer.py:51-61, the class every
pickled model is an instance of) and ``TheTrainer.get_model`` (:113-124, the
hard-coded Fisherfaces + 1-NN Euclidean model) plus ``train_arrays``, the
compute + save part of ``TheTrainer.train`` (:142-179) for already-decoded
face tensors.  Image decoding (``cv2.imread`` + ``cv2.resize``, :72-111) and
k-fold validation are outside the hot path and not provided.
"""
from __future__ import annotations

import numpy as np

from ..facerec.classifier import NearestNeighbor
from ..facerec.distance import EuclideanDistance
from ..facerec.feature import Fisherfaces
from ..facerec.model import PredictableModel
from ..facerec.serialization import save_model


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
    def get_model(image_size, subject_names):
        """thetrainer.py:113-124."""
        feature = Fisherfaces()
        classifier = NearestNeighbor(dist_metric=EuclideanDistance(), k=1)
        return ExtendedPredictableModel(feature=feature, classifier=classifier, image_size=image_size,
                                        subject_names=subject_names)

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
