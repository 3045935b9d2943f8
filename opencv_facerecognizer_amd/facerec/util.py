"""Matrix builders (reference ``src/ocvfacerec/facerec/util.py``).

``as_column_matrix`` / ``as_row_matrix`` (util.py:53-84) keep their results
(np.matrix of the input dtype) but build them with one stack instead of the
reference's O(N^2) ``np.append`` loop (util.py:82-83).  The device hot path
does not go through them: the features and classifiers upload stacked rows
directly.  read_image / minmax / zscore / shuffle are out of scope.
"""
from __future__ import annotations

import numpy as np


def as_row_matrix(X):
    """util.py:53-67: N x D matrix, rows = flattened items."""
    if len(X) == 0:
        return np.array([])
    return np.asmatrix(np.stack([np.asarray(x).reshape(-1) for x in X]).astype(np.asarray(X[0]).dtype, copy=False))


def as_column_matrix(X):
    """util.py:70-84: D x N matrix, columns = flattened items."""
    if len(X) == 0:
        return np.array([])
    return np.asmatrix(np.stack([np.asarray(x).reshape(-1) for x in X], axis=1).astype(np.asarray(X[0]).dtype,
                                                                                     copy=False))
