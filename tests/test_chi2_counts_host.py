"""Host logic of the LBPH counts gallery (no GPU): recognising SpatialHistogram float histograms
(count / cell, feature.py:298-299) as exact integer counts, and refusing anything else."""
import numpy as np

import facerec_oracle as O
from opencv_facerecognizer_amd._device import counts_of, infer_count_denom


def test_spatial_histograms_are_exact_counts():
    r = np.random.Generator(np.random.PCG64(3))
    imgs = r.integers(0, 256, (4, 128, 128), dtype=np.uint8)
    H = np.stack([O.spatial_histogram(x) for x in imgs])          # reference float64 histograms
    assert infer_count_denom(H) == 225.0
    C, cb = counts_of(H, 225.0)
    assert cb == 1 and C.dtype == np.uint8
    ref = np.stack([O.spatial_histogram_counts(O.elbp(x))[0].reshape(-1) for x in imgs])
    assert np.array_equal(C.astype(np.int64), ref)
    assert np.array_equal(C / 225.0, H)                             # bit-exact round trip


def test_non_count_rows_are_refused():
    r = np.random.Generator(np.random.PCG64(4))
    assert infer_count_denom(r.random((3, 50))) is None
    H = np.full((2, 8), 3 / 225.0)
    assert counts_of(H * (1 + 1e-9), 225.0) is None                 # not count / denom
    assert counts_of(-H, 225.0) is None
    assert counts_of(np.array([[np.nan, 0.0]]), 1.0) is None
    assert infer_count_denom(np.zeros((2, 4))) is None
    # large counts pick a wider element type
    C, cb = counts_of(np.array([[300.0, 1.0]]), 1.0)
    assert cb == 2 and C.dtype == np.uint16
    C, cb = counts_of(np.array([[70000.0, 1.0]]), 1.0)
    assert cb == 4 and C.dtype == np.uint32
    assert counts_of(np.array([[300.0]]), 1.0, count_bytes=1) is None
    # integer values past 32-bit counts are not a counts gallery (was StopIteration)
    assert counts_of(np.array([[2.0 ** 33, 1.0]]), 1.0) is None
    assert infer_count_denom(np.array([[2.0 ** 33, 1.0]])) is None
