"""Local binary patterns (reference ``src/ocvfacerec/facerec/lbp.py``).

``ExtendedLBP`` (lbp.py:75-137) keeps its interface (``__call__(X)`` ->
uint32 code image, ``neighbors``, ``radius``) and pickled state
(``_neighbors``, ``_radius``).  The sampling geometry is derived on the host
exactly as the reference derives it (np.sin/np.cos, lbp.py:84-121); the codes
are computed by the ``ofr_elbp_codes`` kernel, which reproduces the
reference's float64 interpolation order bit for bit (see ofr_lbp.hip).

Out of scope: OriginalLBP, VarLBP, LPQ (lbp.py:55-72, 140-318) — not on the
hot path.
"""
from __future__ import annotations

import numpy as np


class LocalDescriptor(object):
    """lbp.py:40-52."""

    def __init__(self, neighbors):
        self._neighbors = neighbors

    def __call__(self, X):
        raise NotImplementedError("Every LBPOperator must implement the __call__ method.")

    @property
    def neighbors(self):
        return self._neighbors

    def __repr__(self):
        return "LBPOperator (neighbors=%s)" % (self._neighbors)


def elbp_geometry(radius, neighbors):
    """lbp.py:84-121: ((oy, ox), (by, bx), offsets int32 [P,4] = (fy, fx, cy, cx), weights fp64 [P,4])."""
    angles = 2 * np.pi / neighbors
    theta = np.arange(0, 2 * np.pi, angles)
    sample_points = np.array([-np.sin(theta), np.cos(theta)]).T
    sample_points *= radius
    miny = min(sample_points[:, 0])
    maxy = max(sample_points[:, 0])
    minx = min(sample_points[:, 1])
    maxx = max(sample_points[:, 1])
    blocksizey = np.ceil(max(maxy, 0)) - np.floor(min(miny, 0)) + 1
    blocksizex = np.ceil(max(maxx, 0)) - np.floor(min(minx, 0)) + 1
    origy = 0 - np.floor(min(miny, 0))
    origx = 0 - np.floor(min(minx, 0))
    offs = np.zeros((len(sample_points), 4), np.int32)
    wts = np.zeros((len(sample_points), 4), np.float64)
    for i, p in enumerate(sample_points):
        y, x = p + (origy, origx)
        fx, fy = np.floor(x), np.floor(y)
        cx, cy = np.ceil(x), np.ceil(y)
        ty, tx = y - fy, x - fx
        wts[i] = ((1 - tx) * (1 - ty), tx * (1 - ty), (1 - tx) * ty, tx * ty)
        offs[i] = (fy, fx, cy, cx)
    return (int(origy), int(origx)), (int(blocksizey), int(blocksizex)), offs, wts


def as_u8_images(X):
    """Image or stack of images -> uint8 array; values must already be integers in [0, 255]."""
    X = np.asanyarray(X)
    if X.dtype == np.uint8:
        return X
    if X.dtype.kind in "iub" or X.dtype.kind == "f":
        Xi = X.astype(np.uint8)
        if np.array_equal(Xi.astype(X.dtype), X):
            return Xi
    raise NotImplementedError("ExtendedLBP (MI355X build) accepts 8-bit grey images (integer values 0..255)")


class ExtendedLBP(LocalDescriptor):
    """lbp.py:75-137 on the GPU."""

    def __init__(self, radius=1, neighbors=8):
        LocalDescriptor.__init__(self, neighbors=neighbors)
        self._radius = radius

    def geometry(self):
        return elbp_geometry(self._radius, self._neighbors)

    def __call__(self, X):
        from .. import _device
        X = as_u8_images(X)
        if X.ndim != 2:
            raise ValueError("ExtendedLBP expects a 2-D image")
        codes = _device.elbp_codes(_device.u8_images(X[None]), self.geometry())
        return codes.cpu().numpy()[0].view(np.uint32)

    def codes_batch(self, imgs_u8_device):
        """uint8 [n][H][W] device tensor -> int32-stored uint32 codes [n][dy][dx] (device)."""
        from .. import _device
        return _device.elbp_codes(imgs_u8_device, self.geometry())

    @property
    def radius(self):
        return self._radius

    def __repr__(self):
        return "ExtendedLBP (neighbors=%s, radius=%s)" % (self._neighbors, self._radius)


for _c in (LocalDescriptor, ExtendedLBP):
    _c.__module__ = "ocvfacerec.facerec.lbp"
