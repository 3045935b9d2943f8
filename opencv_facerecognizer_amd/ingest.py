"""Face-tensor ingestion on the device.

The reference turns pictures into the uint8 face tensors of the hot path with OpenCV on the host,
one image per call:
* training, ``TheTrainer.read_images`` (trainer/thetrainer.py:99-103):
  ``cv2.imread(f, IMREAD_GRAYSCALE)`` then ``cv2.resize(im, image_size)`` (INTER_LINEAR);
* recognition (bin/ocvf_recognizer.py:64-66, _ros.py:113-115, _rsb.py): per detected face
  ``img[y0:y1, x0:x1]`` -> ``cv2.cvtColor(BGR2GRAY)`` -> ``cv2.resize(size, INTER_CUBIC)``.

Here decoding stays on the host (a JPEG/PNG decoder, as in the reference), and every crop,
grey conversion and resize of a batch -- images of any sizes -- is ONE launch of
``ofr_ingest_faces`` writing ``uint8 [n][h][w]`` rows straight into device memory, where
``PredictableModel.predict_batch`` / ``compute`` read them without a host round trip.  The
arithmetic is OpenCV's 8-bit fixed point (restated in ``oracle/facerec_oracle.py``; parity with
cv2 itself is unpinned, cv2 is absent from this image -- see DESIGN.md).

``imread_gray`` mirrors ``cv2.imread(path, IMREAD_GRAYSCALE)``: cv2 when it is importable;
otherwise PIL -- JPEGs decoded straight to their luma plane (libjpeg grayscale output, what
OpenCV's JPEG reader asks libjpeg for) and other formats decoded to BGR and converted with
OpenCV's integer grey weights on the device.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream

INTER_LINEAR = 1   # cv2.INTER_LINEAR
INTER_CUBIC = 2    # cv2.INTER_CUBIC
_MODES = {"linear": INTER_LINEAR, "cubic": INTER_CUBIC, INTER_LINEAR: INTER_LINEAR, INTER_CUBIC: INTER_CUBIC}


def _cv2():
    try:
        import cv2  # noqa: F401
    except ImportError:
        return None
    return cv2


def _channels(a):
    if a.ndim == 2:
        return 1
    if a.ndim == 3 and a.shape[2] in (3, 4):
        return a.shape[2]
    raise ValueError(f"image of shape {a.shape}: expected (H, W) grey or (H, W, 3|4) BGR(A)")


def faces(images, size, interpolation=INTER_LINEAR, boxes=None, device=None, host=False):
    """Crop + grey + resize a batch in one launch.

    images: list of uint8 host arrays, (H, W) grey or (H, W, 3|4) BGR(A) -- any sizes.
    size: (width, height), cv2's dsize order.  boxes: None (every image whole) or a list of
    (image index, x0, y0, x1, y1) crops (``img[y0:y1, x0:x1]``), one output face each.
    Returns uint8 [n][height][width] on the device (or host numpy with host=True)."""
    mode = _MODES[interpolation]
    dw, dh = int(size[0]), int(size[1])
    if dw < 1 or dh < 1:
        raise ValueError("size must be positive (width, height)")
    device = device or _lib.device()
    arrs = [np.ascontiguousarray(np.asarray(a)) for a in images]
    for a in arrs:
        if a.dtype != np.uint8:
            raise TypeError("images must be uint8")
    if boxes is None:
        boxes = [(i, 0, 0, a.shape[1], a.shape[0]) for i, a in enumerate(arrs)]
    n = len(boxes)
    out = torch.empty((n, dh, dw), dtype=torch.uint8, device=device)
    if n == 0:
        return out.cpu().numpy() if host else out
    offs = np.zeros(len(arrs) + 1, np.int64)
    offs[1:] = np.cumsum([a.nbytes for a in arrs])
    jobs = np.empty((n, 7), np.int64)
    for j, (i, x0, y0, x1, y1) in enumerate(boxes):
        a = arrs[i]
        H, W, ch = a.shape[0], a.shape[1], _channels(a)
        if not (0 <= x0 < x1 <= W and 0 <= y0 < y1 <= H):
            raise ValueError(f"crop {(x0, y0, x1, y1)} outside image {i} of size {W}x{H}")
        jobs[j] = (offs[i], W * ch, x0, y0, x1 - x0, y1 - y0, ch)
    flat = np.empty(int(offs[-1]), np.uint8)
    for i, a in enumerate(arrs):
        flat[offs[i]:offs[i + 1]] = a.reshape(-1)
    src = torch.from_numpy(flat).pin_memory().to(device, non_blocking=True)
    jobs_d = torch.from_numpy(jobs).to(device)
    call("ofr_ingest_faces", stream(), ptr(src), ptr(jobs_d), n, dh, dw, mode, ptr(out))
    return out.cpu().numpy() if host else out


def imread_gray(path):
    """cv2.imread(path, IMREAD_GRAYSCALE) -> (uint8 (H, W) grey array, None) or, for a colour
    non-JPEG decoded without cv2, (None, uint8 (H, W, 3) BGR array) still to be converted.
    Raises ValueError when the file cannot be decoded (cv2.imread returns None there, and the
    reference's next call on it raises, thetrainer.py:99-109)."""
    cv2 = _cv2()
    if cv2 is not None:
        im = cv2.imread(path, cv2.IMREAD_GRAYSCALE)
        if im is None:
            raise ValueError(f"cannot decode image {path!r}")
        return np.asarray(im, dtype=np.uint8), None
    from PIL import Image
    try:
        with Image.open(path) as im:
            if im.format == "JPEG":
                im.draft("L", im.size)                 # libjpeg's grayscale output = the luma plane
                return np.asarray(im.convert("L"), dtype=np.uint8), None
            if im.mode in ("I;16", "I"):               # 16-bit grey: OpenCV keeps the high byte
                return (np.asarray(im, dtype=np.uint32) >> 8).astype(np.uint8), None
            if im.mode in ("L", "1"):
                return np.asarray(im.convert("L"), dtype=np.uint8), None
            rgb = np.asarray(im.convert("RGB"), dtype=np.uint8)
    except (OSError, SyntaxError, ValueError) as e:
        raise ValueError(f"cannot decode image {path!r}: {e}") from e
    return None, np.ascontiguousarray(rgb[..., ::-1])


def read_faces(paths, image_size=None, interpolation=INTER_LINEAR):
    """Decode files as IMREAD_GRAYSCALE and (if image_size = (width, height)) resize them all in
    one device launch.  Returns a list of uint8 host arrays (the reference's X list)."""
    grey, colour = [], []
    for p in paths:
        g, c = imread_gray(p)
        grey.append(g)
        colour.append(c)
    if image_size is None:
        out = list(grey)
        todo = [i for i, g in enumerate(grey) if g is None]
        for i in todo:                             # colour non-JPEG without cv2: grey on the device
            c = colour[i]
            out[i] = faces([c], (c.shape[1], c.shape[0]), interpolation, host=True)[0]
        return out
    src = [g if g is not None else c for g, c in zip(grey, colour)]
    if not src:
        return []
    return list(faces(src, image_size, interpolation, host=True))
