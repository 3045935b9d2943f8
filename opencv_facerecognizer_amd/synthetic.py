"""Synthetic face tensors for the benchmarks, generated on the device.

Identity prototype = a coarse N(0,1) grid (13x13) bilinearly upsampled to
HxW, x40 + 128; an image of that identity = prototype + N(0,12) pixel noise
+ U(-10,10) brightness, rounded and clipped to uint8.  Image j of the gallery
shows identity j // per_id.  Queries are fresh images of uniformly drawn
identities from a disjoint seed stream.  Everything is a pure function of
(seed, index) so every rank of a sharded run generates identical data.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

SEED = 20261015


def _gen(seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


class IdentityBank:
    """Caches coarse grids of all identities on the device for fast batch generation."""

    def __init__(self, n_ids, H, W, seed=SEED, device="cuda"):
        self.H, self.W, self.device, self.n_ids = H, W, device, int(n_ids)
        g = _gen(seed, device)
        self.grids = torch.randn((n_ids, 1, 13, 13), generator=g, device=device, dtype=torch.float32)

    def images(self, ids, seed, noise=12.0):
        """ids: int64 device tensor -> uint8 [len(ids)][H*W] images (pixel noise N(0, noise^2); the
        bench's stress runs raise it to crowd the identities together).  Ids outside 0 .. n_ids - 1
        raise ValueError on the host (an out-of-range gather of the grids would fault the device)."""
        if len(ids) and (int(ids.min()) < 0 or int(ids.max()) >= self.n_ids):
            raise ValueError(f"identity ids must lie in 0..{self.n_ids - 1} (got {int(ids.min())}..{int(ids.max())})")
        g = _gen(seed, self.device)
        up = F.interpolate(self.grids[ids], size=(self.H, self.W), mode="bilinear", align_corners=False)[:, 0]
        noise = torch.randn(up.shape, generator=g, device=self.device) * float(noise)
        bright = (torch.rand((len(ids), 1, 1), generator=g, device=self.device) * 20.0 - 10.0)
        img = torch.clamp(torch.round(up * 40.0 + 128.0 + noise + bright), 0, 255).to(torch.uint8)
        return img.reshape(len(ids), -1)


def build_projection(D, d, device):
    """Random W (no trained checkpoint exists at this scale): N(0, 1/D), prepared for the exact int8
    projection kernel.  Returns (Projection, W^T fp32 device [d][D])."""
    from ._device import Projection
    g = torch.Generator(device=device)
    g.manual_seed(SEED + 5)
    Wt = torch.randn((d, D), generator=g, device=device) / np.sqrt(D)
    return Projection(Wt_device=Wt, D=D, device=device), Wt


def build_trained_projection(bank, per_id, n_train, D, device, num_components=0, group=None):
    """The Fisherfaces W the reference's trainer would produce (thetrainer.py:120-124: Fisherfaces()
    defaults) from the synthetic training set of configs[1]: the n_train faces of gallery_chunks' rows
    0 .. n_train - 1 of an n_train-image gallery (identity j // per_id, labels 0..c-1), trained on the
    device (feature.fisherfaces_device: pixel regime at 100k x 10,000).  With torch.distributed
    initialised, rank 0 trains and W is broadcast (every rank must project with the same bits).
    Returns (Projection, W^T device fp64 [d][D], info dict)."""
    import time
    import torch.distributed as dist
    from ._device import Projection
    from .facerec.feature import fisherfaces_device
    n_ids = -(-n_train // per_id)
    _check_ids(bank, n_ids)
    sharded = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    t0 = time.perf_counter()
    info = {}
    if not sharded or dist.get_rank(group) == 0:
        X = torch.empty((n_train, D), dtype=torch.uint8, device=device)
        for c0 in range(0, n_train, GALLERY_CHUNK):
            rows = torch.arange(c0, min(c0 + GALLERY_CHUNK, n_train), device=device)
            X[c0:c0 + len(rows)] = bank.images(rows // per_id, seed=SEED + 1000 + c0 // GALLERY_CHUNK)
        y = np.arange(n_train) // per_id
        evals, Wd, m, regime = fisherfaces_device(X, D, y, num_components)
        del X
        Wt = Wd.t().contiguous()
        del Wd
        info = {"regime": regime, "n_train": n_train, "identities": n_ids, "d": m,
                "eigenvalues_head": [float(v) for v in np.asarray(evals)[:4]]}
    if sharded:
        shape = torch.zeros(2, dtype=torch.int64, device=device)
        if dist.get_rank(group) == 0:
            shape[0], shape[1] = Wt.shape[0], Wt.shape[1]
        dist.broadcast(shape, 0, group=group)
        if dist.get_rank(group) != 0:
            Wt = torch.empty((int(shape[0]), int(shape[1])), dtype=torch.float64, device=device)
        dist.broadcast(Wt, 0, group=group)
    torch.cuda.synchronize(device)
    info["train_s"] = time.perf_counter() - t0
    return Projection(Wt_device=Wt, D=D, device=device), Wt, info


def _check_ids(bank, n_ids):
    """Identity indices past the bank would index its device grids out of bounds: refuse on the host."""
    if n_ids > bank.n_ids:
        raise ValueError(f"{n_ids} identities requested from a bank of {bank.n_ids}")


GALLERY_CHUNK = 8192


def gallery_centre(P, bank, per_id, N, device, noise=12.0):
    """c = W^T round(mean image of the gallery's first chunk), fp64 [d] (the same on every rank)."""
    from ._device import col_mean_u8
    rows = torch.arange(0, min(N, GALLERY_CHUNK), device=device)
    m = col_mean_u8(bank.images(rows // per_id, seed=SEED + 1000, noise=noise), P.D)
    m_img = torch.clamp(torch.round(m), 0, 255).to(torch.uint8).reshape(1, -1).contiguous()
    return P.project(m_img, f64=True)[0].contiguous()


def gallery_chunks(P, bank, per_id, n0, n1, N, centre, noise=12.0, f64=False):
    """Yield (row0, rows) over rows [n0, n1) of the N-image synthetic gallery: the faces of each
    piece projected exactly and centred on `centre` (fp32 search rows [n][ldy], or fp64 [n][d] with
    f64).  Row j shows identity j // per_id; its pixel noise comes from chunk j // GALLERY_CHUNK,
    generated whole (rows [cb, min(cb + GALLERY_CHUNK, N)), seed SEED + 1000 + j // GALLERY_CHUNK: the
    device generator's values depend on the tensor size), so every shard holds exactly the rows of
    the unsharded gallery."""
    c0 = n0
    while c0 < n1:
        cb = c0 // GALLERY_CHUNK * GALLERY_CHUNK
        c1 = min(n1, cb + GALLERY_CHUNK)
        rows = torch.arange(cb, min(cb + GALLERY_CHUNK, N), device=centre.device)
        imgs = bank.images(rows // per_id, seed=SEED + 1000 + cb // GALLERY_CHUNK, noise=noise)
        yield c0, P.project(imgs[c0 - cb:c1 - cb].contiguous(), shift64=centre, f64=f64)
        c0 = c1


def build_gallery(P, bank, per_id, n0, nl, N, d, ld, device, noise=12.0):
    """Gallery rows [n0, n0 + nl) of the N-image synthetic gallery (a FloatGallery shard with
    index_base n0), centred on gallery_centre (fp64, the same on every rank)."""
    from . import _lib
    from ._device import FloatGallery
    _check_ids(bank, -(-N // per_id))
    if not (0 <= n0 and nl >= 0 and n0 + nl <= N):
        raise ValueError(f"gallery rows [{n0}, {n0 + nl}) outside the {N}-image gallery")
    centre = gallery_centre(P, bank, per_id, N, device, noise)
    G = torch.zeros((nl, ld), dtype=torch.float32, device=device)
    for c0, Y in gallery_chunks(P, bank, per_id, n0, n0 + nl, N, centre, noise):
        G[c0 - n0:c0 - n0 + Y.shape[0], :Y.shape[1]] = Y
    g = FloatGallery.from_device_rows(G, d, _lib.METRIC_EUCLIDEAN, shift64=centre)
    g.index_base = n0
    return g
