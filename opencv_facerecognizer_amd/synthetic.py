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
        self.H, self.W, self.device = H, W, device
        g = _gen(seed, device)
        self.grids = torch.randn((n_ids, 1, 13, 13), generator=g, device=device, dtype=torch.float32)

    def images(self, ids, seed, noise=12.0):
        """ids: int64 device tensor -> uint8 [len(ids)][H*W] images (pixel noise N(0, noise^2); the
        bench's stress runs raise it to crowd the identities together)."""
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
    centre = gallery_centre(P, bank, per_id, N, device, noise)
    G = torch.zeros((nl, ld), dtype=torch.float32, device=device)
    for c0, Y in gallery_chunks(P, bank, per_id, n0, n0 + nl, N, centre, noise):
        G[c0 - n0:c0 - n0 + Y.shape[0], :Y.shape[1]] = Y
    g = FloatGallery.from_device_rows(G, d, _lib.METRIC_EUCLIDEAN, shift64=centre)
    g.index_base = n0
    return g
