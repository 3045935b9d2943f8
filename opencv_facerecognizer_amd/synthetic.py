"""Synthetic face tensors for the benchmarks, generated on the device.

Identity prototype = a coarse N(0,1) grid (13x13) bilinearly upsampled to
HxW, x40 + 128; an image of that identity = prototype + N(0,12) pixel noise
+ U(-10,10) brightness, rounded and clipped to uint8.  Image j of the gallery
shows identity j // per_id.  Queries are fresh images of uniformly drawn
identities from a disjoint seed stream.  Everything is a pure function of
(seed, index) so every rank of a sharded run generates identical data.
"""
from __future__ import annotations

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
