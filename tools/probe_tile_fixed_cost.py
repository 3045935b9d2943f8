"""Per-tile fixed cost of the wide fp6 sieve pass: times the sample pass + thresholds and the sieve pass
(HIP events, median of reps) for one gallery size and batch at several feature dimensions d; the
sieve time against the number of 128-feature stages extrapolates to the cost of a tile with no
stages (prologue fill + epilogue).  One JSON line per d.

    python tools/probe_tile_fixed_cost.py [--gallery 262144] [--batch 4096] [--dims 128,256,512,1024,2048]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import FloatGallery, center_round, round_up  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=262144)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dims", default="128,256,512,1024,2048")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--synthetic", action="store_true",
                    help="the bench's identity-bank faces through the projection (d = 9999) instead")
    args = ap.parse_args()
    if args.synthetic:
        return synthetic(args)
    dev = _lib.device()
    N, B = args.gallery, args.batch
    g0 = torch.Generator(device=dev)
    g0.manual_seed(7)
    for d in [int(x) for x in args.dims.split(",")]:
        ld = max(32, round_up(d, 32))
        C = torch.randn((N // 8, d), generator=g0, device=dev, dtype=torch.float64) * 20
        G = C.repeat_interleave(8, 0) + torch.randn((N, d), generator=g0, device=dev, dtype=torch.float64) * 3
        Q = C[torch.randint(0, N // 8, (B,), generator=g0, device=dev)] + \
            torch.randn((B, d), generator=g0, device=dev, dtype=torch.float64) * 3
        shift = G.mean(0)
        g = FloatGallery.from_device_rows(center_round(G, shift, ld), d, _lib.METRIC_EUCLIDEAN, shift64=shift)
        Qd = center_round(Q, shift, ld)
        qq = g.quantize_queries(Qd, tier="f6")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        samp, siev = [], []
        for r in range(args.reps + 1):
            torch.cuda.synchronize()
            ev[0].record()
            g.search_q8_phase(4, Qd, qq, 1)
            ev[1].record()
            g.search_q8_phase(8, Qd, qq, 1)
            ev[2].record()
            torch.cuda.synchronize()
            if r:
                samp.append(ev[0].elapsed_time(ev[1]))
                siev.append(ev[1].elapsed_time(ev[2]))
        tiles = -(-N // 384) * -(-B // 256)
        med = lambda v: sorted(v)[len(v) // 2]
        print(json.dumps({"d": d, "stages": -(-d // 128), "gallery": N, "batch": B, "tiles": tiles,
                          "sample_ms": med(samp), "sieve_ms": med(siev),
                          "us_per_tile_round": med(siev) * 1e3 / (tiles / 256)}), flush=True)
        del g, G, C, Q, Qd, qq
        torch.cuda.empty_cache()


def synthetic(args):
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank, build_gallery, build_projection
    dev = _lib.device()
    D, d, B, per, N = 10000, 9999, args.batch, 10, args.gallery
    P, _ = build_projection(D, d, dev)
    n_ids = -(-N // per)                       # row j shows identity j // per: every row needs one
    bank = IdentityBank(n_ids, 100, 100, device=dev)
    g = build_gallery(P, bank, per, 0, N, N, d, max(32, round_up(d, 32)), dev)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    Qd = P.project(bank.images(torch.randint(0, n_ids, (B,), generator=gq, device=dev), seed=SEED + 99),
                   shift64=g.shift64)
    qq = g.quantize_queries(Qd, tier="f6")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    siev = []
    for r in range(args.reps + 1):
        torch.cuda.synchronize()
        ev[0].record()
        g.search_q8_phase(4, Qd, qq, 1)
        ev[1].record()
        g.search_q8_phase(8, Qd, qq, 1)
        ev[2].record()
        torch.cuda.synchronize()
        if r:
            siev.append(ev[1].elapsed_time(ev[2]))
    tiles = -(-N // 384) * -(-B // 256)
    kept = g.sieve_counts(B)
    ms = sorted(siev)[len(siev) // 2]
    print(json.dumps({"d": d, "synthetic": True, "gallery": N, "batch": B, "tiles": tiles, "sieve_ms": ms,
                      "us_per_tile_round": ms * 1e3 / (tiles / 256), "kept_mean": float(kept.double().mean())}),
          flush=True)


if __name__ == "__main__":
    main()
