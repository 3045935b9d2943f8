"""CosineDistance 1-NN at the headline scale (1M gallery, d = 9999, B = 4096; bench.py's synthetic
faces and projection, features NOT centred -- cosine is not translation invariant).  Times the
certified path (unit-row twin on the fp6 -> int8 -> fp32 chain, then distance.py:77 in fp64) and the
fp32-MFMA path (OFR_SEARCH=fp32).  Prints one JSON line.

    python tools/bench_cosine.py [--gallery 1000000] [--batch 4096] [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import build_projection  # noqa: E402
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import FloatGallery, round_up  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dim", type=int, default=9999)
    ap.add_argument("--per-id", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    device = _lib.device()
    D, d, N, B = 100 * 100, args.dim, args.gallery, args.batch
    P, _ = build_projection(D, d, device)
    bank = IdentityBank((N + args.per_id - 1) // args.per_id, 100, 100, device=device)
    ld = max(32, round_up(d, 32))
    G = torch.zeros((N, ld), dtype=torch.float32, device=device)
    for c0 in range(0, N, 8192):
        c1 = min(N, c0 + 8192)
        rows = torch.arange(c0, c1, device=device)
        P.project(bank.images(rows // args.per_id, seed=SEED + 1000 + c0 // 8192), out=G[c0:c1])
    g = FloatGallery.from_device_rows(G, d, _lib.METRIC_COSINE)
    gq = torch.Generator(device=device)
    gq.manual_seed(SEED + 7)
    ids = torch.randint(0, N // args.per_id, (B,), generator=gq, device=device)
    Qd = P.project(bank.images(ids, seed=SEED + 99))
    out = {"metric": "CosineDistance 1-NN queries/s (1M gallery, projected queries)",
           "config": {"gallery": N, "batch": B, "d": d, "k": 1}, "data": "synthetic"}
    for mode in ("auto", "fp32"):
        os.environ["OFR_SEARCH"] = mode
        ms, (dd, ii) = timed(lambda: g.search(Qd, 1), args.steps)
        acc = float(((ii[:, 0] // args.per_id) == ids).double().mean())
        out[mode] = {"ms_per_batch": ms, "queries_per_s": B / (ms * 1e-3), "top1_identity_acc": acc,
                     "uncertified_after_each_tier": (list(g.last_fallbacks) if mode == "auto" else None)}
        if mode == "auto":
            first = ii.clone()
    out["same_top1_as_fp32_path"] = float((first[:, 0] == ii[:, 0]).double().mean())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
