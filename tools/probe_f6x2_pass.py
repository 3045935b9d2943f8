"""Times the two-slice tier's passes (sample + thresholds, sieve) against the fp6 tier's on the same
gallery and batch (B = 4096, d = 9999), at pixel noise 12 (headline) and 96 (crowded), with the kept-row
counts: separates the cost of the three segments from the data (sieve hits).  One JSON line per noise.

    python tools/probe_f6x2_pass.py [--gallery 1000000] [--noise 12,96]
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
from opencv_facerecognizer_amd._device import round_up  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank, build_gallery, build_projection  # noqa: E402


def timed(fn, reps, before=None):
    """Median event time of fn over reps runs (after one warm-up); before() runs untimed ahead of each."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for r in range(reps + 1):
        if before:
            before()
        torch.cuda.synchronize()
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        if r:
            out.append(s.elapsed_time(e))
    return sorted(out)[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=1_000_000)
    ap.add_argument("--noise", default="12,96")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = _lib.device()
    D, d, B, k, per = 10000, 9999, 4096, 1, 10
    N = args.gallery
    P, _ = build_projection(D, d, dev)
    bank = IdentityBank(-(-N // per), 100, 100, device=dev)   # row j shows identity j // per
    ld = max(32, round_up(d, 32))
    for noise in [float(x) for x in args.noise.split(",")]:
        g = build_gallery(P, bank, per, 0, N, N, d, ld, dev, noise=noise)
        gq = torch.Generator(device=dev)
        gq.manual_seed(SEED + 7)
        ids_q = torch.randint(0, N // per, (B,), generator=gq, device=dev)
        Qd = P.project(bank.images(ids_q, seed=SEED + 99, noise=noise), shift64=g.shift64)
        res = {"noise": noise, "gallery": N, "batch": B}
        for tier in ("f6", "f6x2"):
            qq = g.quantize_queries(Qd, tier=tier)
            # the sieve pass appends to the buckets its sample pass reset: one sample pass before each
            res[tier] = {"sample_ms": timed(lambda: g.search_q8_phase(4, Qd, qq, k), args.reps),
                         "sieve_ms": timed(lambda: g.search_q8_phase(8, Qd, qq, k), args.reps,
                                           before=lambda: g.search_q8_phase(4, Qd, qq, k))}
            cnt = g.sieve_counts(B)
            res[tier]["kept_mean"] = float(cnt.double().mean())
            res[tier]["kept_max"] = int(cnt.max())
            g.search_q8_phase(2, Qd, qq, k)
            torch.cuda.synchronize()
            res[tier]["uncertified"] = int((qq["cert"] == 0).sum())
        res["f6x2_over_3x_f6"] = res["f6x2"]["sieve_ms"] / (3 * res["f6"]["sieve_ms"])
        print(json.dumps(res), flush=True)
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
