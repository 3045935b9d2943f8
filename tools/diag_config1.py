"""Diagnostic for the bench's configs[1] line (100k-row gallery, B = 4096, d = 9999): builds the gallery
twice (determinism), runs the certified chain and the exact fp32 path on the same batch and reports
where they differ, the identity accuracy of each, and the fp6 tier's uncertified count.  One JSON line.

    python tools/diag_config1.py [--gallery 100000]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=100_000)
    ap.add_argument("--ids", type=int, default=100_000, help="identities in the bank (bench: 1M / 10)")
    ap.add_argument("--bench-loop", type=int, default=0,
                    help="instead: bench.stress_run's pipelined step (side-stream preparation) this many times")
    args = ap.parse_args()
    if args.bench_loop:
        return bench_loop(args)
    dev = _lib.device()
    D, d, B, k, per = 10000, 9999, 4096, 1, 10
    N = args.gallery
    P, _ = build_projection(D, d, dev)
    bank = IdentityBank(args.ids, 100, 100, device=dev)
    ld = max(32, round_up(d, 32))
    g = build_gallery(P, bank, per, 0, N, N, d, ld, dev)
    g2 = build_gallery(P, bank, per, 0, N, N, d, ld, dev)
    same_build = bool(torch.equal(g.G, g2.G))
    del g2
    n_ids = (N + per - 1) // per
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    ids_q = torch.randint(0, n_ids, (B,), generator=gq, device=dev)
    Xq = bank.images(ids_q, seed=SEED + 99)
    Qd = P.project(Xq, shift64=g.shift64)
    qq = g.quantize_queries(Qd, tier="f6")
    out = g.search_q8_phase(3, Qd, qq, k)
    n_open = g.fallback(Qd, qq, k, out)
    fb = list(g.last_fallbacks)
    d32, i32 = g._search_f32(Qd, k)
    i_c, d_c = out[1][:, 0], out[0][:, 0]
    diff = (i_c != i32[:, 0])
    rel = ((d_c - d32[:, 0]).abs() / d32[:, 0].clamp_min(1e-30))
    res = {
        "gallery": N, "bank_ids": args.ids, "same_gallery_twice": same_build,
        "gallery_finite": bool(torch.isfinite(g.G).all()), "aux_finite": bool(torch.isfinite(g.aux).all()),
        "uncertified_after_each_tier": fb, "first_tier_open": int(n_open),
        "acc_certified": float(((i_c // per) == ids_q).double().mean()),
        "acc_fp32": float(((i32[:, 0] // per) == ids_q).double().mean()),
        "rows_differ": int(diff.sum()), "max_rel_dist_diff": float(rel.max()),
        "max_rel_dist_diff_where_rows_differ": float(rel[diff].max()) if int(diff.sum()) else 0.0,
    }
    print(json.dumps(res), flush=True)


def bench_loop(args):
    """bench.py's configs[1] line (stress_run at N = 100k, noise 12) in a fresh process, repeated."""
    import types
    import bench
    dev = _lib.device()
    P, _ = build_projection(10000, 9999, dev)
    bank = IdentityBank(args.ids, 100, 100, device=dev)
    a = types.SimpleNamespace(gallery=1_000_000, per_id=10, batch=4096, dim=9999, k=1, stress_steps=3)
    for rep in range(args.bench_loop):
        r = bench.stress_run(P, bank, a, 12.0, dev, N=args.gallery)
        print(json.dumps({"rep": rep, "queries_per_s": r["queries_per_s"], "uncertified": r["uncertified_after_each_tier"],
                          "acc": r["top1_identity_acc"], "margin": r["certificate_margin_fp6"]}), flush=True)


if __name__ == "__main__":
    main()
