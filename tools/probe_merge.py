"""Probe: the fp6 merge (phase 2 of ofr_knn_f6: bucket best-16, exact re-rank, certificate) at the
headline batch on galleries of one GPU's share at 1/2/4/8 GPUs (N = 1M / world), bench data.
HIP events around each phase on the current stream; one JSON line.

    python tools/probe_merge.py [--sizes 1000000,500000,250000,125000]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000000,500000,250000,125000")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--foreign", action="store_true",
                    help="queries of identities outside the gallery (a shard at G > 1 that does not hold them)")
    a = ap.parse_args()
    dev = _lib.device()
    side, d, per_id, B = 100, 9999, 10, a.batch
    P, _ = bench.build_projection(side * side, d, dev)
    sizes = [int(x) for x in a.sizes.split(",")]
    bank = IdentityBank(2 * max(sizes) // per_id, side, side, device=dev)
    ld = bench.round_up(d, 32)
    res = {"B": B, "d": d, "foreign_queries": a.foreign, "sizes": {}}
    for N in sizes:
        gal = bench.build_gallery(P, bank, per_id, 0, N, N, d, ld, dev)
        gal._tier_gallery("f6")
        gq = torch.Generator(device=dev)
        gq.manual_seed(SEED + 7)
        lo = N // per_id if a.foreign else 0
        ids = torch.randint(lo, lo + N // per_id, (B,), generator=gq, device=dev)
        Qd = torch.zeros((B, ld), dtype=torch.float32, device=dev)
        P.project(bank.images(ids, seed=SEED + 99), shift64=gal.shift64, out=Qd)
        qq = gal.quantize_queries(Qd, tier="f6")
        out = gal.search_q8_phase(3, Qd, qq, 1)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t1 = t2 = 0.0
        for _ in range(a.reps):
            ev[0].record()
            gal.search_q8_phase(1, Qd, qq, 1, out=out)
            ev[1].record()
            gal.search_q8_phase(2, Qd, qq, 1, out=out)
            ev[2].record()
            ev[2].synchronize()
            t1 += ev[0].elapsed_time(ev[1])
            t2 += ev[1].elapsed_time(ev[2])
        kept = gal.sieve_counts(B).double()
        res["sizes"][N] = {"phase1_ms": t1 / a.reps, "merge_ms": t2 / a.reps,
                           "kept_rows_per_query": {"mean": float(kept.mean()), "max": int(kept.max())},
                           "uncertified": int((qq["cert"] == 0).sum())}
        print(json.dumps({N: res["sizes"][N]}), file=sys.stderr, flush=True)
        del gal, qq, Qd
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
