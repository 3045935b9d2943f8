"""The prefix tier's sieve pass alone on the headline shape (trained W, 1M gallery, B = 4096): the pass
(ofr_knn_f6p_sampled phase 8, after its sample pass + thresholds) timed by HIP events, median of reps,
for each engine (OFR_F6P_ENGINE 1 = tile_kernel_f6p, 2 = prefix_pass_kernel) -- and, with OFR_LIB pointing
at a probe build (tools/build_pp_probes.sh: OFR_PP_PROBE bits 1 no flush, 2 no compares, 4 no MFMAs), the
cost of each part.  One JSON line per engine.
  OFR_LIB=tools/var/libpp_1.so python tools/probe_prefix_pass.py --tag pp1
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from opencv_facerecognizer_amd._device import round_up  # noqa: E402
from opencv_facerecognizer_amd.synthetic import (SEED, IdentityBank, build_gallery,  # noqa: E402
                                                 build_trained_projection)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--engines", default="2,1")
    ap.add_argument("--tag", default="")
    ap.add_argument("--query-ids", type=int, default=0,
                    help="draw the queries from this many identities (0: the gallery's own; 100000 at --gallery "
                         "125000 = rank 0's shard at G = 8, 7/8 of the queries foreign)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    N, per, side, B = a.gallery, 10, 100, a.batch
    nid = a.query_ids or N // per
    bank = IdentityBank(max(N // per, 10_000, nid), side, side, device=dev)
    P, _, _ = build_trained_projection(bank, per, 100_000, side * side, dev)
    d = P.d
    g = build_gallery(P, bank, per, 0, N, N, d, max(32, round_up(d, 32)), dev)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    ids = torch.randint(0, nid, (B,), generator=gq, device=dev)
    Qd = P.project(bank.images(ids, seed=SEED + 99), shift64=g.shift64)
    qq = g.quantize_queries(Qd, tier="f6p")
    for e in [x for x in a.engines.split(",") if x]:
        e, _, occ = e.partition(":")  # "4:3" = engine 4 at 3 workgroups per CU
        os.environ["OFR_F6P_ENGINE"] = e
        os.environ["OFR_F6P_OCC"] = occ or "2"
        ms, ms4 = [], []
        for rep in range(a.reps + 2):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e2.record()
            g.search_q8_phase(4, Qd, qq, 1)
            e0.record()
            g.search_q8_phase(8, Qd, qq, 1)
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                ms.append(e0.elapsed_time(e1))
                ms4.append(e2.elapsed_time(e0))
        kept = g.sieve_counts(B)
        m = float(np.median(ms))
        ops = 2.0 * B * N * min(d, 128 * g.prefix_stages())
        print(json.dumps({"tag": a.tag, "lib": os.environ.get("OFR_LIB", "in-tree"), "engine": int(e), "occ": int(occ or 2),
                          "pass_ms_median": m, "sample_ms_median": float(np.median(ms4)), "gallery": N, "pass_ms_min": float(min(ms)), "pass_ms_max": float(max(ms)),
                          "frac_fp6_peak": ops / (m * 1e-3) / 10e15, "kept_mean": float(kept.double().mean()),
                          "kept_max": int(kept.max()), "pstages": g.prefix_stages()}), flush=True)


if __name__ == "__main__":
    main()
