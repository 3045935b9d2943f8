"""How far down the coarse order would the fp6 certificate have to look on crowded data?

For the bench's 1M-row gallery at several pixel-noise levels, 64 sampled queries: exact squared
distances to every row (fp64 GEMM on the device rows), then (d_M^2 - d_1^2) / dS for ranks
M = 16 (today's list), 64, 256, 1024, 4096 and for the sieve threshold's rank (the 16th best row of
the sampled panels 0, 64, 128, ...).  The certificate needs this ratio above ~2 at the rank whose
coarse score bounds the excluded rows.  One JSON line per noise level.

    python tools/probe_deep_margin.py [--noise 12,48,96,192]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--noise", default="12,48,96,192")
    ap.add_argument("--gallery", type=int, default=1_000_000)
    ap.add_argument("--queries", type=int, default=64)
    a = ap.parse_args()
    dev = _lib.device()
    side, d, per_id, N = 100, 9999, 10, a.gallery
    P, _ = bench.build_projection(side * side, d, dev)
    n_ids = N // per_id
    bank = IdentityBank(n_ids, side, side, device=dev)
    ld = bench.round_up(d, 32)
    ranks = [16, 64, 256, 1024, 4096]
    stride = 64 * 256
    sampled = (torch.arange(N, device=dev) % stride) < 256
    for noise in [float(x) for x in a.noise.split(",")]:
        gal = bench.build_gallery(P, bank, per_id, 0, N, N, d, ld, dev, noise=noise)
        gq = torch.Generator(device=dev)
        gq.manual_seed(SEED + 7)
        ids_q = torch.randint(0, n_ids, (a.queries,), generator=gq, device=dev)
        Xq = bank.images(ids_q, seed=SEED + 99, noise=noise)
        Qd = torch.zeros((a.queries, ld), dtype=torch.float32, device=dev)
        P.project(Xq, shift64=gal.shift64, out=Qd)
        qq = gal.quantize_queries(Qd, None, tier="f6")
        Q64 = Qd[:, :d].double()
        D2 = torch.empty((a.queries, N), dtype=torch.float64, device=dev)
        for c0 in range(0, N, 65536):
            c1 = min(N, c0 + 65536)
            Gc = gal.G[c0:c1, :d].double()
            D2[:, c0:c1] = (Q64 * Q64).sum(1, keepdim=True) + (Gc * Gc).sum(1)[None, :] - 2.0 * Q64 @ Gc.T
            del Gc
        srt = torch.sort(D2, dim=1).values
        th = torch.sort(D2[:, sampled], dim=1).values[:, 15]
        theta_rank = (D2 <= th[:, None]).sum(1).double()
        st = qq["stats"].cpu().numpy()
        gmax = gal._tier_gallery("f6")["gmax"].cpu().numpy()
        A, E, aux = gmax[0], gmax[1], gmax[3]
        qa, qe = st[:, 0], st[:, 1]
        gamma = (2 * -(-d // 128) + 64) * 2.0 ** -23
        dS = 2 * (qa * E + qe * A + qe * E) + 2.0 ** -20 * (aux + 2 * qa * A) + 2 * gamma * qa * A
        s = srt.cpu().numpy()
        res = {"pixel_noise": noise, "queries": a.queries, "dS_median": float(np.median(dS)),
               "top1_identity_acc": float(((torch.argmin(D2, 1) // per_id) == ids_q).double().mean().item())}
        for M in ranks:
            r = (s[:, M - 1] - s[:, 0]) / dS
            res[f"margin_rank{M}"] = {"median": float(np.median(r)), "min": float(r.min()),
                                      "frac_ge_2": float((r >= 2).mean())}
        r = (th.cpu().numpy() - s[:, 0]) / dS
        res["margin_theta"] = {"median": float(np.median(r)), "min": float(r.min()), "frac_ge_2": float((r >= 2).mean()),
                               "theta_rank_median": float(theta_rank.median().item())}
        print(json.dumps(res), flush=True)
        del gal, D2, srt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
