"""BASELINE.json configs[4] (Fisherfaces training) at a scale one box finishes in about a minute:
n synthetic 100x100 faces of c identities, Fisherfaces().compute (PCA -> LDA, thetrainer.py:120 defaults).

    python tools/bench_train.py [--n 4000] [--ids 400]

Splits the wall time into the host LAPACK eigensolves the reference itself calls (np.linalg.eigh for the
PCA Gram / covariance, inv + eig for LDA, feature.py:94/170; timed by wrapping numpy) and the rest: the
device work (centring, Gram, left vectors, class centring, Sw/Sb, W = P.L, feature projections on the
fp64 / int8 MFMA) plus host transfers.  The CPU baseline runs the oracle's reference-faithful
Fisherfaces.compute (SVD, O(N^2) as_column_matrix) on a smaller sample and scales it by (n / n_cpu)^2
(N^2 scaling measured).  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd.facerec.feature import Fisherfaces  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402

HOST = {"eigh": 0.0, "eig": 0.0, "inv": 0.0}


def _timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        HOST[name] += time.perf_counter() - t0
        return r
    return w


def faces(n, ids, side, device, seed):
    bank = IdentityBank(ids, side, side, device=device)
    y = torch.arange(n, device=device) % ids
    X = bank.images(y, seed=seed).reshape(n, side, side).cpu().numpy()
    return list(X), y.cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--ids", type=int, default=400)
    ap.add_argument("--side", type=int, default=100)
    ap.add_argument("--n-cpu", type=int, default=600)
    args = ap.parse_args()
    device = _lib.device()
    X, y = faces(args.n, args.ids, args.side, device, SEED + 21)
    la = np.linalg
    la.eigh, la.eig, la.inv = _timed("eigh", la.eigh), _timed("eig", la.eig), _timed("inv", la.inv)
    ff = Fisherfaces()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    feats = ff.compute(X, y)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    host = sum(HOST.values())
    n, D, c = args.n, args.side * args.side, args.ids
    k = min(n - c, n - 1)
    d = c - 1
    W = np.asarray(ff._eigenvectors)
    # resubstitution 1-NN on the training features (sanity, host)
    F = np.stack([np.asarray(f).reshape(-1) for f in feats])
    flops = {"pca_gram": 2.0 * n * n * D, "pca_left_vectors": 2.0 * D * n * n, "pca_features": 2.0 * n * D * k,
             "lda_sw": 2.0 * k * k * n, "lda_sb": 2.0 * k * k * c, "lda_features": 2.0 * n * k * d,
             "w_pl": 2.0 * D * k * d, "train_projection_int8x4": 4 * 2.0 * n * D * d}

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import facerec_oracle as O  # the checker; timed here as the CPU baseline
    Xc, yc = faces(args.n_cpu, max(2, args.ids * args.n_cpu // args.n), args.side, device, SEED + 22)
    t1 = time.perf_counter()
    O.fisherfaces_compute([x.astype(np.uint8) for x in Xc], yc)
    t_cpu = time.perf_counter() - t1
    out = {
        "metric": "Fisherfaces.compute wall time (configs[4] at reduced scale)",
        "config": {"n": n, "identities": c, "D": D, "pca_components": k, "d": d},
        "data": "synthetic",
        "wall_s": total, "host_lapack_s": dict(HOST), "device_and_transfers_s": total - host,
        "device_flops": flops, "device_flops_total": sum(flops.values()),
        "device_tflops_upper_bound": sum(flops.values()) / max(total - host, 1e-9) / 1e12,
        "W_shape": list(W.shape), "finite": bool(np.isfinite(W).all() and np.isfinite(F).all()),
        "cpu_baseline": {"kind": "port", "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                         "sample": f"oracle fisherfaces_compute (reference-faithful: SVD, as_column_matrix) on "
                                   f"n={args.n_cpu}, scaled by (n/n_cpu)^2",
                         "sample_s": t_cpu, "wall_s_estimate": t_cpu * (n / args.n_cpu) ** 2},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
