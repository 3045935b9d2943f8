"""BASELINE.json configs[4] (Fisherfaces training) at a scale one box finishes in about a minute:
n synthetic 100x100 faces of c identities, Fisherfaces().compute (PCA -> LDA, thetrainer.py:120 defaults).

    python tools/bench_train.py [--n 4000] [--ids 400] [--solver auto|eig|eigh|device]
    python tools/bench_train.py --n 100000 --ids 10000                   # configs[4] at full scale

Splits the wall time into the host LAPACK eigensolves the reference itself calls (np.linalg.eigh for the
PCA Gram / covariance, inv + eig for LDA, feature.py:94/170; timed by wrapping numpy) and the rest: the
device work (centring, Gram, left vectors, class centring, Sw/Sb, W = P.L, feature projections on the
fp64 / int8 MFMA) plus host transfers; the device eigensolves (rocSOLVER dsyevd / dsygvd, ofr_eig.hip)
are reported apart.  --solver picks the LDA eigensolve (feature.lda_eigen): auto (default: the
reference's inv + eig up to order 1024, the device pencil solver above), eig, eigh (host sygvx/sygvd),
device.  The CPU baseline runs the oracle's reference-faithful
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
from opencv_facerecognizer_amd.facerec.classifier import NearestNeighbor  # noqa: E402
from opencv_facerecognizer_amd.facerec.distance import EuclideanDistance  # noqa: E402
from opencv_facerecognizer_amd.facerec.feature import Fisherfaces  # noqa: E402
from opencv_facerecognizer_amd.facerec.model import PredictableModel  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402

HOST = {"eigh": 0.0, "eig": 0.0, "inv": 0.0, "sygv": 0.0}
DEV_EIG = {"eigh_dsyevd": 0.0, "sygv_dsygvd": 0.0}


def _dev_timed(name, fn):
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        DEV_EIG[name] += time.perf_counter() - t0
        return r
    return w


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
    ap.add_argument("--solver", choices=["eig", "eigh", "device", "auto"], default="auto")
    ap.add_argument("--predict", type=int, default=4096)
    args = ap.parse_args()
    device = _lib.device()
    X, y = faces(args.n, args.ids, args.side, device, SEED + 21)
    la = np.linalg
    la.eigh, la.eig, la.inv = _timed("eigh", la.eigh), _timed("eig", la.eig), _timed("inv", la.inv)
    import scipy.linalg
    scipy.linalg.eigh = _timed("sygv", scipy.linalg.eigh)
    from opencv_facerecognizer_amd import _device
    _device.eigh_desc_f64 = _dev_timed("eigh_dsyevd", _device.eigh_desc_f64)
    _device.sygv_desc_f64 = _dev_timed("sygv_dsygvd", _device.sygv_desc_f64)
    os.environ["OFR_LDA_SOLVER"] = args.solver
    # the reference's training call: PredictableModel.compute = Fisherfaces.compute + NearestNeighbor.compute
    # (model.py:49-51, thetrainer.py:176)
    model = PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.compute(X, y)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    ff = model.feature
    feats = model.classifier.X
    # then predict (configs[4]): fresh faces of random identities, one batch; the first call also
    # builds the device gallery from the training features
    gq = torch.Generator(device=device)
    gq.manual_seed(SEED + 23)
    ids_q = torch.randint(0, args.ids, (args.predict,), generator=gq, device=device)
    Xq = IdentityBank(args.ids, args.side, args.side, device=device).images(ids_q, seed=SEED + 24)
    Xq = Xq.reshape(args.predict, args.side, args.side).cpu().numpy()
    pred_s = []
    for _ in range(3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        labels = np.array([p[0] for p in model.predict_batch(Xq)])
        torch.cuda.synchronize()
        pred_s.append(time.perf_counter() - t1)
    acc = float((labels == ids_q.cpu().numpy()).mean())
    host = sum(HOST.values())
    n, D, c = args.n, args.side * args.side, args.ids
    k = min(n - c if 0 < n - c <= n - 1 else n - 1, D, n)   # PCA components (feature.py:88-89)
    d = c - 1
    W = np.asarray(ff._eigenvectors)
    F = np.stack([np.asarray(f).reshape(-1) for f in feats])
    regime = getattr(ff, "_regime", "?")
    # algorithmic work of the device products per regime (training.py); int8 ops are exact Gram
    # products on the int8 MFMA, fp64 flops on the fp64 MFMA
    t = lambda R: -(-R // 256)                                             # noqa: E731
    gram_ops = lambda R, K: 2.0 * (t(R) * (t(R) + 1) // 2) * 256 * 256 * (-(-K // 128) * 128)   # noqa: E731
    if regime == "pixel":
        work = {"gram_u8_XtX_int8": gram_ops(D, n), "class_means_T_fp64": 2.0 * c * D * D}
    elif regime == "gram":
        work = {"gram_u8_XXt_int8": gram_ops(n, D), "lda_sw_sb_fp64": 2.0 * k * k * (n + c),
                "xct_M_int8x4": 4 * 2.0 * D * n * d}
    else:
        work = {"gram_u8_XtX_int8": gram_ops(D, n), "pca_features_int8x4": 4 * 2.0 * n * D * k,
                "lda_sw_sb_fp64": 2.0 * k * k * (n + c), "w_pl_fp64": 2.0 * D * k * d}
    work["train_projection_int8x4"] = 4 * 2.0 * n * D * d
    flops = work
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import facerec_oracle as O  # the checker; timed here as the CPU baseline
    Xc, yc = faces(args.n_cpu, max(2, args.ids * args.n_cpu // args.n), args.side, device, SEED + 22)
    t1 = time.perf_counter()
    O.fisherfaces_compute([x.astype(np.uint8) for x in Xc], yc)
    t_cpu = time.perf_counter() - t1
    out = {
        "metric": "PredictableModel(Fisherfaces, NearestNeighbor).compute wall time, then predict (configs[4])",
        "config": {"n": n, "identities": c, "D": D, "pca_components": k, "d": d, "lda_solver": args.solver,
                   "regime": regime},
        "data": "synthetic",
        "wall_s": total, "host_lapack_s": dict(HOST), "device_eigensolve_s": dict(DEV_EIG),
        "device_and_transfers_s": total - host,
        "predict": {"batch": args.predict, "first_call_s": pred_s[0], "steady_s": min(pred_s[1:]),
                    "queries_per_s": args.predict / min(pred_s[1:]), "top1_identity_acc": acc,
                    "note": "first call builds the device gallery (upload + quantized tiers) from the training features"},
        "device_ops": flops, "device_ops_total": sum(flops.values()),
        "W_shape": list(W.shape), "finite": bool(np.isfinite(W).all() and np.isfinite(F).all()),
        "cpu_baseline": {"kind": "port", "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                         "sample": f"oracle fisherfaces_compute (reference-faithful: SVD, as_column_matrix) on "
                                   f"n={args.n_cpu}, scaled by (n/n_cpu)^2",
                         "sample_s": t_cpu, "wall_s_estimate": t_cpu * (n / args.n_cpu) ** 2},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
