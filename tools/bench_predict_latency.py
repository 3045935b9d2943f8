"""One face per call through the reference's API, the recognizers' pattern (bin/ocvf_recognizer.py:67:
``model.predict(face)`` per detected face): wall-clock latency of PredictableModel.predict on a
Fisherfaces + NearestNeighbor(Euclidean, k=1) model, next to the device time of the same steps.

The model is assembled from synthetic parts (random W, D = 10,000 -> d = 9,999; a gallery of
synthetic identity-bank faces projected on the device and adopted as the classifier's rows; the
classifier's host X is a placeholder list of the right length -- predict never reads it).

    python tools/bench_predict_latency.py [--gallery 100000] [--calls 50]
"""
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
from opencv_facerecognizer_amd._device import Projection  # noqa: E402
from opencv_facerecognizer_amd.facerec.classifier import NearestNeighbor  # noqa: E402
from opencv_facerecognizer_amd.facerec.distance import EuclideanDistance  # noqa: E402
from opencv_facerecognizer_amd.facerec.feature import Fisherfaces  # noqa: E402
from opencv_facerecognizer_amd.facerec.model import PredictableModel  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=100_000)
    ap.add_argument("--per-id", type=int, default=10)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--side", type=int, default=100)
    ap.add_argument("--dim", type=int, default=9999)
    args = ap.parse_args()
    dev = _lib.device()
    D, d, N = args.side * args.side, args.dim, args.gallery
    g = torch.Generator(device=dev).manual_seed(SEED + 3)
    W = (torch.randn((D, d), generator=g, device=dev, dtype=torch.float64) / np.sqrt(D)).cpu().numpy()
    ff = Fisherfaces()
    ff._eigenvectors = np.asmatrix(W)
    ff._eigenvalues = np.ones(d, np.float32)
    ff._num_components = d
    ids = N // args.per_id
    bank = IdentityBank(ids, args.side, args.side, device=dev)
    P = Projection(W=W, device=dev)
    F = torch.empty((N, d), dtype=torch.float64, device=dev)
    for c0 in range(0, N, 8192):
        c1 = min(N, c0 + 8192)
        F[c0:c1] = P.project(bank.images(torch.arange(c0, c1, device=dev) // args.per_id, seed=SEED + 1000 + c0),
                             f64=True)
    clf = NearestNeighbor(EuclideanDistance(), k=1)
    y = np.arange(N) // args.per_id
    clf.compute([None] * N, y)
    clf.adopt_device_rows(F)
    del F
    model = PredictableModel(ff, clf)
    qid = torch.randint(0, ids, (args.calls + 5,), generator=g, device=dev)
    faces = bank.images(qid, seed=SEED + 99).reshape(-1, args.side, args.side).cpu().numpy()
    for i in range(5):                                  # warm: projection slices, gallery tiers, kernels
        model.predict(faces[i])
    torch.cuda.synchronize()
    lat, ok = [], 0
    for i in range(5, 5 + args.calls):
        t0 = time.perf_counter()
        label = model.predict(faces[i])[0]
        lat.append(time.perf_counter() - t0)
        ok += int(label == int(qid[i]))
    lat = np.array(lat) * 1e3
    # device time of the same one-face step (projection + fp6 stream pass + merge + certificate)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gal = clf._gallery()
    Xq = torch.from_numpy(faces[5:6].reshape(1, -1)).to(dev)
    e0.record()
    for _ in range(20):
        Qd = ff.project_device(Xq, shift64=gal.shift64)
        clf._search_prepared(Qd, 1)
    e1.record()
    e1.synchronize()
    res = {"metric": "PredictableModel.predict(face) wall-clock latency, one face per call",
           "config": {"gallery": N, "D": D, "d": d, "k": 1, "metric": "Euclidean"}, "data": "synthetic",
           "calls": args.calls, "latency_ms": {"median": float(np.median(lat)), "p90": float(np.percentile(lat, 90)),
                                              "min": float(lat.min())},
           "device_step_ms": e0.elapsed_time(e1) / 20, "top1_identity_acc": ok / args.calls}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
