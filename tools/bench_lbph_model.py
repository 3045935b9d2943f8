"""BASELINE.json configs[3] through the reference model API: PredictableModel(SpatialHistogram(
ExtendedLBP(1, 8), (8, 8)), NearestNeighbor(ChiSquareDistance(), k=1)) -- compute on 65,536 gallery
faces at 128x128, then predict_batch of B = 4,096 query faces.  Prints one JSON line.

    python tools/bench_lbph_model.py [--gallery 65536] [--batch 4096] [--reps 3]

The same synthetic faces as tools/bench_lbp_chi2.py (which calls the kernels directly).  Timed:
* compute (model.py:49-51): wall clock, including the float64 histograms the API returns (the
  reference's return type, feature.py:274-280) -- one ofr_elbp_hist launch, the counts kept on the
  device as the classifier's gallery;
* predict_batch (model.py:53-55 for a batch) from host faces: wall clock of the whole call (upload,
  one histogram launch, the counts search, the label votes on the host);
* the device part alone (HIP events): histogram launch + ofr_chi2_knn, the direct path's pieces.
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

from ocvfacerec.facerec.classifier import NearestNeighbor  # noqa: E402
from ocvfacerec.facerec.distance import ChiSquareDistance  # noqa: E402
from ocvfacerec.facerec.feature import SpatialHistogram  # noqa: E402
from ocvfacerec.facerec.lbp import ExtendedLBP  # noqa: E402
from ocvfacerec.facerec.model import PredictableModel  # noqa: E402
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=65536)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--per-id", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    device = _lib.device()
    N, B, H = args.gallery, args.batch, 128
    n_ids = (N + args.per_id - 1) // args.per_id
    bank = IdentityBank(n_ids, H, H, device=device)
    G_img = bank.images(torch.arange(N, device=device) // args.per_id, seed=SEED + 11).reshape(N, H, H)
    gq = torch.Generator(device=device)
    gq.manual_seed(SEED + 12)
    ids_q = torch.randint(0, n_ids, (B,), generator=gq, device=device)
    Q_img = bank.images(ids_q, seed=SEED + 13).reshape(B, H, H)
    Xg = G_img.cpu().numpy()
    Xq = Q_img.cpu().numpy()
    y = np.arange(N) // args.per_id
    del G_img

    model = PredictableModel(SpatialHistogram(ExtendedLBP(1, 8), (8, 8)), NearestNeighbor(ChiSquareDistance(), k=1))
    t0 = time.perf_counter()
    model.compute(list(Xg), y)
    torch.cuda.synchronize()
    t_compute = time.perf_counter() - t0
    g = model.classifier._gallery()
    gal_form = {"dtype": {0: "u8 counts", 1: "u16 counts", 2: "u32 counts", 3: "fp32"}[g.dtype], "denom": g.denom,
                "bytes": int(g.G.numel() * g.G.element_size())}

    preds = model.predict_batch(Xq)                     # warm (workspace, kernels)
    torch.cuda.synchronize()
    walls = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        preds = model.predict_batch(Xq)
        walls.append(time.perf_counter() - t0)
    ms_predict = 1e3 * float(np.median(walls))
    labels = np.array([p[0] for p in preds])
    acc = float(np.mean(labels == ids_q.cpu().numpy()))

    # the device pieces of the same call (events): histogram launch + counts search
    sh, clf = model.feature, model.classifier
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    Qd = torch.from_numpy(Xq).to(device)
    ms_h, ms_s = [], []
    for _ in range(args.reps):
        e[0].record()
        C, cell, cb = sh.counts_batch(Qd)
        e[1].record()
        clf.search_counts(C, cell, cb, 1)
        e[2].record()
        torch.cuda.synchronize()
        ms_h.append(e[0].elapsed_time(e[1]))
        ms_s.append(e[1].elapsed_time(e[2]))
    out = {
        "metric": "query faces/sec through PredictableModel.predict_batch (LBPH: ExtendedLBP + SpatialHistogram 8x8 "
                  "+ ChiSquare 1-NN, configs[3])",
        "config": {"gallery": N, "batch": B, "side": H, "lbp": "ExtendedLBP(radius=1, neighbors=8)", "grid": [8, 8],
                   "k": 1},
        "data": "synthetic",
        "compute_s": t_compute, "gallery_form": gal_form,
        "predict_batch_ms": ms_predict, "queries_per_s": B / (ms_predict * 1e-3),
        "device_ms": {"query_histograms": float(np.median(ms_h)), "chi2_search": float(np.median(ms_s))},
        "chi2_uncertified_after_each_pass": list(g.last_fallbacks),
        "top1_identity_acc": acc,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
