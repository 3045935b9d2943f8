"""Probe: one face per call (the recognizers' pattern) as a captured HIP graph vs eager launches.

The device part of PredictableModel.predict for a Fisherfaces + NearestNeighbor(Euclidean, k=1)
model -- projection (GEMV over the int8 slices), fp6 query quantization, the fp6 stream pass,
premerge, merge + certificate -- captured once with torch.cuda.graph on the current stream and
replayed; HIP events around eager and replayed sequences.  One JSON line.

    python tools/probe_graph_predict.py [--gallery 100000]
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
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    dev = _lib.device()
    side, d, N, per_id = 100, 9999, args.gallery, 10
    D = side * side
    g = torch.Generator(device=dev).manual_seed(SEED + 3)
    W = (torch.randn((D, d), generator=g, device=dev, dtype=torch.float64) / np.sqrt(D)).cpu().numpy()
    ff = Fisherfaces()
    ff._eigenvectors = np.asmatrix(W)
    ff._eigenvalues = np.ones(d, np.float32)
    ff._num_components = d
    bank = IdentityBank(-(-N // per_id), side, side, device=dev)   # row j shows identity j // per_id
    P = Projection(W=W, device=dev)
    F = torch.empty((N, d), dtype=torch.float64, device=dev)
    for c0 in range(0, N, 8192):
        c1 = min(N, c0 + 8192)
        F[c0:c1] = P.project(bank.images(torch.arange(c0, c1, device=dev) // per_id, seed=SEED + 1000 + c0), f64=True)
    clf = NearestNeighbor(EuclideanDistance(), k=1)
    clf.compute([None] * N, np.arange(N) // per_id)
    clf.adopt_device_rows(F)
    del F
    gal = clf._gallery()
    face = bank.images(torch.tensor([7], device=dev), seed=SEED + 99).reshape(1, side, side).contiguous()
    out = (torch.empty((1, 1), dtype=torch.float64, device=dev), torch.empty((1, 1), dtype=torch.int64, device=dev))
    state = {}

    def seq():
        Qd = ff.project_device(face, shift64=gal.shift64)
        state["qq"] = gal.quantize_queries(Qd, state.get("qq"), tier="f6")
        gal.search_q8_phase(3, Qd, state["qq"], 1, out=out)

    for _ in range(5):
        seq()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        seq()
    e1.record()
    e1.synchronize()
    eager_ms = e0.elapsed_time(e1) / args.reps
    res = {"gallery": N, "eager_device_ms": eager_ms, "eager_index": int(out[1][0, 0])}
    t0 = time.perf_counter()
    for _ in range(args.reps):
        seq()
        torch.cuda.synchronize()
    res["eager_wall_ms"] = (time.perf_counter() - t0) * 1e3 / args.reps
    try:
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            seq()                       # warm on the capture stream
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(graph):
            seq()
        out[1].fill_(-7)
        graph.replay()
        torch.cuda.synchronize()
        res["graph_index"] = int(out[1][0, 0])
        e0.record()
        for _ in range(args.reps):
            graph.replay()
        e1.record()
        e1.synchronize()
        res["graph_device_ms"] = e0.elapsed_time(e1) / args.reps
        t0 = time.perf_counter()
        for _ in range(args.reps):
            graph.replay()
            torch.cuda.synchronize()
        res["graph_wall_ms"] = (time.perf_counter() - t0) * 1e3 / args.reps
    except Exception as exc:   # noqa: BLE001 (probe: report why capture failed)
        res["graph_error"] = repr(exc)[:400]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
