"""Face-tensor ingestion throughput: ofr_ingest_faces on device-resident images.

  recognizer: 4,096 face boxes (80-240 px squares) cropped from 64 BGR 640x480 frames, BGR2GRAY,
              INTER_CUBIC to 100x100 (bin/ocvf_recognizer.py:64-66 per face);
  trainer:    4,096 grey 112x92 images, INTER_LINEAR to 70x70 (trainer/thetrainer.py:99-103).
Timed with HIP events over repeated launches on the current stream; roofline against HBM with the
algorithmic bytes = every source byte of the crops read once + the output written once.  The CPU
baseline is the oracle's OpenCV fixed-point restatement (numpy, 1 thread) on a sample of faces.
Prints one JSON line.

    python tools/bench_ingest.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._lib import call, ptr, stream  # noqa: E402

PEAK_HBM = 8.0e12


def run(src, jobs, n, dh, dw, mode, reps=20):
    out = torch.empty((n, dh, dw), dtype=torch.uint8, device=src.device)
    call("ofr_ingest_faces", stream(), ptr(src), ptr(jobs), n, dh, dw, mode, ptr(out))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        call("ofr_ingest_faces", stream(), ptr(src), ptr(jobs), n, dh, dw, mode, ptr(out))
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, out


def main():
    dev = _lib.device()
    r = np.random.Generator(np.random.PCG64(20261015))
    res = {"metric": "faces/s, crop + grey + resize into uint8 face rows (SURVEY 8f row 1)", "data": "synthetic"}
    # recognizer: BGR frames, square boxes, cubic to 100x100
    F, H, W, n = 64, 480, 640, 4096
    frames = r.integers(0, 256, (F, H, W, 3), dtype=np.uint8)
    sz = r.integers(80, 241, n)
    x0 = (r.random(n) * (W - sz)).astype(np.int64)
    y0 = (r.random(n) * (H - sz)).astype(np.int64)
    fi = r.integers(0, F, n)
    jobs = np.stack([fi * H * W * 3, np.full(n, W * 3), x0, y0, sz, sz, np.full(n, 3)], 1).astype(np.int64)
    src = torch.from_numpy(frames.reshape(-1)).to(dev)
    ms, out = run(src, torch.from_numpy(jobs).to(dev), n, 100, 100, 2)
    alg = float((sz.astype(np.float64) ** 2 * 3).sum() + n * 100 * 100)
    # CPU baseline: the oracle restatement per face (bin/ocvf_recognizer.py:64-66)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import facerec_oracle as O   # the checker; timed here as the CPU baseline
    m = 16
    t0 = time.perf_counter()
    ref = [O.recognizer_face(frames[fi[j]], (x0[j], y0[j], x0[j] + sz[j], y0[j] + sz[j]), (100, 100)) for j in range(m)]
    t_cpu = (time.perf_counter() - t0) / m
    exact = bool(all(np.array_equal(ref[j], out[j].cpu().numpy()) for j in range(m)))
    res["recognizer"] = {"faces": n, "from": "64 BGR 640x480 frames, 80-240 px boxes", "to": "100x100 INTER_CUBIC",
                         "ms": ms, "faces_per_s": n / (ms * 1e-3),
                         "roofline": {"bound": "hbm", "algorithmic_bytes": alg, "achieved_gbs": alg / (ms * 1e-3) / 1e9,
                                      "peak_gbs": PEAK_HBM / 1e9, "frac": alg / (ms * 1e-3) / PEAK_HBM},
                         "bit_exact_vs_oracle_sample": exact,
                         "cpu_baseline": {"kind": "port", "cores": 1, "faces_per_s": 1.0 / t_cpu,
                                          "sample": f"{m} faces through the oracle's OpenCV restatement (numpy)"}}
    # trainer: grey images, linear to 70x70
    n2, h2, w2 = 4096, 112, 92
    imgs = r.integers(0, 256, (n2, h2, w2), dtype=np.uint8)
    jobs2 = np.stack([np.arange(n2) * h2 * w2, np.full(n2, w2), np.zeros(n2), np.zeros(n2), np.full(n2, w2),
                      np.full(n2, h2), np.ones(n2)], 1).astype(np.int64)
    src2 = torch.from_numpy(imgs.reshape(-1)).to(dev)
    ms2, out2 = run(src2, torch.from_numpy(jobs2).to(dev), n2, 70, 70, 1)
    alg2 = float(n2 * (h2 * w2 + 70 * 70))
    t0 = time.perf_counter()
    ref2 = [O.cv_resize_u8(imgs[j], (70, 70), "linear") for j in range(m)]
    t_cpu2 = (time.perf_counter() - t0) / m
    exact2 = bool(all(np.array_equal(ref2[j], out2[j].cpu().numpy()) for j in range(m)))
    res["trainer"] = {"faces": n2, "from": "112x92 grey", "to": "70x70 INTER_LINEAR", "ms": ms2,
                      "faces_per_s": n2 / (ms2 * 1e-3),
                      "roofline": {"bound": "hbm", "algorithmic_bytes": alg2, "achieved_gbs": alg2 / (ms2 * 1e-3) / 1e9,
                                   "peak_gbs": PEAK_HBM / 1e9, "frac": alg2 / (ms2 * 1e-3) / PEAK_HBM},
                      "bit_exact_vs_oracle_sample": exact2,
                      "cpu_baseline": {"kind": "port", "cores": 1, "faces_per_s": 1.0 / t_cpu2,
                                       "sample": f"{m} images through the oracle's OpenCV restatement (numpy)"}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
