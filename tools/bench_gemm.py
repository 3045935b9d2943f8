"""Throughput of the training products on one MI355X (one JSON line):
* ofr_gemm_f64 (v_mfma_f64_16x16x4_f64) on the configs[4] shape of its largest call, T = M^T S
  (10,000 x 10,000 over K = 10,000 class means / sums, training.pixel_scatter): 2 M N K flop;
* ofr_gram_u8 (v_mfma_i32_32x32x32_i8, exact) on configs[4]'s X'^T X' (D = 10,000 over n = 100,000):
  int8 ops of the upper-triangle tiles it computes.
Peaks: MI355X_MICROARCH.md (fp64 matrix 78.6 TF, int8 ~5 POPS dense)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opencv_facerecognizer_amd import _device, _lib, training  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = _lib.device()
    out = {}
    M = N = K = 10_000
    A = torch.randn((K, M), dtype=torch.float64, device=dev)
    B = torch.randn((K, N), dtype=torch.float64, device=dev)
    ms = timed(lambda: _device.gemm_f64(A, B, transA=True))
    out["gemm_f64_MtS"] = {"M": M, "N": N, "K": K, "ms": ms, "tflops": 2.0 * M * N * K / ms / 1e9,
                           "frac_of_78.6TF": 2.0 * M * N * K / ms / 1e9 / 78.6}
    A2 = torch.randn((4096, 4096), dtype=torch.float64, device=dev)
    ms2 = timed(lambda: _device.gemm_f64(A2, A2))
    out["gemm_f64_4096"] = {"ms": ms2, "tflops": 2.0 * 4096 ** 3 / ms2 / 1e9}
    del A, B, A2
    n, D = 100_000, 10_000
    X = torch.randint(0, 256, (n, D), dtype=torch.uint8, device=dev)
    Xt, _ = training.padded(X, n, D, transpose=True)
    ms3 = timed(lambda: training.gram(Xt, D, n), reps=3)
    nt = -(-D // 256)
    ops = 2.0 * nt * (nt + 1) / 2 * 256 * 256 * Xt.shape[1]
    out["gram_u8_XtX"] = {"D": D, "n": n, "ms": ms3, "tops_executed": ops / ms3 / 1e9,
                          "frac_of_5POPS": ops / ms3 / 1e9 / 5000.0}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
