"""Probe: phase timings of the B <= 32 fp6 search (stream pass vs merge + certificate) on a
synthetic gallery, HIP events around each phase of ofr_knn_f6 on the current stream."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import FloatGallery  # noqa: E402


def main():
    dev = _lib.device()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    d = 9999
    g = torch.Generator(device=dev).manual_seed(3)
    protos = torch.randn((N // 10, d), generator=g, device=dev, dtype=torch.float64) * 5
    F = protos.repeat_interleave(10, 0)[:N] + torch.randn((N, d), generator=g, device=dev, dtype=torch.float64)
    gal = FloatGallery(F, _lib.METRIC_EUCLIDEAN)
    del F
    gal._tier_gallery("f6")
    res = {"N": N}
    for B in (1, 8, 32):
        Q = (protos[:B] + torch.randn((B, d), generator=g, device=dev, dtype=torch.float64)).contiguous()
        Qd = gal.query_rows(Q)
        qq = gal.quantize_queries(Qd, tier="f6")
        for _ in range(3):
            gal.search_q8_phase(3, Qd, qq, 1)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t1 = t2 = 0.0
        for _ in range(20):
            ev[0].record()
            gal.search_q8_phase(1, Qd, qq, 1)
            ev[1].record()
            gal.search_q8_phase(2, Qd, qq, 1)
            ev[2].record()
            ev[2].synchronize()
            t1 += ev[0].elapsed_time(ev[1])
            t2 += ev[1].elapsed_time(ev[2])
        res[f"B{B}"] = {"phase1_ms": t1 / 20, "phase2_merge_ms": t2 / 20}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
