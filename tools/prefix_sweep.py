"""Cost model of the prefix tier's sieve pass (ofr_knn_f6p_sampled phase 8) on the headline shape:
the pass timed (HIP events, median of 5) at prefix lengths pst = 1, 2, 3, 4, 8, 16 stages on the
trained-W 1M gallery, B = 4096, so that t(pst) = T0 + pst * Tstage separates the per-tile fixed cost
from the per-stage MFMA work.  Probe only (results are not certified at every pst).
  python tools/prefix_sweep.py [--gallery N] > gpurun_out/prefix_sweep.txt
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import round_up  # noqa: E402
from opencv_facerecognizer_amd._lib import call, ptr, stream  # noqa: E402
from opencv_facerecognizer_amd.synthetic import (SEED, IdentityBank, build_gallery,  # noqa: E402
                                                 build_trained_projection)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--pst", default="1,2,3,4,8,16")
    ap.add_argument("--trace", action="store_true",
                    help="library built with -DOFR_F6P_TRACE (OFR_LIB): print workgroup 0's phase clocks")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    N, per, side, B = a.gallery, 10, 100, a.batch
    bank = IdentityBank(max(N // per, 10_000), side, side, device=dev)
    P, _, info = build_trained_projection(bank, per, 100_000, side * side, dev)
    d = P.d
    g = build_gallery(P, bank, per, 0, N, N, d, max(32, round_up(d, 32)), dev)
    print("prefix_stages", g.prefix_stages(), "d", d, flush=True)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    ids = torch.randint(0, N // per, (B,), generator=gq, device=dev)
    Qd = P.project(bank.images(ids, seed=SEED + 99), shift64=g.shift64)
    gt = g._tier_gallery("f6p")
    qq = g.quantize_queries(Qd, tier="f6p")
    for pst in [int(x) for x in a.pst.split(",")]:
        gt["pst"] = pst
        pdim = min(d, 128 * pst)
        call("ofr_row_aux", stream(), _lib.METRIC_EUCLIDEAN, ptr(g.G), g.N, pdim, g.ld, ptr(gt["paux"]))
        gt["spaux"] = g._prefix_sample_aux(gt["paux"], g.N)
        ms = []
        for rep in range(7):
            g.search_q8_phase(4, Qd, qq, 1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.search_q8_phase(8, Qd, qq, 1)
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                ms.append(e0.elapsed_time(e1))
        kept = g.sieve_counts(B).double().mean().item()
        mm = []
        for rep in range(5):                           # the merge (exact re-rank + certificate) alone
            g.search_q8_phase(4 | 8, Qd, qq, 1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.search_q8_phase(2, Qd, qq, 1)
            e1.record()
            torch.cuda.synchronize()
            mm.append(e0.elapsed_time(e1))
        print(f"pst {pst} sieve_ms {np.median(ms):.3f} kept_mean {kept:.1f} merge_ms {np.median(mm):.3f} "
              f"certified {int(qq['cert'].sum())}/{B}", flush=True)
        if a.trace:
            t = g.ws.buf[:64 * 8 * 8].view(torch.int64).view(64, 8).cpu().numpy()
            names = ["wait_copies", "flush_begin", "mfmas", "barrier", "copy_issue+tables", "compares", "sync"]
            rows = [r for r in t if r[0] > 0 and r[5] > r[0]]
            dd = np.array([[r[1] - r[0], r[6] - r[1], r[7] - r[6], r[2] - r[7], r[3] - r[2], r[4] - r[3], r[5] - r[4]]
                           for r in rows], np.float64)
            gaps = np.array([rows[j + 1][0] - rows[j][5] for j in range(len(rows) - 1)], np.float64)
            print("  trace panels", len(rows), "median cycles:",
                  {n: float(np.median(dd[:, j])) for j, n in enumerate(names)},
                  "gap", float(np.median(gaps)) if len(gaps) else None, flush=True)


if __name__ == "__main__":
    main()
