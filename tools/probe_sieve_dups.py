"""Probe: the fp6 sieve on a shard of identical rows (test_config2_sharded_overflow's rank 1 data):
kept rows per query and the distinct coarse keys of the kept rows, for the engine OFR_F6_SHAPE selects.
One JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery, center_round, f64_dev, round_up
    r = np.random.default_rng(1234)
    d = 96
    x = r.normal(0, 20, d)
    G = np.concatenate([r.normal(0, 20, (34000, d)), np.tile(x, (34000, 1))]).astype(np.float32).astype(np.float64)
    Q = (x + r.normal(0, 0.5, (40, d))).astype(np.float32).astype(np.float64)
    n0, n1 = 34000, 68000
    shift = f64_dev(G.mean(0))
    Gd = center_round(f64_dev(G[n0:n1]), shift, max(32, round_up(d, 32)))
    g = FloatGallery.from_device_rows(Gd, d, _lib.METRIC_EUCLIDEAN, shift64=shift)
    Qd = center_round(f64_dev(Q), shift, g.ld)
    qq = g.quantize_queries(Qd, tier="f6")
    g.search_q8_phase(1, Qd, qq, 3, index_base=n0)
    torch.cuda.synchronize()
    kept = g.sieve_counts(len(Q)).cpu().numpy()
    lib = _lib.load()
    B, N = len(Q), g.N
    ws = g.ws.buf
    off_b = int(lib.ofr_knn_f6_sieve_counts_offset(B, N)) + ((B * 4 + 255) // 256) * 256
    cap = 32768
    bucket = ws[off_b: off_b + B * cap * 8].view(torch.int32).view(B, cap, 2).cpu().numpy()
    q0 = int(np.argmax(kept))
    n = min(int(kept[q0]), cap)
    keys = bucket[q0, :n, 0].view(np.float32)
    rows = bucket[q0, :n, 1]
    theta = ws[int(lib.ofr_knn_f6_sieve_counts_offset(B, N)) - ((B * 4 + 255) // 256) * 256:][:B * 4].view(torch.int32).cpu().numpy()
    print(json.dumps({"engine": os.environ.get("OFR_F6_SHAPE", "default"), "kept": kept.tolist()[:8],
                      "kept_max": int(kept.max()), "query": q0, "distinct_keys": int(len(np.unique(keys))),
                      "key_values": [float(v) for v in np.unique(keys)[:6]],
                      "rows_min": int(rows.min()) if n else None, "rows_max": int(rows.max()) if n else None,
                      "distinct_rows": int(len(np.unique(rows))),
                      "missing_row_blocks_of_128": sorted(set(int(v) for v in np.setdiff1d(np.arange(N), rows - 0) // 128))[:40]}))


if __name__ == "__main__":
    main()
