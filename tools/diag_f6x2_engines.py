"""Diagnostic: the two-slice tier's sieve buckets on the wide engine (tile_kernel_f6w<3>) against the 8-wave
engine (OFR_F6_SHAPE=16) on the data of tests/test_gpu_sieve.py::test_f6x2_wide_engine_matches_8wave_engine;
prints per query the rows kept by one engine only, with their position in the wide engine's tile
(tile, wave row WR, row block, lane group)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_sieve import _clustered  # noqa: E402

from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import FloatGallery  # noqa: E402

torch.cuda.set_device(0)
G, Q = _clustered(2003, 9, 320, 300, 31)
g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
Qd = g.query_rows(Q)
st = {}
for eng in ("wide", "8wave"):
    if eng == "8wave":
        os.environ["OFR_F6_SHAPE"] = "16"
    else:
        os.environ.pop("OFR_F6_SHAPE", None)
    qq = g.quantize_queries(Qd, tier="f6x2")
    g.search_q8_phase(4 | 8 | 2, Qd, qq, 4)
    torch.cuda.synchronize()
    theta, count, keys, rows = g.sieve_state(len(Q))
    c = count.cpu().numpy().copy()
    st[eng] = [(dict(zip(rows[b, :c[b]].cpu().numpy().tolist(), keys[b, :c[b]].cpu().numpy().view(np.uint32).tolist())))
               for b in range(len(Q))]
nd = 0
for b in range(len(Q)):
    w, e = st["wide"][b], st["8wave"][b]
    only_w = sorted(set(w) - set(e))
    only_e = sorted(set(e) - set(w))
    diff_k = [r for r in set(w) & set(e) if w[r] != e[r]]
    if only_w or only_e or diff_k:
        nd += 1
        if nd <= 12:
            loc = lambda r: (r // 384, (r % 384) // 192, ((r % 192) // 16), (r % 16) // 4)
            print("query", b, "tile/WR/block/lanegrp only wide", [(r, loc(r)) for r in only_w[:6]],
                  "only 8wave", [(r, loc(r)) for r in only_e[:6]], "key diffs", len(diff_k), "qpanel", b // 256,
                  "WC", (b % 256) // 128, "colblock", (b % 128) // 16)
print("queries differing:", nd, "of", len(Q))
