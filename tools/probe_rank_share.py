"""Probe: one rank's share of the sharded bench step at G GPUs, timed on one GPU.

At G GPUs (bench.py under torch.distributed.run) a rank projects and quantizes B/G of the faces,
searches its N/G gallery rows for the whole batch and merges.  This probe runs those pieces at the
sizes one rank sees (no collectives: they are absent on one GPU) and times each with HIP events,
so the fixed costs that do not shrink with G show up beside the tile pass that does:
projection + quantization of B/G faces, the fp6 sample pass + thresholds + sieve pass over N/G
rows, the split merge (stage 1, stage 2), and the whole local step.  One JSON line.
Round 6: the bench's operating point by default -- the Fisherfaces W trained on configs[1]
(--w trained) and the batch's start tier (f6p, the prefix tier, on that W) -- and the bytes of the
two query all-gathers a rank receives (the quantized query panels, the fp32 rows).

    python tools/probe_rank_share.py [--gpus 8] [--reps 10] [--w trained|random]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import round_up  # noqa: E402
from opencv_facerecognizer_amd.synthetic import (SEED, IdentityBank, build_gallery, build_projection,  # noqa: E402
                                                 build_trained_projection)


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--gallery", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--w", default="trained", choices=("trained", "random"))
    a = ap.parse_args()
    dev = _lib.device()
    side, d, per_id, B, k, G = 100, 9999, 10, a.batch, 1, a.gpus
    N = a.gallery // G
    bank = IdentityBank(-(-a.gallery // per_id), side, side, device=dev)   # row j shows identity j // per_id
    if a.w == "trained":
        P, _, _ = build_trained_projection(bank, per_id, 100_000, side * side, dev)
        d = P.d
    else:
        P, _ = build_projection(side * side, d, dev)
    ld = round_up(d, 32)
    g = build_gallery(P, bank, per_id, 0, N, a.gallery, d, ld, dev)          # rank 0's rows
    tier = g.start_tier(B)
    g._tier_gallery(tier)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    ids = torch.randint(0, a.gallery // per_id, (B,), generator=gq, device=dev)
    Xq = bank.images(ids, seed=SEED + 99)
    b1 = B // G
    Qloc = torch.zeros((b1, ld), dtype=torch.float32, device=dev)
    Qd = torch.zeros((B, ld), dtype=torch.float32, device=dev)
    P.project(Xq, shift64=g.shift64, out=Qd)
    qq = g.quantize_queries(Qd, tier=tier)
    ql = {}

    def prep():
        P.project(Xq[:b1], shift64=g.shift64, out=Qloc)
        ql["q"] = g.quantize_queries(Qloc, ql.get("q"), tier=tier)

    ub_loc = torch.empty((B, k), dtype=torch.float64, device=dev)
    out = (torch.empty((B, k), dtype=torch.float64, device=dev), torch.empty((B, k), dtype=torch.int64, device=dev))

    def tiles():
        g.search_q8_phase(1, Qd, qq, k)

    def stage1():
        g.merge_pruned(1, Qd, qq, k, ub_loc)

    ub = torch.full((B,), float("inf"), dtype=torch.float64, device=dev)

    def stage2():
        g.merge_pruned(2, Qd, qq, k, ub, 0, out)

    def local_step():
        prep()
        tiles()
        stage1()
        ub.copy_(ub_loc[:, k - 1])
        stage2()

    tiles()
    stage1()
    # the global bound at G ranks: for a query whose identity lives on this shard (rows 10 i .. 10 i + 9
    # below N) this shard's own k-th bound; for the others the owner's k-th distance, far below this
    # shard's candidates -- emulated by 0, which prunes every candidate (merge_sharded's stage 2 then
    # re-ranks nothing for that query, as on a real foreign shard)
    own = (ids * per_id + per_id - 1) < N
    ub_own = ub_loc[:, k - 1].clone()
    ub.copy_(torch.where(own, ub_own, torch.zeros_like(ub_own)) if G > 1 else ub_own)
    res = {"gpus": G, "w": a.w, "tier": tier, "pstages": g.prefix_stages() if tier == "f6p" else 0, "rows_per_rank": N, "batch": B, "faces_projected_per_rank": b1,
           "queries_owned_by_this_shard": int(own.sum()),
           "prep_ms": timed(prep, a.reps), "tiles_ms": timed(tiles, a.reps), "merge_stage1_ms": timed(stage1, a.reps),
           "merge_stage2_ms": timed(stage2, a.reps), "local_step_ms": timed(local_step, a.reps)}
    # bench.py's pipelined step: the next batch's preparation runs on a side stream beside this batch's
    # merge, so the critical path is the tile pass + max(merge, preparation) (collectives not included)
    res["pipelined_step_ms"] = res["tiles_ms"] + max(res["merge_stage1_ms"] + res["merge_stage2_ms"], res["prep_ms"])
    full = {"prep_full_batch_ms": timed(lambda: (P.project(Xq, shift64=g.shift64, out=Qd),
                                                 g.quantize_queries(Qd, qq, tier=tier)), a.reps)}
    res.update(full)
    res["uncertified_local"] = int((qq["cert"] == 0).sum())
    # a rank receives G-1 of the G shares of each all-gathered query array (parallel.gather_queries:
    # the tier's quantized panels; gather_rows_async: the fp32 rows)
    qbytes = sum(t.numel() * t.element_size() for key, t in ql["q"].items()
                 if isinstance(t, torch.Tensor) and key in ("Qs", "Qs2", "scale", "stats"))
    res["allgather_bytes_received"] = {"query_panels": qbytes * (G - 1), "fp32_rows": b1 * ld * 4 * (G - 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
