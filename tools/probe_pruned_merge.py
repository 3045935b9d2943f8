"""Probe: the pruned split merge of a sharded gallery (parallel.merge_sharded) on one GPU.

Two shards of the bench's synthetic gallery live in one process: "own" holds the queries'
identities, "foreign" holds none of them (at G = 8, 7 of every query's 8 shards are foreign).
Times, per shard, the plain phase-2 merge against the split merge: stage 1 (selection + upper
bounds), the global bound (k-th smallest over both shards, computed here instead of all-gathered),
stage 2 (the pruned re-rank).  HIP events; one JSON line.

    python tools/probe_pruned_merge.py [--rows 125000]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402


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
    ap.add_argument("--rows", type=int, default=125_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = _lib.device()
    side, d, per_id, B, N, k = 100, 9999, 10, a.batch, a.rows, 1
    P, _ = bench.build_projection(side * side, d, dev)
    bank = IdentityBank(2 * N // per_id, side, side, device=dev)
    ld = bench.round_up(d, 32)
    own = bench.build_gallery(P, bank, per_id, 0, N, 2 * N, d, ld, dev)           # rows [0, N)
    foreign = bench.build_gallery(P, bank, per_id, N, N, 2 * N, d, ld, dev)       # rows [N, 2N)
    assert torch.equal(own.shift64, foreign.shift64)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 7)
    ids = torch.randint(0, N // per_id, (B,), generator=gq, device=dev)            # identities of "own"
    Qd = torch.zeros((B, ld), dtype=torch.float32, device=dev)
    P.project(bank.images(ids, seed=SEED + 99), shift64=own.shift64, out=Qd)
    res = {"rows_per_shard": N, "B": B, "k": k}
    state = {}
    for name, g, base in (("own", own, 0), ("foreign", foreign, N)):
        g._tier_gallery("f6")
        qq = g.quantize_queries(Qd, tier="f6")
        out = g.search_q8_phase(1, Qd, qq, k, base)
        res[name] = {"plain_merge_ms": timed(lambda: g.search_q8_phase(2, Qd, qq, k, base, out=out), a.reps)}
        ubl = torch.empty((B, k), dtype=torch.float64, device=dev)
        res[name]["stage1_ms"] = timed(lambda: g.merge_pruned(1, Qd, qq, k, ubl, base), a.reps)
        state[name] = (g, qq, out, ubl, base)
    ub = torch.cat([state["own"][3], state["foreign"][3]], 1).kthvalue(k, dim=1).values.contiguous()
    for name in ("own", "foreign"):
        g, qq, out, _, base = state[name]
        res[name]["stage2_ms"] = timed(lambda: g.merge_pruned(2, Qd, qq, k, ub, base, out), a.reps)
        res[name]["queries_reranked"] = int(torch.isfinite(out[0][:, 0]).sum())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
