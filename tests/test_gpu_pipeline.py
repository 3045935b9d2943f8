"""bench.py's StepPipeline (the timed step's schedule): the tile pass of batch s on the
main stream (sample pass, then sieve pass), batch s-1's merge on a side stream behind sample pass s
(merge_at "sieve") or behind the whole tile pass s (merge_at "after", with batch s+1's preparation on
the main stream behind that merge), batch s-1's certificate read and fallback tiers, three query
buffers and two search workspaces.  Every batch's final top-k must equal the one-shot search of the same batch
(quantize, ofr_knn_f6 phases 1+2, fallback tiers) on the default stream -- bit for bit: the schedule
changes only which stream runs a kernel and which buffer it reads."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _setup(noise, N=20_000, d=512, side=32, per=10, B=512, batches=5):
    from opencv_facerecognizer_amd._device import round_up
    from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank, build_gallery, build_projection
    dev = torch.device("cuda", 0)
    n_ids = N // per
    P, _ = build_projection(side * side, d, dev)
    bank = IdentityBank(n_ids, side, side, device=dev)
    g = build_gallery(P, bank, per, 0, N, N, d, max(32, round_up(d, 32)), dev, noise=noise)
    gq = torch.Generator(device=dev)
    gq.manual_seed(SEED + 11)
    X = [bank.images(torch.randint(0, n_ids, (B,), generator=gq, device=dev), seed=SEED + 100 + s, noise=noise)
         for s in range(batches)]
    return P, g, X


@pytest.mark.parametrize("merge_at", ["after", "sieve", "sample", "prep", "tail"])
@pytest.mark.parametrize("noise", [12.0, 40.0])
def test_step_pipeline_matches_one_shot(noise, merge_at):
    """noise 40: crowded identities, so the fallback tiers run inside finish() while the next tile
    pass and the next preparation are in flight.  merge_at "after" (the default since round 6): the
    merge behind the tile pass and the next preparation on the main stream behind it."""
    from bench import StepPipeline
    P, g, X = _setup(noise)
    k, dev = 3, torch.device("cuda", 0)
    for t in g.tier_path("f6")[:-1]:
        g._tier_gallery(t)

    # one-shot, serial, default stream
    want, fell = [], 0
    for Xs in X:
        Qd = P.project(Xs, shift64=g.shift64)
        qq = g.quantize_queries(Qd, tier="f6")
        out = g.search_q8_phase(3, Qd, qq, k)
        fell += g.fallback(Qd, qq, k, out)
        want.append((out[0].cpu(), out[1].cpu()))

    B, ld = X[0].shape[0], g.ld
    bufs = [dict(Qd=torch.zeros((B, ld), dtype=torch.float32, device=dev), qq=None,
                 out=(torch.empty((B, k), dtype=torch.float64, device=dev),
                      torch.empty((B, k), dtype=torch.int64, device=dev))) for _ in range(StepPipeline.NBUF)]
    order = []           # batch index per preparation, in enqueue order
    got = []

    def prep(j, hook=None):
        s = len(order)
        order.append(s)
        bufs[j]["batch"] = s
        if hook is None:
            P.project(X[s], shift64=g.shift64, out=bufs[j]["Qd"])
        else:   # "tail": the projection in two tile ranges, the merge launched between them
            nt = P.tile_count(B)
            assert nt >= 2
            P.project(X[s], shift64=g.shift64, out=bufs[j]["Qd"], tiles=(0, nt // 2))
            hook()
            P.project(X[s], shift64=g.shift64, out=bufs[j]["Qd"], tiles=(nt // 2, nt))
        bufs[j]["qq"] = g.quantize_queries(bufs[j]["Qd"], bufs[j]["qq"], tier="f6")

    def tiles(j, w, part):
        g.search_q8_phase(4 if part == "sample" else 8, bufs[j]["Qd"], bufs[j]["qq"], k, workspace=w)

    def merge(j, w):
        g.search_q8_phase(2, bufs[j]["Qd"], bufs[j]["qq"], k, out=bufs[j]["out"], workspace=w)

    def finish(j):
        b = bufs[j]
        g.fallback(b["Qd"], b["qq"], k, b["out"])
        got.append((b["batch"], b["out"][0].clone(), b["out"][1].clone()))
        return b["out"]

    pipe = StepPipeline(dev, prep, tiles, merge, finish, merge_at=merge_at)
    assert pipe.side is not pipe.main
    pipe.run(len(X))
    torch.cuda.synchronize()
    assert order == list(range(len(X)))
    assert [s for s, _, _ in got] == list(range(len(X)))
    for s, d_, i_ in got:
        assert torch.equal(i_.cpu(), want[s][1]), f"batch {s}: indices differ"
        assert torch.equal(d_.cpu(), want[s][0]), f"batch {s}: distances differ"
    print(f"noise {noise}: {fell} first-tier failures over {len(X)} batches")


def test_adaptive_start_tier_skips_failing_fp6(monkeypatch):
    """FloatGallery.start_tier: on clusters the fp6 tier cannot certify (>= 90 % fail, the f6x2 test's
    data), the second batch starts at f6x2; the results equal the fixed-start chain's bit for bit,
    and every REPROBE-th batch starts at fp6 again.  (The merge's deep continuation off: with it the fp6
    tier certifies these clusters itself.)"""
    import numpy as np
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    monkeypatch.setenv("OFR_MERGE_DEEP", "0")
    r = np.random.default_rng(3)
    d, K, per, B = 128, 200, 40, 300
    mu = r.normal(0, 1, (K, d))
    G = (mu[np.arange(K * per) % K] + r.normal(0, 0.5, (K * per, d))).astype(np.float32).astype(np.float64)
    Q = (mu[r.integers(0, K, B)] + r.normal(0, 0.5, (B, d))).astype(np.float32).astype(np.float64)
    monkeypatch.setenv("OFR_ADAPTIVE_TIER", "0")
    fixed = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    want = fixed.search(fixed.query_rows(Q), 2)
    assert fixed.last_fallbacks[0] >= 0.9 * B, fixed.last_fallbacks
    monkeypatch.setenv("OFR_ADAPTIVE_TIER", "1")
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    starts = []
    for it in range(FloatGallery.REPROBE + 1):
        dd, ii = g.search(g.query_rows(Q), 2)
        starts.append(g.last_start_tier)
        assert torch.equal(ii, want[1]) and torch.equal(dd, want[0]), (it, starts)
    assert starts[0] == "f6" and starts[1] == "f6x2", starts
    assert starts[FloatGallery.REPROBE - 1] == "f6", starts          # the re-probe
    assert starts.count("f6") == 2, starts
    g.append(G[:3])                                                   # new rows: statistics start over
    assert g.tier_failures == {} and g.start_tier(B) in ("f6",)
