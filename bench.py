"""Headline benchmark: query faces/sec, Fisherfaces projection + 1-NN against a 1M-image gallery.

Workload (BASELINE.json configs[2], which fits one MI355X: the 1M x 9999 fp32
gallery is 40 GB of the 288 GB HBM): synthetic 100x100 uint8 faces (D=10000),
a Fisherfaces projection to d=9999 (= c-1 for 10k identities, thetrainer.py
get_model defaults), a 1M-row gallery (100k identities x 10 images), batches of
B=4096 query faces, k=1, Euclidean distance.  One step = project the batch
(ofr_project_u8_exact: int8-slice MFMA, exact) + quantize it to fp6 + the fp6
sample and sieve passes (ofr_knn_f6 phase 1) + merge / exact fp64 re-rank /
certificate (phase 2) + the fallback tiers of the uncertified queries
[+ the RCCL exchanges of DESIGN.md §6 when sharded].  --search fp32 runs the
fp32-MFMA pass (ofr_knn_tiles_f32) instead.  The steps are pipelined over three
query buffers (StepPipeline): the tile pass owns the main stream, the next
batch's preparation and this batch's merge follow it on a side stream.
Inputs are resident in HBM before the timed region.  W is the Fisherfaces W the
reference's trainer produces (thetrainer.py:120-124, Fisherfaces() defaults) from
configs[1]'s synthetic training set (10k identities x 10 faces), trained on the
device in the untimed setup ("1M images projected with config-2 W");
--w random keeps the round-1..4 random N(0, 1/D) W.  Gallery/queries are synthetic
(see opencv_facerecognizer_amd/synthetic.py).

Multi-GPU (torch.distributed.run, one process per GPU): the 1M gallery is
sharded by rows over the ranks; each rank projects and quantizes B/G of the
query faces and the centred fp32 rows + fp6 panels are all-gathered (RCCL), every
rank searches its shard for the whole batch, and the per-rank top-k lists are
merged after one RCCL all-gather -> strong scaling (total work fixed).
OFR_DIST_BACKEND=gloo OFR_ONE_DEVICE=1 rehearse the multi-rank path on one GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import FloatGallery, Workspace, round_up  # noqa: E402
from opencv_facerecognizer_amd.parallel import (certify_sharded, exchange_topk, gather_rows, gather_rows_async,  # noqa: E402
                                                merge_sharded, merge_topk, shard_range, share_block_scales)
from opencv_facerecognizer_amd.synthetic import (SEED, IdentityBank, build_gallery, build_projection,  # noqa: E402
                                                 build_trained_projection)

PEAK_FP32_MFMA = 157.3e12   # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (spec)
PEAK_I8_MFMA = 5.0e15       # int8 MFMA: 2x the ~2.5 PF dense bf16 rate (MI355X_MICROARCH.md, matrix cores)
PEAK_F6_MFMA = 10.0e15      # fp6 (block-scaled f8f6f4 MFMA): ~10 PF dense, the FP4 rate (MI355X_MICROARCH.md)
# what the chip sustains on v_mfma_scale_f32_16x16x128_f8f6f4 (fp6 x fp6) with every CU busy and the
# operands in registers, at the clock it holds under that load (tools/f6_shape_probe.hip,
# profiles/r02_f6_shape_probe.log): the ceiling of any fp6 kernel on this part
SUSTAINED_F6_MFMA = 6.28e15
PEAK_HBM = 8.0e12           # HBM3E 8 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gallery", type=int, default=1_000_000)
    ap.add_argument("--per-id", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dim", type=int, default=9999)
    ap.add_argument("--side", type=int, default=100)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--small-batches", default="32,1", help="extra HBM-regime measurements (B <= 32); '' to skip")
    ap.add_argument("--stress", default="48,96,192",
                    help="pixel-noise levels of the crowded-neighbour stress runs (same shape, 1 GPU); '' to skip")
    ap.add_argument("--stress-steps", type=int, default=3)
    ap.add_argument("--config1", type=int, default=1, help="also time configs[1] (100k-row gallery), 1 GPU")
    ap.add_argument("--w", choices=["trained", "random"], default="trained",
                    help="trained: Fisherfaces W trained on configs[1]'s 100k faces (SURVEY §8d); random: N(0, 1/D)")
    ap.add_argument("--train-ids", type=int, default=10_000, help="identities of the W training set (x --per-id faces)")
    ap.add_argument("--config4", type=int, default=1,
                    help="1 GPU: train the headline's W through the reference API (PredictableModel(Fisherfaces(), "
                         "NearestNeighbor()).compute on configs[1]'s faces) and report it as configs[4]; 0: the "
                         "device-only training pipeline (untimed)")
    ap.add_argument("--api", type=int, default=1,
                    help="1 GPU, with --config4: configs[1] through PredictableModel.predict_batch on host faces")
    ap.add_argument("--config3", type=int, default=1,
                    help="1 GPU: configs[3] (LBPH: ExtendedLBP + SpatialHistogram + ChiSquare 1-NN) through the API")
    ap.add_argument("--search", choices=["f6", "q8", "fp32"], default="f6",
                    help="f6: certified fp6 coarse pass (uncertified queries go down the int8 tiers, then fp32); "
                         "q8: start at the certified int8 tier; fp32: fp32-MFMA pass")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(P, gallery, Xq, N_total, seconds):
    """Reference-faithful oracle (classifier.py:104-108 loop, 1 Python thread) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import facerec_oracle as O  # the checker; timed here as the CPU baseline
    n_s = min(4000, gallery.N)
    G_s = gallery.G[:n_s, : gallery.d].double().cpu().numpy() + gallery.shift64.cpu().numpy()
    W = P.weights_f64().cpu().numpy()                         # D x d, float64 like the reference
    X = Xq.cpu().numpy()
    t_proj, t_item, nq = 0.0, 0.0, 0
    deadline = time.perf_counter() + seconds
    while time.perf_counter() < deadline and nq < len(X):
        t0 = time.perf_counter()
        q = O.fisherfaces_project(W, X[nq])                  # feature.py:241-242
        t1 = time.perf_counter()
        for gi in G_s:                                       # classifier.py:104-108
            O.euclidean(gi.reshape(-1, 1), q)
        t2 = time.perf_counter()
        t_proj += t1 - t0
        t_item += (t2 - t1) / n_s
        nq += 1
    per_query = t_proj / nq + (t_item / nq) * N_total
    # vectorised float64 mode (BLAS dgemm, all BLAS threads) on the same sample: projection of a batch
    # and ||q||^2 + ||g||^2 - 2 q.g distances, extrapolated linearly in N
    nv = min(256, len(X))
    t0 = time.perf_counter()
    Qv = X[:nv].astype(np.float64) @ W
    t1 = time.perf_counter()
    O.nn_search_blas(Qv, G_s, 1)
    t2 = time.perf_counter()
    per_query_vec = (t1 - t0) / nv + (t2 - t1) / nv * (N_total / n_s)
    blas_threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {
        "value": 1.0 / per_query, "unit": "queries/s", "cores": 1, "kind": "port",
        "sample": f"{nq} queries x {n_s} gallery rows, d={gallery.d}, D={W.shape[0]}: reference-faithful per-item "
                  f"distance loop + W^T x, extrapolated linearly to N={N_total}",
        "per_item_us": 1e6 * t_item / nq, "projection_ms": 1e3 * t_proj / nq,
        "vectorized_f64": {"value": 1.0 / per_query_vec, "unit": "queries/s", "cores": blas_threads,
                           "sample": f"{nv} queries x {n_s} rows, float64 BLAS (dgemm) projection + distances, "
                                     f"extrapolated to N={N_total}"},
    }


def sieve_engine(name):
    """Short name of the sieve-pass kernel a roofline / PMC record refers to (the committed traffic of one
    engine is never attributed to another)."""
    for e in ("prefix_wave_kernel", "prefix_pass_kernel", "tile_kernel_f6p", "tile_kernel_f6w", "tile_kernel_f6s", "tile_kernel<1>",
              "knn_tile_kernel"):
        if e in (name or ""):
            return e
    return "other"


def committed_traffic(cfg):
    """HBM-side bytes per launch of the search pass from the committed rocprofv3 PMC passes
    (profiles/*_pmc_summary.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950 guide), if measured at this
    config: among the summaries of this exact config (W kind included; summaries without one were
    measured on the random W) the one with the latest measured_utc (written by tools/pmc_summary.py;
    summaries without it count as older than any with it).  (bytes, file) or None."""
    import glob
    cands = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")):
        try:
            s = json.load(open(f))
        except (OSError, ValueError):
            continue
        c = dict(s.get("config") or {})
        c.setdefault("w", "random")
        c.setdefault("tier", c.get("search"))         # summaries before the prefix tier: the search's tier
        c.setdefault("engine", sieve_engine(s.get("kernel")))   # summaries before round 6: from their kernel
        if c == cfg and s.get("traffic_bytes_per_launch") is not None:
            cands.append((s.get("measured_utc", ""), os.path.basename(f), s["traffic_bytes_per_launch"]))
    if not cands:
        return None
    _, name, tr = max(cands)
    return tr, os.path.join("profiles", name)


class StepPipeline:
    """The timed step's schedule over a sequence of query batches.  Default since late round 6
    (merge_at "tail", one GPU): as "after" below, except that merge s-1 runs beside the last, partial round of
    preparation s+1's projection (prep's hook, project_split).  merge_at "after" (round 6; N > 1): one kernel at a time, in the order sample pass s, sieve pass s, merge s-1 (side
    stream, behind the sieve pass), preparation s+1 (main stream, behind that merge), with the host's
    certificate read of batch s-1 (a sync of the side stream only) issued after preparation s+1 is queued.
    merge_at "sieve" (rounds 3-5):

      main stream  tile pass of batch s (behind its preparation): its sample pass + thresholds, then
                   its sieve pass;
      side stream  behind sample pass s: batch s-1's merge (exact re-rank + certificate), which so
                   runs under sieve pass s and leaves the short sample pass alone; behind tile pass s:
                   batch s+1's preparation (projection, quantization, its all-gathers), which runs
                   alone;
      host         batch s-1's certificate read (one sync, on the side stream up to merge s-1,
                   which finishes early in sieve pass s) and its fallback tiers, enqueued on the side
                   stream before batch s+1's preparation.

    Three query buffers (preparation s+1 / merge s / fallback s-1), two search workspaces (tile
    pass s writes one while merge s-1 reads the other).  Callbacks, each enqueueing on the current
    stream: prep(j) fills buffer j; tiles(j, w, part) runs part "sample" (sample pass + thresholds)
    or "sieve" of phase 1 of buffer j on workspace w, merge(j, w) phase 2; finish(j) reads the
    certificate (host sync) and runs the fallback, returning the batch's result.  overlap=False: one
    stream, the same order."""

    NBUF, NWS = 3, 2

    def __init__(self, device, prep, tiles, merge, finish, overlap=True, prep_behind=None, merge_at=None):
        self.prep_fn, self.tiles_fn, self.merge_fn, self.finish_fn = prep, tiles, merge, finish
        # prep_behind "tiles" (default): batch s+1's preparation waits for tile pass s and runs alone;
        # "sample": it waits only for sample pass s and shares the chip with sieve pass s
        self.prep_behind = prep_behind or os.environ.get("OFR_BENCH_PREP", "tiles")
        assert self.prep_behind in ("tiles", "sample"), self.prep_behind
        # merge_at "after" (default, round 6): merge s-1 behind sieve pass s, then batch s+1's preparation
        # on the main stream behind that merge -- every kernel alone on the chip, and the host's certificate
        # read (side stream, up to the merge) never leaves the GPU without queued work.  Neither the
        # persistent prefix pass (two workgroups per CU) nor the projection leaves a CU room for merge
        # blocks: run beside the sieve pass, the merge held its CUs and the pass (whose work items are
        # dealt statically) ended with its last workgroups: 0.83 -> 1.59 ms for 0.47 ms of merge
        # (profiles/r06_merge_at_ab.txt).  "sieve": merge s-1 under sieve pass s (rounds 3-5).
        # "sample": merge s-1 beside sample pass s (both behind preparation s), sieve pass s behind both, then
        # preparation s+1 -- the short sample pass and the HBM-bound merge share the chip, everything else
        # runs alone
        # "prep": merge s-1 behind tile pass s on the side stream, beside preparation s+1 on the main one
        self.merge_at = merge_at or os.environ.get("OFR_BENCH_MERGE", "tail")
        # "tail" (the default since late round 6): as "after", but merge s-1 waits only for the full rounds of
        # preparation s+1's projection and runs beside its last, partial round (144 of 1,680 tiles on 256 CUs:
        # 112 CUs idle), the prep function taking a hook it calls between the two launches: 2.335 -> 2.29 ms
        # per step (profiles/r06_merge_tail_ab.txt)
        assert self.merge_at in ("after", "sieve", "sample", "prep", "tail"), self.merge_at
        self.main = torch.cuda.current_stream(device)
        self.side = torch.cuda.Stream(device=device) if overlap else self.main
        self.ws = [Workspace() for _ in range(self.NWS)]
        self.ev_ready = [torch.cuda.Event() for _ in range(self.NBUF)]    # buffer prepared (side)
        self.ev_merged = [torch.cuda.Event() for _ in range(self.NWS)]    # workspace's merge done (side)
        self.ev_tiles = torch.cuda.Event()                                # latest tile pass done (main)
        self.ev_sample = torch.cuda.Event()                               # latest sample pass done (main)
        self.ev_parta = torch.cuda.Event()                                # projection's full rounds done (tail)
        self.ev_done = [torch.cuda.Event() for _ in range(self.NBUF)]     # buffer's fallback done (side)
        # the side stream starts behind everything the main stream has queued (gallery and tier builds,
        # the query images, buffer fills): an unrecorded event is no dependency, and once the caching
        # allocator stops calling hipMalloc (which synchronises) nothing else would order the first
        # preparations (without this, a second run in one process projected stale queries)
        if self.side is not self.main:
            self.side.wait_stream(self.main)

    def _prep(self, s, ev, stream=None, hook=None):
        with torch.cuda.stream(stream or self.side):
            if ev:
                ev[0].record()
            if hook is None:
                self.prep_fn(s % self.NBUF)
            else:
                self.prep_fn(s % self.NBUF, hook)
            if ev:
                ev[1].record()
            self.ev_ready[s % self.NBUF].record(stream or self.side)

    def _finish(self, s):
        with torch.cuda.stream(self.side):
            return self.finish_fn(s % self.NBUF)

    def _merge_tail(self, s, ev):
        """The prep hook of merge_at "tail" (called on the main stream between the projection's launches)."""
        self.ev_parta.record(self.main)
        self._merge(s, ev, after=self.ev_parta)

    def _merge(self, s, ev, after=None):
        j, w = s % self.NBUF, s % self.NWS
        with torch.cuda.stream(self.side):
            # behind the next batch's sample pass ("sieve"), its preparation ("sample") or its whole tile pass
            # ("after"); "tail": behind the full rounds of the next preparation's projection
            if after is not None:
                self.side.wait_event(after)
            elif self.merge_at == "sample":   # (the tile pass too: the last batch has no next preparation)
                self.side.wait_event(self.ev_tiles)
                self.side.wait_event(self.ev_ready[(s + 1) % self.NBUF])
            else:
                self.side.wait_event(self.ev_sample if self.merge_at == "sieve" else self.ev_tiles)
            if ev:
                ev[5].record()
            self.merge_fn(j, self.ws[w])
            if ev:
                ev[3].record()
            self.ev_merged[w].record(self.side)

    def run(self, steps, events=None):
        """Exactly `steps` preparations, tile passes, merges and fallbacks; returns the last batch's
        result.  events[s]: 7 timing events (prep start/end on the side stream, tile pass end and start
        on the main stream, merge end and start on the side stream, sample pass end on the main stream)."""
        ev = events or [None] * steps
        res = None
        self._prep(0, ev[0])
        for s in range(steps):
            j, w = s % self.NBUF, s % self.NWS
            self.main.wait_event(self.ev_ready[j])
            self.main.wait_event(self.ev_merged[w])         # merge s-2 done with this workspace
            if ev[s]:
                ev[s][4].record(self.main)
            if s >= 1 and self.merge_at == "sample":        # merge s-1 beside sample pass s
                self._merge(s - 1, ev[s - 1])
            self.tiles_fn(j, self.ws[w], "sample")
            self.ev_sample.record(self.main)
            if ev[s]:
                ev[s][6].record(self.main)
            if s >= 1 and self.merge_at == "sieve":         # merge s-1 under sieve pass s
                self._merge(s - 1, ev[s - 1])
            if s >= 1 and self.merge_at == "sample":        # sieve pass s alone: behind merge s-1
                self.main.wait_event(self.ev_merged[(s - 1) % self.NWS])
            self.tiles_fn(j, self.ws[w], "sieve")
            if ev[s]:
                ev[s][2].record(self.main)
            self.ev_tiles.record(self.main)
            if self.merge_at in ("after", "sample", "prep", "tail"):
                tail = self.merge_at == "tail" and s >= 1 and s + 1 < steps
                if s >= 1 and (self.merge_at in ("after", "prep") or (self.merge_at == "tail" and not tail)):
                    self._merge(s - 1, ev[s - 1])           # merge s-1 behind tile pass s
                if s + 1 < steps:                           # preparation s+1 behind that merge, on main
                    if s >= 1 and self.merge_at not in ("prep", "tail"):
                        self.main.wait_event(self.ev_merged[(s - 1) % self.NWS])
                    self.main.wait_event(self.ev_done[(s + 1) % self.NBUF])   # its buffer's fallback done
                    hook = (lambda s_=s: self._merge_tail(s_ - 1, ev[s_ - 1])) if tail else None
                    self._prep(s + 1, ev[s + 1], stream=self.main, hook=hook)
                if s >= 1:
                    res = self._finish(s - 1)
                    self.ev_done[(s - 1) % self.NBUF].record(self.side)
                continue
            if s >= 1:
                res = self._finish(s - 1)
            self.side.wait_event(self.ev_tiles if self.prep_behind == "tiles" else self.ev_sample)
            if s + 1 < steps:
                self._prep(s + 1, ev[s + 1])
        if steps:
            self._merge(steps - 1, ev[steps - 1])
            res = self._finish(steps - 1)
            self.ev_done[(steps - 1) % self.NBUF].record(self.side)
        # the caller's stream sees everything the side stream did
        self.main.wait_stream(self.side)
        return res


def certificate_margin(gallery, Qd, qq, nsample=64):
    """(d_16^2 - d_1^2) / dS of the fp6 tier for a sample of queries: the certificate needs about 2
    (the 16th coarse candidate must clear the k-th exact distance by the bound on both sides).
    d from the exact fp32 path, dS = the bound merge_kernel uses.  The fp6 tier's own
    query stats (a batch that started at another tier is quantized for fp6 here)."""
    if qq.get("tier") != "f6":
        qq = gallery.quantize_queries(Qd, tier="f6")
    s = torch.arange(0, Qd.shape[0], max(1, Qd.shape[0] // nsample), device=Qd.device)[:nsample]
    dd, _ = gallery._search_f32(Qd.index_select(0, s).contiguous(), 16)
    dd = dd.cpu().numpy()
    st = qq["stats"].index_select(0, s).cpu().numpy()
    gmax = gallery._tier_gallery("f6")["gmax"].cpu().numpy()
    A, E, aux = gmax[0], gmax[1], gmax[3]
    a, e = st[:, 0], st[:, 1]
    gamma = (2 * -(-gallery.d // 128) + 64) * 2.0 ** -23
    dS = 2 * (a * E + e * A + e * E) + 2.0 ** -20 * (aux + 2 * a * A) + 2 * gamma * a * A
    r = (dd[:, 15] ** 2 - dd[:, 0] ** 2) / dS
    return {"median": float(np.median(r)), "min": float(r.min()), "sample": int(len(r))}


def train_config4(bank, per_id, n_train, H, W, device):
    """configs[4] through the reference API, timed: PredictableModel(Fisherfaces(), NearestNeighbor(
    EuclideanDistance(), k=1)).compute(list of n_train uint8 HxW faces, labels) -- thetrainer.py:113-124
    + :176 (TheTrainer.get_model / train), model.py:49-51, feature.py:211-235.  The faces are configs[1]'s
    training set (identities 0 .. n_train / per_id - 1, synthetic.gallery_chunks' seeds).  Returns the
    model (its W is the headline's, its classifier the configs[1] gallery of the training features)
    and the record: wall time, the device eigensolve split out (rocSOLVER dsygvd / dsyevd)."""
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    from opencv_facerecognizer_amd import _device as dv
    from opencv_facerecognizer_amd.synthetic import GALLERY_CHUNK
    D = H * W
    X = torch.empty((n_train, D), dtype=torch.uint8, device=device)
    for c0 in range(0, n_train, GALLERY_CHUNK):
        rows = torch.arange(c0, min(c0 + GALLERY_CHUNK, n_train), device=device)
        X[c0:c0 + len(rows)] = bank.images(rows // per_id, seed=SEED + 1000 + c0 // GALLERY_CHUNK)
    X_list = list(X.reshape(n_train, H, W).cpu().numpy())     # the reference's input: a list of 2-D images
    del X
    y = np.arange(n_train) // per_id
    eig = {"sygv_dsygvd": 0.0, "eigh_dsyevd": 0.0}
    saved = dv.sygv_desc_f64, dv.eigh_desc_f64

    def timed(name, fn):
        def w(*a, **kw):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = fn(*a, **kw)
            torch.cuda.synchronize()
            eig[name] += time.perf_counter() - t
            return r
        return w
    dv.sygv_desc_f64, dv.eigh_desc_f64 = timed("sygv_dsygvd", saved[0]), timed("eigh_dsyevd", saved[1])
    try:
        model = PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.compute(X_list, y)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    finally:
        dv.sygv_desc_f64, dv.eigh_desc_f64 = saved
    ff = model.feature
    rec = {"workload": f"configs[4]: PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))"
                       f".compute on {n_train} faces of {n_train // per_id} identities, {H}x{W} (D={D})",
           "wall_s": wall, "device_eigensolve_s": eig, "rest_s": wall - sum(eig.values()),
           "regime": getattr(ff, "_regime", "?"), "d": int(ff._num_components),
           "eigenvalues_head": [float(v) for v in np.asarray(ff._eigenvalues)[:4]],
           "note": "wall includes the host list -> device upload and the host (d, 1) feature matrices the API "
                   "returns; the W it trains is the headline's"}
    del X_list
    return model, rec


def api_predict(model, bank, n_ids, B, H, W, device, reps=3):
    """configs[1] through the reference API: PredictableModel.predict_batch (model.py:53-55 for a batch)
    on a host list of B uint8 HxW faces against the model's own 100k-row gallery.  Wall clock per call
    (stack + upload, projection, the certified search, the host results), and its parts."""
    from ocvfacerec.facerec.classifier import results
    gq = torch.Generator(device=device)
    gq.manual_seed(SEED + 37)
    ids_q = torch.randint(0, n_ids, (B,), generator=gq, device=device)
    Xq = list(bank.images(ids_q, seed=SEED + 98).reshape(B, H, W).cpu().numpy())
    model.predict_batch(Xq)                              # warm: the gallery's tiers, workspaces
    torch.cuda.synchronize()
    walls, parts = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        preds = model.predict_batch(Xq)
        walls.append(time.perf_counter() - t0)
    from opencv_facerecognizer_amd._device import upload_u8_items
    for _ in range(reps):                                # the same call in its three parts
        t0 = time.perf_counter()
        Xd = upload_u8_items(Xq, device)                 # predict_batch's staging (pinned, chunked)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        d_, i_ = model._search_device(Xd)
        dh, ih = d_.cpu().numpy(), i_.cpu().numpy()
        t2 = time.perf_counter()
        results(dh, ih, model.classifier.y)
        t3 = time.perf_counter()
        parts.append((t1 - t0, t2 - t1, t3 - t2))
    ms = 1e3 * float(np.median(walls))
    labels = np.array([p[0] for p in preds])
    g = model.classifier._gallery()
    pm = 1e3 * np.median(np.array(parts), axis=0)
    return {"workload": f"configs[1] through PredictableModel.predict_batch: a host list of {B} uint8 {H}x{W} faces "
                        f"against the trained model's {g.N}-row gallery",
            "queries_per_s": B / (ms * 1e-3), "ms_per_call": ms,
            "parts_ms": {"stack_and_upload": float(pm[0]), "projection_and_search": float(pm[1]),
                         "results_host": float(pm[2])},
            "gap_to_engine": "host staging of the B faces (a host list: stacked into pinned memory, copied to "
                             "the device) and the synchronous call (the engine's step pipeline overlaps the "
                             "next batch's preparation and this batch's merge with the tile passes)",
            "uncertified_after_each_tier": list(g.last_fallbacks),
            "top1_identity_acc": float(np.mean(labels == ids_q.cpu().numpy()))}


def config3_run(device, N=65536, B=4096, per_id=8, reps=3):
    """configs[3] through the reference API (tools/bench_lbph_model.py): PredictableModel(SpatialHistogram(
    ExtendedLBP(1, 8), (8, 8)), NearestNeighbor(ChiSquareDistance(), k=1)).compute on N 128x128 faces, then
    predict_batch of B query faces (feature.py:266-305, lbp.py:80-130, distance.py:112-116).  The chi2 pass's
    roofline: 16 fp16 MFMA flops per (pair, bin) of the low-rank form against 2.5 PF dense."""
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import ChiSquareDistance
    from ocvfacerec.facerec.feature import SpatialHistogram
    from ocvfacerec.facerec.lbp import ExtendedLBP
    from ocvfacerec.facerec.model import PredictableModel
    H = 128
    n_ids = (N + per_id - 1) // per_id
    bank = IdentityBank(n_ids, H, H, device=device)
    Xg = bank.images(torch.arange(N, device=device) // per_id, seed=SEED + 11).reshape(N, H, H).cpu().numpy()
    gq = torch.Generator(device=device)
    gq.manual_seed(SEED + 12)
    ids_q = torch.randint(0, n_ids, (B,), generator=gq, device=device)
    Xq = bank.images(ids_q, seed=SEED + 13).reshape(B, H, H).cpu().numpy()
    model = PredictableModel(SpatialHistogram(ExtendedLBP(1, 8), (8, 8)), NearestNeighbor(ChiSquareDistance(), k=1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.compute(list(Xg), np.arange(N) // per_id)
    torch.cuda.synchronize()
    t_compute = time.perf_counter() - t0
    del Xg
    model.predict_batch(Xq)
    torch.cuda.synchronize()
    walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        preds = model.predict_batch(Xq)
        walls.append(time.perf_counter() - t0)
    sh, clf = model.feature, model.classifier
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    Qd = torch.from_numpy(Xq).to(device)
    ms_h, ms_s = [], []
    for _ in range(reps):
        e[0].record()
        C, cell, cb = sh.counts_batch(Qd)
        e[1].record()
        clf.search_counts(C, cell, cb, 1)
        e[2].record()
        torch.cuda.synchronize()
        ms_h.append(e[0].elapsed_time(e[1]))
        ms_s.append(e[1].elapsed_time(e[2]))
    g = clf._gallery()
    ms = 1e3 * float(np.median(walls))
    flops = 16.0 * B * N * 16384
    ms_s_med = float(np.median(ms_s))
    labels = np.array([p[0] for p in preds])
    out = {"workload": f"configs[3]: PredictableModel(SpatialHistogram(ExtendedLBP(1, 8), (8, 8)), NearestNeighbor("
                       f"ChiSquareDistance(), k=1)): compute on {N} faces {H}x{H}, predict_batch of {B}",
           "queries_per_s": B / (ms * 1e-3), "ms_per_call": ms, "compute_s": t_compute,
           "device_ms": {"query_histograms": float(np.median(ms_h)), "chi2_search": ms_s_med},
           "chi2_roofline": {"kernel": "c2m::chi2_mfma_kernel + merge (ofr_chi2_knn, whole search)", "bound": "mfma",
                             "achieved": flops / (ms_s_med * 1e-3) / 1e12, "peak": 2500.0, "unit": "TFLOP/s",
                             "frac": flops / (ms_s_med * 1e-3) / 2.5e15,
                             "algorithmic_flops": flops},
           "chi2_uncertified_after_each_pass": list(g.last_fallbacks),
           "top1_identity_acc": float(np.mean(labels == ids_q.cpu().numpy()))}
    del model, clf, sh, g
    torch.cuda.empty_cache()
    return out


def feature_profile(gallery, rows=8192):
    """How the centred gallery features spread over the 32-feature blocks (the fp6 tier quantizes a
    row with ONE scale, so a row whose energy sits in a few blocks loses the rest to the step size),
    and the fp6 tier's residual ||x - x~|| / ||x~|| per row (the e / a of the certificate)."""
    n = min(rows, gallery.N)
    G = gallery.G[:n, :gallery.d].double()
    nb = -(-gallery.d // 32)
    Gp = torch.nn.functional.pad(G, (0, nb * 32 - gallery.d))
    rms = Gp.pow(2).reshape(n, nb, 32).mean(dim=(0, 2)).sqrt().cpu().numpy()
    st = gallery._tier_gallery("f6")["stats"][:n]
    rel = (st[:, 1] / st[:, 0]).cpu().numpy()
    return {"block_rms_first8": [round(float(x), 2) for x in rms[:8]],
            "block_rms_quantiles_rest": [round(float(x), 2) for x in np.quantile(rms[8:], [0, 0.5, 1])] if nb > 8 else [],
            "row_max_over_rms": float(torch.median(G.abs().amax(1) / G.pow(2).mean(1).sqrt()).item()),
            "f6_residual_rel_median": float(np.median(rel)), "f6_residual_rel_max": float(rel.max()), "rows": n}


def project_split(P, X, shift64, out, hook, device):
    """The batch's exact projection into out; with a hook (StepPipeline merge_at "tail"): its full rounds of
    tiles, the hook (which launches the previous batch's merge behind them), then the last, partial round."""
    nt = P.tile_count(X.shape[0]) if hook is not None else 0
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    if nt > ncu:
        split = (nt - 1) // ncu * ncu
        P.project(X, shift64=shift64, out=out, tiles=(0, split))
        hook()
        P.project(X, shift64=shift64, out=out, tiles=(split, nt))
    else:
        P.project(X, shift64=shift64, out=out)
        if hook is not None:
            hook()


def stress_run(P, bank, args, noise, device, N=None):
    """Crowded neighbours: the headline shape (1M gallery, B = 4096, d = 9999) with the pixel noise
    raised so that identities crowd together and the fp6 certificate fails; the uncertified queries
    then run down the int8 / fp32 tiers inside the timed step.  One GPU.  With N (and the
    headline noise) the same full step on another gallery size: configs[1] = 100k rows."""
    N = N or args.gallery
    B, d, k = args.batch, args.dim, args.k
    ld = max(32, round_up(d, 32))
    n_ids = (N + args.per_id - 1) // args.per_id
    gallery = build_gallery(P, bank, args.per_id, 0, N, N, d, ld, device, noise=noise)
    for t in gallery.tier_path("f6")[:-1]:
        gallery._tier_gallery(t)
    gq = torch.Generator(device=device)
    gq.manual_seed(SEED + 7)
    ids_q = torch.randint(0, n_ids, (B,), generator=gq, device=device)
    Xq = bank.images(ids_q, seed=SEED + 99, noise=noise)
    tiers = []
    # the headline's step pipeline (main()), exactly K preparations and K searches in the timed region
    bufs = [dict(Qd=torch.zeros((B, ld), dtype=torch.float32, device=device), qq=None,
                 out=(torch.empty((B, k), dtype=torch.float64, device=device),
                      torch.empty((B, k), dtype=torch.int64, device=device)))
            for _ in range(StepPipeline.NBUF)]
    timed = []

    starts = []

    def prep(j, hook=None):
        project_split(P, Xq, gallery.shift64, bufs[j]["Qd"], hook, device)
        tier = gallery.start_tier(B)          # adaptive start (FloatGallery.start_tier): f6 unless it keeps failing
        if timed:
            starts.append(str(tier))
        bufs[j]["qq"] = gallery.quantize_queries(bufs[j]["Qd"], bufs[j]["qq"], tier=tier)

    def finish(j):
        b = bufs[j]
        gallery.fallback(b["Qd"], b["qq"], k, b["out"], timings=tiers if timed else None)
        return b["out"]

    pipe = StepPipeline(device, prep,
                        lambda j, w, part: gallery.search_q8_phase(4 if part == "sample" else 8, bufs[j]["Qd"],
                                                                   bufs[j]["qq"], k, workspace=w),
                        lambda j, w: gallery.search_q8_phase(2, bufs[j]["Qd"], bufs[j]["qq"], k, out=bufs[j]["out"],
                                                             workspace=w),
                        finish)
    pipe.run(StepPipeline.NBUF)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = args.stress_steps
    timed.append(True)
    out = pipe.run(K)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / K
    last = (K - 1) % StepPipeline.NBUF
    Qd, qq = bufs[last]["Qd"], bufs[last]["qq"]
    counts = list(gallery.last_fallbacks)
    per_tier = {}
    for t, n, m in tiers:
        e = per_tier.setdefault(t, {"queries": n, "ms": 0.0})
        e["ms"] += m / args.stress_steps
    acc = float(((out[1][:, 0] // args.per_id) == ids_q).double().mean().item())
    res = {"pixel_noise": noise, "queries_per_s": B / (ms * 1e-3), "ms_per_step": ms,
           "start_tiers": {t: starts.count(t) for t in sorted(set(starts))},
           "uncertified_after_each_tier": counts, "skipped_tier": dict(gallery.last_skipped),
           "fallback_ms_per_step": per_tier,
           "certificate_margin_fp6": certificate_margin(gallery, Qd, qq), "top1_identity_acc": acc}
    del gallery
    torch.cuda.empty_cache()
    return res


def launch_ranks(n, cmd=None, poll_s=0.2):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT) and wait for them.  Runs before anything
    touches the GPU; the children are new processes (no exec of this one).  Every child is polled: the
    first non-zero exit, from whichever rank, terminates the others (they would wait in a collective
    forever) and is returned; 0 once all exited cleanly.  Rank 0 prints the JSON line.  cmd: the child
    command line (tests), default this script with the same arguments."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))
    status = 0
    while True:
        live = 0
        for p in procs:
            rc = p.poll()
            if rc is None:
                live += 1
            elif rc and not status:
                status = rc
                for q in procs:
                    if q.poll() is None:
                        q.terminate()
        if not live:
            return status
        time.sleep(poll_s)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU, e.g. "
              f"torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus})", file=sys.stderr)
        sys.exit(2)
    local = 0 if os.environ.get("OFR_ONE_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("OFR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    _lib.device()

    H = W = args.side
    D, d, k, B = H * W, args.dim, args.k, args.batch
    N = args.gallery
    n_ids = (N + args.per_id - 1) // args.per_id
    n0, n1 = shard_range(N, rank, world)
    nl = n1 - n0

    # ---- setup (untimed): W, gallery shard, queries -------------------------------------
    t0 = time.perf_counter()
    # the trained W's training set (configs[1]: identities 0 .. train_ids - 1) may reach past a small gallery's
    bank = IdentityBank(max(n_ids, args.train_ids if args.w == "trained" else 0), H, W, device=device)
    w_info = {"kind": "random N(0, 1/D)"}
    c4 = api = None
    if args.w == "trained" and world == 1 and args.config4:
        # configs[4]: the reference API trains the W (timed); then configs[1] through the API on its model
        model1, c4 = train_config4(bank, args.per_id, args.train_ids * args.per_id, H, W, device)
        log(rank, f"configs[4]: {c4['wall_s']:.2f} s ({c4['device_eigensolve_s']})")
        P = model1.feature._proj()
        Wt = None
        w_info = {"kind": "Fisherfaces() trained on configs[1]'s faces through PredictableModel.compute",
                  "regime": c4["regime"], "n_train": args.train_ids * args.per_id, "identities": args.train_ids,
                  "d": c4["d"], "eigenvalues_head": c4["eigenvalues_head"], "train_s": c4["wall_s"]}
        if args.api:
            api = api_predict(model1, bank, args.train_ids, B, H, W, device)
            log(rank, f"api: {api['queries_per_s']:.0f} q/s {api['parts_ms']}")
        model1.classifier.__dict__.pop("_dev", None)             # the 100k gallery; P (the W) stays
        del model1
        torch.cuda.empty_cache()
    elif args.w == "trained":
        P, Wt, w_info = build_trained_projection(bank, args.per_id, args.train_ids * args.per_id, D, device)
        w_info["kind"] = "Fisherfaces() trained on configs[1]'s faces"
    else:
        P, Wt = build_projection(D, d, device)
    if P.d != d:
        raise SystemExit(f"W has d={P.d}, --dim {d}: pass --dim {P.d}")
    log(rank, f"W: {w_info}")
    ld = max(32, round_up(d, 32))
    gallery = build_gallery(P, bank, args.per_id, n0, nl, N, d, ld, device)
    gq = torch.Generator(device=device)
    gq.manual_seed(SEED + 7)
    # one distinct query batch per pipeline buffer (identities and pixel noise differ): consecutive timed steps
    # never replay the same faces (round 6; before, every step searched one fixed batch)
    ids_qs, Xqs = [], []
    for jb in range(StepPipeline.NBUF):
        ids_qs.append(torch.randint(0, n_ids, (B,), generator=gq, device=device))
        Xqs.append(bank.images(ids_qs[-1], seed=SEED + 99 + jb))
    ids_q, Xq = ids_qs[0], Xqs[0]
    Qd = torch.zeros((B, ld), dtype=torch.float32, device=device)
    out = (torch.empty((B, k), dtype=torch.float64, device=device), torch.empty((B, k), dtype=torch.int64, device=device))
    torch.cuda.synchronize()
    log(rank, f"setup {time.perf_counter() - t0:.1f}s: gallery rows {nl}/{N} per rank, d={d}, D={D}, B={B}")

    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(7)] for _ in range(args.steps)]
    use_q8 = args.search in ("f6", "q8")
    tier0 = "f6" if args.search == "f6" else 1
    if use_q8:
        if world > 1:
            share_block_scales(gallery)     # every rank quantizes alike: the fp6 query panels are all-gathered
        for t in FloatGallery.tier_path(tier0)[:-1]:
            gallery._tier_gallery(t)                              # quantized gallery tiers (once, untimed)
    fallbacks = []
    last_counts = []
    # sharded query preparation: rank r projects / quantizes faces [b0, b1) and the rows are
    # all-gathered (fp6 panels need whole 256-row blocks per rank)
    b0, b1 = shard_range(B, rank, world)
    shard_prep = world > 1 and B % world == 0 and (tier0 != "f6" or (B // world) % 256 == 0)
    starts = []              # the first tier of every batch (FloatGallery.start_tier; sharded too: every rank
                             # keeps the same global failure statistics, certify_sharded)
    # the step pipeline (StepPipeline): three query buffers, each with its own result lists
    bufs = [dict(Qd=Qd if j == 0 else torch.zeros_like(Qd), qq=None, pending=None, qq_loc=None,
                 out=out if j == 0 else tuple(torch.empty_like(t) for t in out),
                 Qd_loc=torch.zeros((b1 - b0, ld), dtype=torch.float32, device=device) if shard_prep else None)
            for j in range(StepPipeline.NBUF)]

    def prep(j, hook=None):
        """Query batch -> centred fp32 search rows (+ the first tier's quantized rows) in buffer j.  hook
        (StepPipeline merge_at "tail"): called between the projection's full rounds and its last round."""
        b = bufs[j]
        if shard_prep:
            P.project(Xqs[j][b0:b1], shift64=gallery.shift64, out=b["Qd_loc"])   # this rank's faces
            if hook is not None:
                hook()
            if use_q8:
                tier = gallery.start_tier(B) if tier0 == "f6" else tier0
                starts.append(str(tier))
                b["qq_loc"] = gallery.quantize_queries(b["Qd_loc"], b["qq_loc"], tier=tier)
                b["qq"] = gallery.gather_queries(b["qq_loc"])
                # the fp32 rows are read from phase 2 on: their all-gather overlaps the tile pass
                b["pending"] = gather_rows_async(b["Qd_loc"])
                b["Qd"] = b["pending"].out
            else:
                b["Qd"] = gather_rows(b["Qd_loc"])                        # RCCL all-gather
        else:
            project_split(P, Xqs[j], gallery.shift64, b["Qd"], hook, device)   # fp32(W^T x - c), exact int8 MFMA
            if use_q8:       # the adaptive start tier (FloatGallery.start_tier; f6 here)
                tier = gallery.start_tier(B) if tier0 == "f6" else tier0
                starts.append(str(tier))
                b["qq"] = gallery.quantize_queries(b["Qd"], b["qq"], tier=tier)
                b["tier"] = tier

    def tiles(j, w, part):
        b = bufs[j]
        if use_q8:
            gallery.search_q8_phase(4 if part == "sample" else 8, b["Qd"], b["qq"], k, workspace=w)
        elif part == "sample":
            gallery.search_phase("tiles", b["Qd"], k, workspace=w)

    def merge(j, w):
        b = bufs[j]
        if b["pending"] is not None:
            b["Qd"] = b["pending"]()
            b["pending"] = None
        if use_q8:
            merge_sharded(gallery, b["Qd"], b["qq"], k, n0, b["out"], workspace=w)   # world 1: the plain phase 2
        else:
            gallery.search_phase("merge", b["Qd"], k, index_base=n0, out=b["out"], workspace=w)

    def finish(j):
        b = bufs[j]
        if use_q8:
            if world > 1:      # global certificate: all-gather + merge + collective fallback
                res, counts = certify_sharded(gallery, b["Qd"], b["qq"], k, b["out"], n0)
                fallbacks.append(counts[0])
                last_counts[:] = counts
                return res
            fallbacks.append(gallery.fallback(b["Qd"], b["qq"], k, b["out"], index_base=n0))
            last_counts[:] = list(gallery.last_fallbacks)
            return b["out"]
        if world > 1:
            gd, gi = exchange_topk(*b["out"])
            return merge_topk(gd, gi, world, k, k)
        return b["out"]

    # OFR_BENCH_OVERLAP=0: everything on the main stream, in the same order
    # N > 1: "after" -- the merge's collectives (the pruned split merge's bound exchange) and the preparation's
    # all-gathers stay strictly ordered on one communicator; "tail" would let them run on two streams at once
    pipe = StepPipeline(device, prep, tiles, merge, finish, overlap=os.environ.get("OFR_BENCH_OVERLAP", "1") == "1",
                        merge_at=None if world == 1 else os.environ.get("OFR_BENCH_MERGE", "after"))
    pipe.run(max(args.warmup, StepPipeline.NBUF))     # untimed; every buffer and workspace allocated
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    res = pipe.run(args.steps, ev)                     # exactly K preparations and K searches
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    last = (args.steps - 1) % StepPipeline.NBUF
    Qd, qq = bufs[last]["Qd"], bufs[last]["qq"]

    ms_proj = np.mean([e[0].elapsed_time(e[1]) for e in ev])
    ms_tiles = np.mean([e[4].elapsed_time(e[2]) for e in ev])     # the tile pass on the main stream
    ms_sample = np.mean([e[4].elapsed_time(e[6]) for e in ev])    # its sample pass + thresholds
    ms_sieve = np.mean([e[6].elapsed_time(e[2]) for e in ev])     # its sieve pass (fp6; else the rest)
    ms_merge = np.mean([e[5].elapsed_time(e[3]) for e in ev])     # merge + certificate on the side stream
    # the preparation alone (the last batch's projection + quantization again, same outputs): with merge_at
    # "tail" the step's preparation events also span the merge run beside the projection's last round
    ms_proj_alone = None
    if not shard_prep and world == 1:
        xs, tq = Xqs[last], bufs[last].get("tier", tier0)
        ms_pa = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            P.project(xs, shift64=gallery.shift64, out=Qd)
            if use_q8:
                qq = gallery.quantize_queries(Qd, qq, tier=tq)
            e1.record()
            torch.cuda.synchronize()
            ms_pa.append(e0.elapsed_time(e1))
        ms_proj_alone = float(np.median(ms_pa))
    ms_prep_roof = ms_proj_alone if ms_proj_alone is not None else ms_proj
    idx = res[1][:, 0]
    acc = float(((idx // args.per_id) == ids_qs[last]).double().mean().item())   # the last batch's identities
    kept = (gallery.sieve_counts(B, pipe.ws[(args.steps - 1) % StepPipeline.NWS]) if args.search == "f6"
            else None)                                                  # last step's fp6 sieve (this rank)
    kept = None if kept is None else {"mean": float(kept.double().mean()), "max": int(kept.max()),
                                      "cap": 32768,
                                      "expected": ("~4 x 64 (row sample)" if FloatGallery.row_sample()
                                                   else "~16 x OFR_SIEVE_STRIDE (64) (panel sample)")}

    # ---- small-batch regime (the recognizers send one face per call): HBM-bound streaming of the gallery ----
    small = []
    for bs in [int(x) for x in args.small_batches.split(",") if x.strip()]:
        # HBM regime (the recognizers send one face per call): the fp6 streaming pass for B <= 32
        Qs = torch.zeros((bs, ld), dtype=torch.float32, device=device)
        P.project(Xq[:bs], shift64=gallery.shift64, out=Qs)
        f6_small = args.search == "f6" and gallery.use_q8(bs, k)
        stier = gallery.start_tier(bs) if f6_small else None      # f6p when the gallery has a prefix
        qs = gallery.quantize_queries(Qs, tier=stier) if f6_small else None

        def small_pass():
            if f6_small:
                gallery.search_q8_phase(1, Qs, qs, k)
            else:
                gallery.search_phase("tiles", Qs, k)

        for _ in range(2):
            small_pass()
        reps = 10
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            small_pass()
        e1.record()
        torch.cuda.synchronize()
        ms_t = e0.elapsed_time(e1) / reps
        t1 = time.perf_counter()
        for _ in range(reps):                 # the whole small-batch step: project, search, merge, certificate
            P.project(Xq[:bs], shift64=gallery.shift64, out=Qs)
            if f6_small:
                qs = gallery.quantize_queries(Qs, qs, tier=stier)
                o = gallery.search_q8_phase(3, Qs, qs, k, index_base=n0)
                gallery.fallback(Qs, qs, k, o, index_base=n0)
            else:
                gallery.search_phase("tiles", Qs, k)
                gallery.search_phase("merge", Qs, k, index_base=n0)
        torch.cuda.synchronize()
        ms_step = (time.perf_counter() - t1) * 1e3 / reps
        if f6_small:
            dm_s = min(d, 128 * gallery.prefix_stages()) if stier == "f6p" else d   # features the pass streams
            kern = ("q8s::stream_kernel_f6 (ofr_knn_f6" + ("p_sampled, first %d features" % dm_s if stier == "f6p" else "")
                    + " phase 1, B<=32)")
            bytes_t = 0.75 * (nl * dm_s + bs * dm_s)                 # fp6 tiles streamed once per batch
        else:
            kern = "knn_tile_kernel<Cfg<32,4,1,4>> (ofr_knn_tiles_f32, B<=32)"
            bytes_t = nl * d * 4 + bs * d * 4                        # fp32 rows streamed once per batch
        small.append({"batch": bs, "queries_per_s": bs / (ms_step * 1e-3), "ms_per_batch": ms_step, "tier": stier,
                      "uncertified": (list(gallery.last_fallbacks) if f6_small else None),
                      "roofline": {"kernel": kern, "bound": "hbm", "achieved": bytes_t / (ms_t * 1e-3) / 1e9,
                                   "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                                   "frac": bytes_t / (ms_t * 1e-3) / PEAK_HBM, "launch_ms": ms_t,
                                   "algorithmic_bytes_per_launch": bytes_t}})

    # the merge alone (phase 2 of the last batch again on its workspace: idempotent), and its bytes: the fp32
    # rows of the candidates it re-ranked exactly (MergeArgs::evals), the query rows, the kept bucket entries
    merge_roof = None
    if args.search == "f6" and world == 1:
        wl = pipe.ws[(args.steps - 1) % StepPipeline.NWS]
        ms_m = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gallery.search_q8_phase(2, Qd, qq, k, workspace=wl)
            e1.record()
            torch.cuda.synchronize()
            ms_m.append(e0.elapsed_time(e1))
        ev_ = gallery.merge_evals(B, wl)
        kc = gallery.sieve_counts(B, wl)
        if ev_ is not None:
            n_ev = float(ev_.double().sum())
            mb = n_ev * d * 4 + B * d * 4 + (float(kc.double().clamp(0, 32768).sum()) * 8 if kc is not None else 0.0)
            mm = float(np.median(ms_m))
            merge_roof = {"kernel": "q8s::merge_kernel<true, true, false> (bucket best-16, exact fp64 re-rank of the "
                                    "candidates by the whole block, one HBM round trip each, certificate) + "
                                    "merge_kernel<true, true, true> (the deep continuation of open queries)", "bound": "hbm", "ms_alone": mm,
                          "exact_reranks_per_query": n_ev / B, "algorithmic_bytes": mb,
                          "achieved": mb / (mm * 1e-3) / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                          "frac": mb / (mm * 1e-3) / PEAK_HBM}
    margin = certificate_margin(gallery, Qd, qq) if args.search == "f6" and world == 1 else None
    flops_tiles = 2.0 * B * nl * d                                    # algorithmic, per launch
    achieved = flops_tiles / (ms_tiles * 1e-3)
    # the tier the timed steps started at (FloatGallery.start_tier): f6p (the prefix tier) when the
    # gallery's features put their variance in the leading columns, f6 otherwise
    tier_used = max(set(starts[-args.steps:]), key=starts[-args.steps:].count) if starts else None
    pst = gallery.prefix_stages() if tier_used == "f6p" else 0
    if args.search == "f6":
        # the dominant kernel is the sieve pass: it scores every (query, row) pair -- over all d features
        # (tier f6: 2 B N d) or over the first m = 128 pst of them (tier f6p: 2 B N m; the rest of each
        # distance is never needed to certify) -- (the sample pass before it re-does 1/64 of it to set the
        # thresholds); its launch is timed by its own events on the main stream, phase 1 (sample +
        # thresholds + sieve) is reported beside it
        lib = _lib.load()                                                     # the variant the library launches
        sieve = (lib.ofr_f6p_sieve_kernel(pst) if pst else lib.ofr_f6_sieve_kernel()).decode()
        dm = min(d, 128 * pst) if pst else d                                 # the features the pass scores
        flops_tiles = 2.0 * B * nl * dm
        peak, kname = PEAK_F6_MFMA, ("ofr_knn_f6p_sampled prefix sieve pass (fp6 e2m3, first %d of %d features): "
                                     % (dm, d) if pst else "ofr_knn_f6 sieve pass (fp6 e2m3): ") + sieve
        achieved = flops_tiles / (ms_sieve * 1e-3)
        alg_bytes_tiles = 0.75 * (nl * dm + B * dm)                  # 6 bits per feature, gallery + queries
        ntg_, ntq_, nst_ = -(-nl // 256), -(-B // 256), -(-dm // 128)
        wide = "f6w" in sieve or "f6p" in sieve                      # 384 x 256 tiles: 60 KiB per stage
        fed = (-(-nl // 384) * 61440.0 if wide else ntg_ * 49152.0) * ntq_ * nst_   # copied into LDS per sieve pass
        if "prefix_pass_kernel" in sieve:   # per 256-row tile: its 24 KiB image per item, 12 KiB per 128-query step
            fed = ntg_ * -(-B // 128) * 12288.0 + ntg_ * 24576.0 * max(1.0, -(-B // 128) / 16.0)
        elif "f6p" in sieve:     # the persistent pass copies a gallery tile once per item of query panels
            fed = -(-nl // 384) * ntq_ * nst_ * 24576.0 + -(-nl // 384) * nst_ * 36864.0 * (ntq_ / 16.0)
        executed = flops_tiles
    elif use_q8:
        peak, kname = PEAK_I8_MFMA, "q8s::tile_kernel<1> (ofr_knn_q8 phase 1, one int8 slice)"
        alg_bytes_tiles = nl * d + B * d                             # one int8 slice of gallery + queries
        executed = flops_tiles                                       # x1.y1
    else:
        peak, kname = PEAK_FP32_MFMA, "knn_tile_kernel (ofr_knn_tiles_f32)"
        alg_bytes_tiles = nl * d * 4 + B * d * 4                     # gallery + queries read once
        executed = flops_tiles

    if rank == 0:
        value = B * args.steps / elapsed
        coll = "RCCL" if world > 1 and dist.get_backend() == "nccl" else "gloo"   # the collectives' backend
        tr = committed_traffic({"gallery": nl, "batch": B, "d": d, "D": D, "k": k, "search": args.search,
                                "w": args.w, "tier": tier_used or args.search, "engine": sieve_engine(kname)})
        result = {
            "metric": "query faces/sec (Fisherfaces proj + 1-NN, 1M gallery) at 1/2/4/8 GPUs",
            "value": value, "unit": "queries/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None,
            "dtype": {"f6": "fp6 e2m3 (fp6 MFMA coarse scores, certified; fp64 exact re-rank)" + (
                      f" -- prefix tier f6p: coarse scores of the first {128 * pst} features, certified by the "
                      f"projection bound" if pst else ""),
                      "q8": "i8 (int8 MFMA coarse scores, certified; fp64 exact re-rank)",
                      "fp32": "f32 (fp32 MFMA scores, fp64 exact re-rank)"}[args.search], "data": "synthetic", "query_batches_cycled": StepPipeline.NBUF,
            "config": {"workload": "configs[2]: Fisherfaces projection + 1-NN, 1M-image gallery (100k ids x 10), "
                                   "100x100 faces, d=9999, B=4096 queries/step, Euclidean, k=1, W = "
                                   + ("Fisherfaces() trained on configs[1]'s 100k faces (10k ids x 10)"
                                      if args.w == "trained" else "random N(0, 1/D)"),
                       "gallery": N, "global_batch": B, "d": d, "D": D, "k": k,
                       "parallelism": (f"gallery-rows/{world}, query prep sharded + {coll} all-gather of rows, {coll} all-gather "
                                       f"of top-k + bounds (global certificate)" if shard_prep else
                                       f"gallery-rows/{world} + {coll} all-gather of top-k")
                       if world > 1 else "1 GPU"},
            "roofline": {"kernel": kname, "bound": "mfma",
                         "achieved": achieved / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s" if not use_q8 else "TOPS",
                         "frac": achieved / peak, "traffic": tr[0] if tr else None,
                         "executed_ops_per_launch": executed,
                         "executed_frac": executed / ((ms_sieve if args.search == "f6" else ms_tiles) * 1e-3) / peak,
                         "traffic_source": tr[1] if tr else None,
                         "algorithmic_flops_per_launch": flops_tiles, "algorithmic_bytes_per_launch": alg_bytes_tiles,
                         "launch_ms": ms_sieve if args.search == "f6" else ms_tiles,
                         **({"phase1": {"what": "sample pass + thresholds + sieve pass (events on the main stream)",
                                        "ms": ms_tiles, "sample_ms": ms_sample,
                                        "frac": flops_tiles / (ms_tiles * 1e-3) / peak},
                             "sustained_peak": SUSTAINED_F6_MFMA / 1e12, "frac_of_sustained": achieved / SUSTAINED_F6_MFMA,
                             "sustained_source": "tools/f6_shape_probe.hip (profiles/r02_f6_shape_probe.log)",
                             "feed": {"what": "bytes copied into the CUs' LDS by the sieve pass (60 KiB per 384x256x128 "
                                              "stage; 48 KiB per 256x256x128 stage on the 8-wave engine)",
                                      "bytes_per_launch": fed,
                                      "achieved_TBps": fed / (ms_sieve * 1e-3) / 1e12}}
                            if args.search == "f6" else {})},
            # the pruned pass against the brute-force work SURVEY §8d prices (2 B N d per step): the rate the step
            # would imply if every feature of every pair were scored -- the pruning factor made visible (the
            # prefix tier scores m = 128 pst of the d features; the rest of a distance is never needed)
            "brute_force_equivalent": {
                "ops_per_step": 2.0 * B * nl * d, "scored_ops_per_step": flops_tiles if args.search == "f6" else None,
                "scored_fraction": (flops_tiles / (2.0 * B * nl * d)) if args.search == "f6" else None,
                "implied_POPS": 2.0 * B * nl * d / (elapsed / args.steps) / 1e15,
                "note": "not comparable with any peak: the pruned features are bounded, not computed"},
            "roofline_merge": merge_roof,
            "kernels_ms": {"project_u8_exact" + ("+quantize" if use_q8 else "") + ("+all_gather" if shard_prep else ""):
                           ms_proj, "knn_tiles": ms_tiles,
                           "knn_merge_rerank" + ("+certificate" if use_q8 else ""): ms_merge,
                           "preparation_alone": ms_proj_alone},
            # the preparation beside the dominant kernel (round 5: the two take about the same time): the
            # exact projection W^T x of the batch's faces on the int8 MFMA, four W slices --
            # 2 D d int8 ops per face and slice, timed with the quantization by the preparation's events
            "roofline_preparation": {
                "kernel": "q8::project_q8w_kernel (ofr_project_u8_exact, 4 int8 slices of W) + quantization",
                "bound": "mfma", "unit": "TOPS", "peak": PEAK_I8_MFMA / 1e12,
                "algorithmic_ops_per_step": 2.0 * 4 * (b1 - b0 if shard_prep else B) * D * d,
                "achieved": 2.0 * 4 * (b1 - b0 if shard_prep else B) * D * d / (ms_prep_roof * 1e-3) / 1e12,
                "frac": 2.0 * 4 * (b1 - b0 if shard_prep else B) * D * d / (ms_prep_roof * 1e-3) / PEAK_I8_MFMA,
                "ms": ms_prep_roof, "ms_source": "alone" if ms_proj_alone is not None else "step events"},
            # which of the two is longer per step: since the one-stage prefix pass, the preparation's
            # projection (roofline_preparation); `roofline` stays the search pass's (the path's own kernel)
            "dominant_by_time": {"kernel": ("q8::project_q8w_kernel (roofline_preparation)"
                                            if ms_prep_roof > (ms_sieve if args.search == "f6" else ms_tiles)
                                            else "the search pass (roofline)"),
                                 "preparation_ms": ms_prep_roof,
                                 "search_pass_ms": ms_sieve if args.search == "f6" else ms_tiles},
            "uncertified_queries_per_step": (float(np.mean(fallbacks[-args.steps:])) if use_q8 else None),
            "start_tiers": ({t: starts[-args.steps:].count(t) for t in sorted(set(starts[-args.steps:]))}
                            if starts else None),
            "uncertified_after_each_tier": (list(last_counts) if use_q8 else None),
            "sieve_kept_rows_per_query": kept,
            "top1_identity_acc": acc,
            "certificate_margin_fp6": margin,
            "projection_w": w_info,
            "config4": c4,
            "api": api,
            "feature_profile": feature_profile(gallery) if args.search == "f6" else None,
            "small_batch": small,
        }
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(P, gallery, Xq, N, args.cpu_seconds)
            result["speedup_vs_cpu"] = value / result["cpu_baseline"]["value"]
        if world == 1 and args.search == "f6" and (args.stress.strip() or args.config1):
            gallery.q8, gallery.G, gallery._Gbuf = None, None, None      # free the headline gallery first
            torch.cuda.empty_cache()
        if world == 1 and args.search == "f6" and args.config1:
            c1 = stress_run(P, bank, args, 12.0, device, N=100_000)
            c1.pop("pixel_noise")
            result["config1"] = dict(workload="configs[1]: 10k identities x 10 = 100k-row gallery, B=4096, d=9999, "
                                              "the same full step (projection + fp6 tier + merge + fallback)", **c1)
            log(rank, f"configs[1]: {c1['queries_per_s']:.0f} q/s, uncertified {c1['uncertified_after_each_tier']}")
        if world == 1 and args.search == "f6" and args.stress.strip():
            result["stress"] = [stress_run(P, bank, args, float(x), device) for x in args.stress.split(",") if x.strip()]
            for r in result["stress"]:
                log(rank, f"stress noise {r['pixel_noise']}: {r['queries_per_s']:.0f} q/s, uncertified "
                          f"{r['uncertified_after_each_tier']}, margin {r['certificate_margin_fp6']}")
        if world == 1 and args.config3:
            del gallery
            torch.cuda.empty_cache()
            result["config3"] = config3_run(device)
            log(rank, f"configs[3]: {result['config3']['queries_per_s']:.0f} q/s")
        if result.get("config1") and api:
            api["vs_engine_config1"] = api["queries_per_s"] / result["config1"]["queries_per_s"]
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
