"""Diagnostic for the round-3 intermittent singular-Sw failure (test_trainer_train_roundtrip).

Runs the Gram-regime Fisherfaces chain (training.centred_gram -> eigh_desc -> feature_scatter) on
the trainer test's faces (the bundled grey JPEG planes resized to 70x70 on the device) in several
process states and reports, per state, whether every stage is bit-identical to the first state's,
the smallest LU pivot of Sw, and whether numpy's inv(Sw) (feature.py:170) succeeds on copies of Sw
at eight buffer alignments.  States: fresh, repeated, after NaN-poisoning the caching allocator,
after large rocSOLVER solves on a side stream, after stream churn.  One JSON line per state."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def poison(total=2 << 30):
    keep = []
    for s in (4096, 65536, 200_000, 1 << 20, 3 << 20, 24 << 20, 160 << 20):
        for _ in range(max(1, min(64, (total // 7) // s))):
            t = torch.empty(s // 8, dtype=torch.float64, device="cuda")
            t.fill_(float("nan"))
            keep.append(t)
    torch.cuda.synchronize()
    del keep


def big_solves():
    from opencv_facerecognizer_amd import _device
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        r = torch.Generator(device="cpu").manual_seed(3)
        A = torch.randn(2048, 2048, generator=r, dtype=torch.float64).cuda()
        A = A @ A.t() + 2048 * torch.eye(2048, dtype=torch.float64, device="cuda")
        B = torch.randn(2048, 2048, generator=r, dtype=torch.float64).cuda()
        B = B @ B.t()
        _device.eigh_desc_f64(A, 100)
        _device.sygv_desc_f64(B, A, 100)
    torch.cuda.synchronize()
    del s


def stream_churn():
    for _ in range(8):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.ones(1 << 20, device="cuda").sum()
        torch.cuda.synchronize()
        del s


def run_chain(imgs, y, perm=None):
    from opencv_facerecognizer_amd import ingest, training
    if perm is not None:
        imgs, y = [imgs[i] for i in perm], y[perm]
    X = ingest.faces(imgs, (70, 70), ingest.INTER_LINEAR)
    Xh = X.cpu().numpy().reshape(len(imgs), -1)
    Xd = torch.from_numpy(Xh).cuda()
    lay = training.Layout(y, Xd.device)
    n, c, D = lay.n, lay.c, Xh.shape[1]
    k = min(n - c, D, n)
    G = training.centred_gram(Xd, D, lay)
    Gh = G.cpu().numpy().copy()
    lam, V = training.eigh_desc(G, k)
    sig = lam.clamp_min(0.0).sqrt()
    Sw, Sb = training.feature_scatter((V * sig).contiguous(), y)
    torch.cuda.synchronize()
    return dict(X=Xh, G=Gh, lam=lam.cpu().numpy(), V=V.cpu().numpy(), Sw=Sw.cpu().numpy(), Sb=Sb.cpu().numpy())


def inv_trials(Sw):
    out = []
    for a in range(8):
        buf = np.empty(Sw.size + 8, np.float64)
        M = buf[a:a + Sw.size].reshape(Sw.shape)
        M[...] = Sw
        try:
            np.linalg.inv(M)
            out.append(True)
        except np.linalg.LinAlgError:
            out.append(False)
    return out


def main():
    import scipy.linalg
    z = np.load(os.path.join(GOLDEN, "individuals_gray.npz"))
    off = np.concatenate([[0], np.cumsum(z["shapes"].prod(1))])
    imgs = [z["pixels"][off[i]:off[i + 1]].reshape(tuple(s)) for i, s in enumerate(z["shapes"])]
    y = np.asarray(z["labels"])
    first = None
    for name, prep in (("fresh", None), ("repeat", None), ("poisoned", poison), ("after_big_solves", big_solves),
                       ("stream_churn", stream_churn), ("poisoned_again", poison)):
        if prep:
            prep()
        cur = run_chain(imgs, y)
        if first is None:
            first = cur
        lu, _ = scipy.linalg.lu_factor(cur["Sw"])
        ev = np.linalg.eigvalsh(cur["Sw"])
        rec = {"state": name,
               "same_as_fresh": {k: bool(np.array_equal(v, first[k])) for k, v in cur.items()},
               "finite": {k: bool(np.isfinite(v.astype(np.float64)).all()) for k, v in cur.items()},
               "Sw_min_abs_pivot": float(np.abs(np.diag(lu)).min()), "Sw_eig_min_max": [float(ev[0]), float(ev[-1])],
               "inv_ok_by_alignment": inv_trials(cur["Sw"])}
        print(json.dumps(rec), flush=True)
    # row orders (TheTrainer.read_images follows os.walk / os.listdir, which differ between file
    # systems): does the reference's inv(Sw) meet an exactly zero pivot for some order?
    r = np.random.default_rng(0)
    fails = []
    for t in range(32):
        perm = r.permutation(len(y))
        Sw = run_chain(imgs, y, perm)["Sw"]
        try:
            np.linalg.inv(Sw)
        except np.linalg.LinAlgError:
            fails.append(t)
    print(json.dumps({"row_orders": 32, "inv_raised_for_orders": fails}), flush=True)


if __name__ == "__main__":
    main()
