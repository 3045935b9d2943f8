"""Diagnostic: repeat the Gram-regime Fisherfaces training of tests/test_gpu_ingest.py's
test_trainer_train_roundtrip (the bundled grey faces resized to 70x70 on the device) and report,
per repetition, whether the centred Gram, its eigenpairs and the scatter matrices are finite and
bit-identical to the first repetition's (the test failed once in four suite runs with a singular Sw).
One JSON line per repetition, then a summary line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def main(reps=int(os.environ.get("REPS", "24"))):
    from opencv_facerecognizer_amd import _device, ingest, training
    z = np.load(os.path.join(GOLDEN, "individuals_gray.npz"))
    off = np.concatenate([[0], np.cumsum(z["shapes"].prod(1))])
    imgs = [z["pixels"][off[i]:off[i + 1]].reshape(tuple(s)) for i, s in enumerate(z["shapes"])]
    y = np.asarray(z["labels"])
    first, bad = None, 0
    for r in range(reps):
        X = np.stack([np.asarray(f).reshape(-1) for f in ingest.faces(imgs, (70, 70), ingest.INTER_LINEAR, host=True)])
        X = X.astype(np.uint8)
        Xd = torch.from_numpy(X).cuda()
        lay = training.Layout(y, Xd.device)
        n, c, D = lay.n, lay.c, X.shape[1]
        k = min(n - c, D, n)
        G = training.centred_gram(Xd, D, lay)
        Gh = G.cpu().numpy().copy()
        lam, V = training.eigh_desc(G, k)
        sig = lam.clamp_min(0.0).sqrt()
        Sw, Sb = training.feature_scatter((V * sig).contiguous(), y)
        torch.cuda.synchronize()
        cur = dict(X=X, G=Gh, lam=lam.cpu().numpy(), V=V.cpu().numpy(), Sw=Sw.cpu().numpy(), Sb=Sb.cpu().numpy())
        if first is None:
            first = cur
        rec = {"rep": r}
        for key, v in cur.items():
            rec[key] = {"finite": bool(np.isfinite(v.astype(np.float64)).all()),
                        "same_as_first": bool(np.array_equal(v, first[key]))}
        ok = all(v["finite"] and v["same_as_first"] for v in rec.values() if isinstance(v, dict))
        bad += not ok
        print(json.dumps(rec), flush=True)
    print(json.dumps({"reps": reps, "reps_not_identical_or_not_finite": bad}), flush=True)


if __name__ == "__main__":
    main()
