"""Diagnose the sharded (ofr_knn_sharded, one device) prefix tier against the single-process search on
test_gpu_parity's 'prefix' data, per prefix-pass engine (OFR_F6P_ENGINE)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    from opencv_facerecognizer_amd.parallel import DeviceComm
    from test_gpu_prefix import _lda_like
    torch.cuda.set_device(0)
    G, Q = _lda_like(1000, 10, 1280, 300, seed=11)
    G = G.astype(np.float32).astype(np.float64)
    Q = Q.astype(np.float32).astype(np.float64)
    D = ((Q[:, None, :] - G[None, :, :]) ** 2).sum(-1)
    ref = np.argsort(D, axis=1, kind="stable")[:, :3]
    for eng in ("3", "2", "1"):
        os.environ["OFR_F6P_ENGINE"] = eng
        g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
        d1, i1 = g.search(g.query_rows(Q), 3)
        single = (i1.cpu().numpy() == ref).all(1).mean()
        with DeviceComm([0]) as comm:
            (dd, ii, cert), = comm.knn([g], [g.query_rows(Q)], 3)
            counts, popen = comm.last_tier_counts, comm.last_prefix_open
        ok = (ii.cpu().numpy() == ref).all(1)
        print(f"engine {eng}: single ok {single:.3f} last_fallbacks {g.last_fallbacks}; sharded ok {ok.mean():.3f} "
              f"popen {popen} counts {counts} cert {cert.cpu().numpy().mean():.3f} bad {np.nonzero(~ok)[0][:10]}",
              flush=True)


if __name__ == "__main__" and not os.environ.get("DIAG_STAGED"):
    main()


def staged():
    """The sharded path's prefix stages from Python (one rank): phase 1, split merge stage 1, ub, stage 2."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    from test_gpu_prefix import _lda_like
    G, Q = _lda_like(1000, 10, 1280, 300, seed=11)
    G = G.astype(np.float32).astype(np.float64)
    Q = Q.astype(np.float32).astype(np.float64)
    D = ((Q[:, None, :] - G[None, :, :]) ** 2).sum(-1)
    ref = np.argsort(D, axis=1, kind="stable")[:, :3]
    for eng in ("3", "2"):
        os.environ["OFR_F6P_ENGINE"] = eng
        g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
        Qd = g.query_rows(Q)
        qq = g.quantize_queries(Qd, tier="f6p")
        from opencv_facerecognizer_amd._device import Workspace
        wsp = Workspace()
        nb = _lib.load().ofr_knn_f6_workspace_bytes(len(Q), g.N)
        wsp.get(nb, Qd.device).fill_(int(os.environ.get("DIAG_FILL", "255")))   # a fresh, dirty workspace
        g.search_q8_phase(1, Qd, qq, 3, workspace=wsp)
        ubl = torch.empty((len(Q), 3), dtype=torch.float64, device=Qd.device)
        g.merge_pruned(1, Qd, qq, 3, ubl, workspace=wsp)
        ub = ubl[:, 2].contiguous()
        out = (torch.empty((len(Q), 3), dtype=torch.float64, device=Qd.device),
               torch.empty((len(Q), 3), dtype=torch.int64, device=Qd.device))
        g.merge_pruned(2, Qd, qq, 3, ub, out=out, workspace=wsp)
        i2 = out[1].cpu().numpy()
        cert = qq["cert"].cpu().numpy()
        ok = (i2 == ref).all(1)
        qq2 = g.quantize_queries(Qd, tier="f6p")
        d0, i0 = g.search_q8_phase(3, Qd, qq2, 3)
        ok0 = (i0.cpu().numpy() == ref).all(1)
        print(f"staged engine {eng}: split cert {cert.mean():.3f} ok {ok.mean():.3f} wrong&cert "
              f"{np.nonzero(cert.astype(bool) & ~ok)[0][:8]}; plain cert {qq2['cert'].cpu().numpy().mean():.3f} "
              f"ok {ok0.mean():.3f}; ubl[0] {ubl[0].cpu().numpy()} bound[0] {qq['bound'][0].item():.4g} "
              f"exact[0] {np.sort(D[0])[:3]}", flush=True)


if __name__ == "__main__" and os.environ.get("DIAG_STAGED"):
    staged()


def fields():
    """The shard struct DeviceComm hands to ofr_knn_sharded, against the f6p tier's tensors."""
    import ctypes
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    from opencv_facerecognizer_amd.parallel import DeviceComm
    from test_gpu_prefix import _lda_like
    G, Q = _lda_like(1000, 10, 1280, 300, seed=11)
    g = FloatGallery(G.astype(np.float32).astype(np.float64), _lib.METRIC_EUCLIDEAN)
    orig = _lib.call

    def spy(name, *args):
        if name == "ofr_knn_sharded":
            sh = ctypes.cast(args[1], ctypes.POINTER(_lib.KnnShard))[0]
            tp = g._tier_gallery("f6p")
            for f, _ in _lib.KnnShard._fields_:
                print(f, getattr(sh, f), flush=True)
            print("tp Gs", tp["Gs"].data_ptr(), "scale", tp["scale"].data_ptr(), "gmax", tp["gmax"].data_ptr(),
                  "gmax vals", tp["gmax"].cpu().numpy(), "paux", tp["paux"].data_ptr(), flush=True)
        return orig(name, *args)
    _lib.call = spy
    import opencv_facerecognizer_amd.parallel as par
    par._lib = _lib
    with DeviceComm([0]) as comm:
        comm.knn([g], [g.query_rows(Q.astype(np.float32).astype(np.float64))], 3)
        print("popen", comm.last_prefix_open, comm.last_tier_counts)


if __name__ == "__main__" and os.environ.get("DIAG_FIELDS"):
    fields()
