"""Probe: symmetric / symmetric-definite eigensolvers at the training sizes of configs[4].

Times, for n x n fp64 matrices (n = 10000 by default):
  * rocSOLVER dsyevd / dsygvd on the device (bound here with ctypes, the library's own handle),
  * torch.linalg.eigh on the device (whatever backend torch picks),
  * host LAPACK (numpy eigh / scipy eigh(Sb, Sw)) -- the path training uses today,
and reports the residual ||A V - B V diag(lam)||_F / ||A||_F of each.

    python tools/bench_eigh.py [n] [--no-host]
"""
import ctypes
import json
import sys
import time

import numpy as np
import torch

RB_FILL_UPPER, RB_FILL_LOWER = 121, 122
RB_EVECT_ORIGINAL = 211
RB_EFORM_AX = 221


def rocsolver():
    blas = ctypes.CDLL("librocblas.so.5", mode=ctypes.RTLD_GLOBAL)
    sol = ctypes.CDLL("librocsolver.so.0", mode=ctypes.RTLD_GLOBAL)
    h = ctypes.c_void_p()
    assert blas.rocblas_create_handle(ctypes.byref(h)) == 0
    assert blas.rocblas_set_stream(h, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    return blas, sol, h


def p(t):
    return ctypes.c_void_p(t.data_ptr())


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10000
    host = "--no-host" not in sys.argv
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.randn((n + n // 5, n), dtype=torch.float64, device=dev, generator=g)
    Sw = X.T @ X / X.shape[0] + 1e-3 * torch.eye(n, dtype=torch.float64, device=dev)
    Y = torch.randn((n, n), dtype=torch.float64, device=dev, generator=g)
    Sb = Y.T @ Y / n
    del X, Y
    blas, sol, h = rocsolver()
    res = {"n": n}
    info = torch.zeros(1, dtype=torch.int32, device=dev)

    # dsyevd on Sb
    A = Sb.clone()
    D = torch.empty(n, dtype=torch.float64, device=dev)
    E = torch.empty(n, dtype=torch.float64, device=dev)
    sol.rocsolver_dsyevd(h, RB_EVECT_ORIGINAL, RB_FILL_LOWER, n, p(A), n, p(D), p(E), p(info))   # warm (workspace)
    A.copy_(Sb)
    t, _ = timed(lambda: sol.rocsolver_dsyevd(h, RB_EVECT_ORIGINAL, RB_FILL_LOWER, n, p(A), n, p(D), p(E), p(info)))
    V = A.T        # column-major result: eigenvectors are the columns of the column-major A = rows of A here
    r = torch.linalg.norm(Sb @ V - V * D) / torch.linalg.norm(Sb)
    res["rocsolver_dsyevd"] = {"s": t, "info": int(info.item()), "residual": float(r)}
    print(json.dumps(res), flush=True)

    # dsygvd on (Sb, Sw)
    A.copy_(Sb)
    B = Sw.clone()
    t, _ = timed(lambda: sol.rocsolver_dsygvd(h, RB_EFORM_AX, RB_EVECT_ORIGINAL, RB_FILL_LOWER, n, p(A), n, p(B), n,
                                              p(D), p(E), p(info)))
    V = A.T
    r = torch.linalg.norm(Sb @ V - (Sw @ V) * D) / torch.linalg.norm(Sb)
    res["rocsolver_dsygvd"] = {"s": t, "info": int(info.item()), "residual": float(r)}
    print(json.dumps(res), flush=True)
    del A, B

    try:
        t, (lam, V) = timed(lambda: torch.linalg.eigh(Sb))
        r = torch.linalg.norm(Sb @ V - V * lam) / torch.linalg.norm(Sb)
        res["torch_eigh"] = {"s": t, "residual": float(r), "backend": str(torch.backends.cuda.preferred_linalg_library())}
    except RuntimeError as e:
        res["torch_eigh"] = {"error": str(e)[:200]}
    print(json.dumps(res), flush=True)

    if host:
        import scipy.linalg
        Sbh, Swh = Sb.cpu().numpy(), Sw.cpu().numpy()
        t0 = time.perf_counter()
        lam, V = np.linalg.eigh(Sbh)
        res["host_eigh_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        lam, V = scipy.linalg.eigh(Sbh, Swh, driver="gvd")
        res["host_sygvd_s"] = time.perf_counter() - t0
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
