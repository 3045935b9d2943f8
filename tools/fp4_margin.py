"""Analysis (not the product path): would an fp4 (e2m1) first tier certify the bench's queries?
Builds bench.py's gallery and queries, quantizes rows to e2m1 with a per-row scale (x~ = s v,
s = max|x|/6), and checks the certificate condition of the certified tiers with exact fp32 scores
standing in for the coarse ones:  S_1 < S_16 - 2 dS  (dS from the fp4 residuals, gallery maxima).
Prints the fraction of queries that pass for fp4 and, for reference, fp6 (e2m3)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import build_projection  # noqa: E402
from opencv_facerecognizer_amd import _lib  # noqa: E402
from opencv_facerecognizer_amd._device import col_mean_u8, round_up  # noqa: E402
from opencv_facerecognizer_amd.synthetic import SEED, IdentityBank  # noqa: E402

E2M1 = torch.tensor([0, 0.5, 1, 1.5, 2, 3, 4, 6], dtype=torch.float64)
E2M3 = torch.tensor([m / 8 for m in range(8)] + [(1 + m / 8) * 2.0 ** (e - 1) for e in (1, 2, 3) for m in range(8)],
                    dtype=torch.float64)


def quant(X, grid):
    g = grid.to(X.device)
    s = X.abs().amax(1, keepdim=True) / g[-1]
    s[s == 0] = 1
    r = (X / s).abs()
    idx = torch.bucketize(r, (g[1:] + g[:-1]) / 2)
    Xt = torch.sign(X) * g[idx] * s
    return Xt, Xt.norm(dim=1), (X - Xt).norm(dim=1)


def main():
    dev = _lib.device()
    N, B, d, per = int(os.environ.get("N", 1_000_000)), 4096, 9999, 10
    P, _ = build_projection(10000, d, dev)
    bank = IdentityBank(-(-N // per), 100, 100, device=dev)   # row j shows identity j // per
    ld = round_up(d, 32)
    G = torch.zeros((N, ld), dtype=torch.float32, device=dev)
    m = col_mean_u8(bank.images(torch.arange(8192, device=dev) // per, seed=SEED + 1000), 10000)
    c = P.project(torch.clamp(torch.round(m), 0, 255).to(torch.uint8).reshape(1, -1), f64=True)[0].contiguous()
    for c0 in range(0, N, 8192):
        rows = torch.arange(c0, min(N, c0 + 8192), device=dev)
        P.project(bank.images(rows // per, seed=SEED + 1000 + c0 // 8192), shift64=c, out=G[c0:c0 + len(rows)])
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + 7)
    ids = torch.randint(0, N // per, (B,), generator=g, device=dev)
    Q = P.project(bank.images(ids, seed=SEED + 99), shift64=c)[:, :d].double()
    qn = (Q * Q).sum(1)
    best = torch.full((B, 16), float("inf"), dtype=torch.float64, device=dev)
    stats = {}
    for name, grid in (("fp4", E2M1), ("fp6", E2M3)):
        stats[name] = [0.0, 0.0, 0.0]           # A, E, auxmax
    for c0 in range(0, N, 65536):
        Gc = G[c0:c0 + 65536, :d].double()
        S = (Gc * Gc).sum(1)[None, :] - 2 * Q @ Gc.T            # d^2 - |q|^2
        best = torch.cat([best, S], 1).topk(16, dim=1, largest=False).values
        for name, grid in (("fp4", E2M1), ("fp6", E2M3)):
            _, a, e = quant(Gc, grid)
            st = stats[name]
            st[0], st[1] = max(st[0], float(a.max())), max(st[1], float(e.max()))
            st[2] = max(st[2], float((Gc * Gc).sum(1).max()))
    out = {}
    for name, grid in (("fp4", E2M1), ("fp6", E2M3)):
        _, a, e = quant(Q, grid)
        A, E, auxmax = stats[name]
        dS = 2 * (a * E + e * A + e * E) + 2 ** -20 * (auxmax + 2 * a * A)
        ok = best[:, 0] < best[:, 15] - 2 * dS
        out[name] = {"certified_frac": float(ok.double().mean()), "rel_residual_q": float((e / a).mean()),
                     "median_margin_over_dS": float(((best[:, 15] - best[:, 0]) / dS).median())}
    print(out, flush=True)


if __name__ == "__main__":
    main()
