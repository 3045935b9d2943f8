import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from opencv_facerecognizer_amd._device import round_up
from opencv_facerecognizer_amd.synthetic import IdentityBank, build_gallery, build_trained_projection
dev = torch.device("cuda", 0)
N, per, side = 1_000_000, 10, 100
bank = IdentityBank(N // per, side, side, device=dev)
P, _, info = build_trained_projection(bank, per, 100_000, side * side, dev)
g = build_gallery(P, bank, per, 0, N, N, P.d, max(32, round_up(P.d, 32)), dev)
print("pst", g.prefix_stages())
sums = g.block_sums().cpu().numpy().astype(np.float64)
d = g.d
width = np.minimum(32, d - 32 * np.arange(len(sums)))
ms = sums / (N * width)
tot = ms.dot(width)
for p in range(1, 9):
    nb = 4 * p
    print("stages", p, "share %.4f" % (ms[:nb].dot(width[:nb]) / tot))
med = np.median(ms)
print("lead blocks", np.nonzero(ms >= 8 * med)[0][:20], "median", med)
