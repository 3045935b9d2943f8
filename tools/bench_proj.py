"""Exact projection engines at the bench shape: time each and check they agree bit for bit.

Runs ofr_project_u8_exact (Fisherfaces.project, reference feature.py:241-242) on B faces of
D pixels against a random d-column W, once per engine (OFR_PROJ_ENGINE is read once per process,
so every engine runs in its own child process), with HIP events on the launch stream, and compares
each engine's fp32 and fp64 outputs with the first engine's (the products are exact integers, so
every engine must give identical bits).  One JSON line.

    python tools/bench_proj.py [--batch 4096] [--D 10000] [--d 9999] [--reps 20] [--engines i8,s4,s5]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(a):
    import numpy as np
    import torch
    from opencv_facerecognizer_amd import _device as D_

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    W = torch.randn((a.d, a.D), generator=g, device=dev, dtype=torch.float32)
    P = D_.Projection(Wt_device=W, D=a.D, device=dev)
    ldx = D_.round_up(a.D, 16)
    X = torch.randint(0, 256, (a.batch, ldx), generator=g, device=dev, dtype=torch.int32).to(torch.uint8)
    shift = torch.randn(a.d, generator=g, device=dev, dtype=torch.float64) * 100
    y32 = P.project(X, shift64=shift)
    y64 = P.project(X[:a.check_rows], shift64=shift, f64=True)
    st = torch.cuda.current_stream()
    for _ in range(3):
        P.project(X, shift64=shift, out=y32)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(st)
    for _ in range(a.reps):
        P.project(X, shift64=shift, out=y32)
    ev[1].record(st)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.reps
    np.save(a.out + "_y32.npy", y32.cpu().numpy())
    np.save(a.out + "_y64.npy", y64.cpu().numpy())
    ops = 2.0 * a.batch * P.Aq.numel()   # int8 ops executed: 2 x B x (4 slices x padded rows) x ldk
    print(json.dumps({"ms": ms, "int8_tops_executed": ops / ms / 1e9}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--D", type=int, default=10000)
    ap.add_argument("--d", type=int, default=9999)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--check-rows", type=int, default=64)
    ap.add_argument("--engines", default="dma,reg")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.child:
        return child(a)
    import numpy as np
    res = {"config": {"batch": a.batch, "D": a.D, "d": a.d}, "engines": {}}
    ref = None
    import tempfile
    tmp = os.path.join(tempfile.mkdtemp(prefix="bench_proj_"), "y")   # outputs are large: not under gpurun_out
    for eng in a.engines.split(","):
        # "lib=<path>": the default engine of another build of the library (same-box A/B)
        # "lib=<path>": another build of the library (same-box A/B); other names: OFR_PROJ_ENGINE
        if eng.startswith("lib="):
            env = dict(os.environ, OFR_LIB=eng[4:])
        else:
            env = dict(os.environ, OFR_PROJ_ENGINE=eng, OFR_PROJ_STAGE=eng)   # stage copies: dma | reg
        key = f"{len(res['engines'])}:{eng}"
        out = f"{tmp}_{len(res['engines'])}"
        cmd = [sys.executable, os.path.abspath(__file__), "--child", "--out", out, "--batch", str(a.batch), "--D",
               str(a.D), "--d", str(a.d), "--reps", str(a.reps), "--check-rows", str(a.check_rows)]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            res["engines"][key] = {"error": r.stderr[-2000:]}
            print(json.dumps(res), flush=True)
            sys.exit(r.returncode)
        rec = json.loads(r.stdout.strip().splitlines()[-1])
        y32, y64 = np.load(out + "_y32.npy"), np.load(out + "_y64.npy")
        os.remove(out + "_y32.npy")
        os.remove(out + "_y64.npy")
        if ref is None:
            ref = (eng, y32, y64)
        else:
            rec["identical_to_" + ref[0]] = bool(np.array_equal(y32, ref[1]) and np.array_equal(y64, ref[2]))
            rec["max_abs_diff_f64"] = float(np.max(np.abs(y64 - ref[2])))
            bad = np.argwhere(y64 != ref[2])        # where the first rows differ: (image, feature) pattern
            if len(bad):
                rec["mismatch"] = {"count": int(len(bad)), "of": int(y64.size),
                                   "images": sorted(set(int(x) for x in bad[:, 0]))[:16],
                                   "features_mod_128": sorted(set(int(x) % 128 for x in bad[:, 1]))[:40],
                                   "features_first": [int(x) for x in bad[:12, 1]],
                                   "image0_features": [int(x) for x in bad[bad[:, 0] == 0][:64, 1]],
                                   "image0_diffs": [float(y64[0, x] - ref[2][0, x]) for x in bad[bad[:, 0] == 0][:12, 1]],
                                   "per_image": [int((bad[:, 0] == i).sum()) for i in range(16)]}
        res["engines"][key] = rec
        print(eng, rec, file=sys.stderr, flush=True)
    ok = all(v.get("identical_to_" + ref[0], True) for v in res["engines"].values())
    res["all_identical"] = ok
    print(json.dumps(res), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
