"""Reference point for the projection engine: the library int8 GEMM (torch._int_mm -> hipBLASLt) on the
projection's shape, 4,096 faces x D = 10,000 (padded to 10,048) x 4 slices of d = 9,999 features (39,996 + pad).
Prints ms per GEMM (median of reps) and the fraction of the 5 POPS int8 dense peak."""
import json
import torch

M, K, N = 4096, 10048, 40064
dev = torch.device("cuda", 0)
a = torch.randint(-128, 127, (M, K), dtype=torch.int8, device=dev)
for layout in ("nt", "nn"):
    if layout == "nt":
        b = torch.randint(-128, 127, (N, K), dtype=torch.int8, device=dev).t()
    else:
        b = torch.randint(-128, 127, (K, N), dtype=torch.int8, device=dev)
    try:
        for _ in range(3):
            c = torch._int_mm(a, b)
        torch.cuda.synchronize()
        ms = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            c = torch._int_mm(a, b)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        ms.sort()
        m = ms[len(ms) // 2]
        print(json.dumps({"layout": layout, "ms": m, "min": ms[0], "frac_int8_peak": 2.0 * M * K * N / (m * 1e-3) / 5e15}), flush=True)
    except Exception as ex:  # noqa: BLE001
        print(json.dumps({"layout": layout, "error": str(ex)[:300]}), flush=True)
