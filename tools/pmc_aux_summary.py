"""Summarise tools/prof_aux_pmc.sh (gpurun_out/prof_auxpmc) into profiles/<name>_aux_pmc_summary.json.

    python tools/pmc_aux_summary.py <name>

Per kernel and launch shape (grid size): rocprofv3 average duration, counters per launch, HBM-side
traffic = FETCH_SIZE x 2 + WRITE_SIZE (the gfx950 correction of MI355X_MICROARCH.md §HBM), effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), MFMA busy per SIMD cycle and VALU instructions per
wave-cycle.  Copies the --stats tables to profiles/<name>_aux_<tag>_kernel_stats.csv.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "gpurun_out", "prof_auxpmc")
KERNELS = ("gemm_f64_kernel", "gram_u8_kernel", "elbp_hist_r1p8_kernel", "chi2_tile_kernel")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def grid_of(row):
    """Total work-items of the dispatch: Grid_Size (counter CSV) or Grid_Size_X*Y*Z (kernel trace)."""
    if row.get("Grid_Size"):
        return row["Grid_Size"]
    try:
        return str(int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"]))
    except (KeyError, ValueError):
        return "?"


def main():
    name = sys.argv[1]
    out = {"correction": "gfx950: FETCH_SIZE reports half of the bytes of wide coalesced reads -> x2",
           "kernels": {}}
    for tag in ("gemm", "lbp"):
        base = os.path.join(P, tag)
        stats = os.path.join(base, "kt", "kt_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(ROOT, "profiles", f"{name}_aux_{tag}_kernel_stats.csv"))
        # durations per (kernel, grid) from the trace
        dur = collections.defaultdict(list)
        for f in glob.glob(os.path.join(base, "kt", "*kernel_trace.csv")):
            for r in csv.DictReader(open(f)):
                k = short(r.get("Kernel_Name", ""))
                if k:
                    dur[(k, grid_of(r))].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
        cnt = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in glob.glob(os.path.join(base, "p*", "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = short(r.get("Kernel_Name", ""))
                if k:
                    cnt[(k, grid_of(r))][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for key, cs in cnt.items():
            c = {n: sum(v) / len(v) for n, v in cs.items()}
            ds = dur.get(key, [])
            ns = sum(ds) / len(ds) if ds else None
            e = {"tool": tag, "grid": key[1], "launches_traced": len(ds), "avg_ns": ns, "counters_per_launch": c}
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                e["hbm_traffic_bytes"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
                if ns:
                    e["hbm_gbs"] = e["hbm_traffic_bytes"] / ns
            if "GRBM_GUI_ACTIVE" in c and ns:
                e["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / ns
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
                e["mfma_busy_per_simd_cycle"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
            if "SQ_INSTS_VALU" in c and "SQ_WAVE_CYCLES" in c:
                e["valu_insts_per_wave_cycle"] = c["SQ_INSTS_VALU"] / c["SQ_WAVE_CYCLES"]
            if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
                e["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
            out["kernels"][f"{key[0]} grid={key[1]}"] = e
    path = os.path.join(ROOT, "profiles", f"{name}_aux_pmc_summary.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
