"""Clock and MFMA busy per kernel variant from one `rocprofv3 --pmc GRBM_GUI_ACTIVE
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES` pass over tools/f6_probe (tools/gpu_pclk.sh).

    python tools/pmc_clock_summary.py gpurun_out/pclk4/p/p_counter_collection.csv [out.json]

Per kernel (template arguments kept: the probe variants differ only in them): launches, mean
duration (counter-collection timestamps), effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration,
MFMA busy per SIMD cycle = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs).
"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "tile_kernel" not in name:
            continue
        key = name.split("(")[0]
        rows[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[key][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {}
    for k, cs in rows.items():
        c = {n: sum(v) / len(v) for n, v in cs.items()}
        ns = sum(dur[k].values()) / len(dur[k])
        e = {"launches": len(dur[k]), "avg_ms": ns / 1e6, "counters_per_launch": c}
        if "GRBM_GUI_ACTIVE" in c:
            e["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / ns
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                e["mfma_busy_per_simd_cycle"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
        out[k] = e
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
