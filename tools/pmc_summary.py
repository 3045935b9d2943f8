"""Summarise the rocprofv3 passes of tools/prof_search.sh (gpurun_out/prof) into profiles/.

    python tools/pmc_summary.py <name> ["kernel-substring[;kernel-substring...]"]

Several substrings (the kernels of one phase, e.g. the fp6 sieve's sample pass, thresholds and
sieve pass) are summed: durations and counters per phase launch, with the per-kernel split.

writes profiles/<name>_kernel_stats.csv (the --stats table) and profiles/<name>_pmc_summary.json
(per-launch counters of the search tile kernel; traffic = FETCH_SIZE x 2 + WRITE_SIZE, the gfx950
correction of MI355X_MICROARCH.md §HBM).  bench.py reads traffic_bytes_per_launch back when the
config matches its own run.
"""
import collections
import csv
import datetime
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "gpurun_out", "prof")


def sieve_engine(name):
    sys.path.insert(0, ROOT)
    import bench
    return bench.sieve_engine(name)


def counters(kname):
    agg = collections.defaultdict(list)
    for p in ("p1", "p2", "p3", "p4", "p5"):
        f = os.path.join(P, p, f"{p}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, max((len(v) for v in agg.values()), default=0)


def main():
    name = sys.argv[1]
    knames = (sys.argv[2] if len(sys.argv) > 2 else "tile_kernel_f6<8, 0, 1>;sieve_threshold_kernel;tile_kernel_f6s<").split(";")
    stats = os.path.join(P, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{name}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    per = {}
    for kn in knames:
        ns = [float(r["AverageNs"]) for r in rows if kn in r["Name"]]
        c, n = counters(kn)
        per[kn] = {"rocprof_avg_ns": ns[-1] if ns else None, "launches": n, "counters_per_launch": c}
    c = collections.Counter()
    for v in per.values():
        c.update(v["counters_per_launch"])
    avg_ns = sum(v["rocprof_avg_ns"] or 0.0 for v in per.values()) or None
    log = open(os.path.join(P, "kt.log")).read().strip().splitlines()
    bench = json.loads([ln for ln in log if ln.startswith("{")][-1])
    cfg = bench["config"]
    search = "f6" if "fp6" in bench["dtype"] else ("q8" if "i8" in bench["dtype"] else "fp32")
    out = {
        "config": {"gallery": cfg["gallery"], "batch": cfg["global_batch"], "d": cfg["d"], "D": cfg["D"],
                   "k": cfg["k"],
                   "search": search,
                   "w": "trained" if "trained" in cfg.get("workload", "") else "random",
                   # the tier the timed steps started at (f6p: the prefix tier's pass)
                   "tier": max((bench.get("start_tiers") or {"": 0}).items(), key=lambda t: t[1])[0] or search,
                   # the sieve kernel the bench's roofline names (bench.sieve_engine)
                   "engine": sieve_engine(bench["roofline"].get("kernel"))},
        # bench.committed_traffic takes the newest summary of its config (file names do not order rounds)
        "measured_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
        "kernel": " + ".join(knames), "launches": min(v["launches"] for v in per.values()), "rocprof_avg_ns": avg_ns,
        "bench_launch_ms": bench["roofline"].get("launch_ms"),
        "counters_per_launch": dict(c),
        "per_kernel": per if len(knames) > 1 else None,
        "correction": "gfx950: FETCH_SIZE reports half of the bytes of wide coalesced streaming reads "
                      "(MI355X_MICROARCH.md §HBM) -> x2; WRITE_SIZE exact for 16-B stores",
    }
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["traffic_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    if "TCC_HIT_sum" in c:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in c and avg_ns:
        out["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / avg_ns
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "SQ_WAVE_CYCLES" in c:
        out["mfma_busy_per_wave_cycle"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * c["SQ_WAVE_CYCLES"])
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{name}_pmc_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
