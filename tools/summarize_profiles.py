"""Condense gpurun_out/prof_ROUND/<leg>/ (tools/profile_round.sh) into profiles/:
ROUND_<leg>_kernel_stats.csv (rocprofv3 --stats) and ROUND_profile_summary.json with, per leg,
the kernel's rocprof average duration, algorithmic bytes per launch, PMC
traffic per launch (FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 rule + WRITE_SIZE)
and SQ counters; plus ROUND_pmc_traffic.json for the bench headline kernel (bench.py reads it).

    python tools/summarize_profiles.py ROUND"""
import csv
import glob
import json
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEGS = {"cfg2": (64, 1499, 300, 500, 1000, 32), "cfg5": (64, 2999, 850, 950, 55, 40),
        "sat3000": (2048, 2999, 850, 951, 78, 32), "trellis3000": (2048, 2999, 850, 951, 78, 32)}
# bench.py's pmc_traffic() reads these (newest round first, matched by kernel name)
TRAFFIC_FILES = {"cfg2": "pmc_traffic.json", "cfg5": "pmc_traffic_cfg5.json", "sat3000": "pmc_traffic_sat3000.json"}


def Ns(S, T, lo, hi, seed, V=32):
    """Token counts of tools/satbench.make_batch (replays its numpy draws)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(S):
        N = int(rng.integers(lo, hi + 1))
        rng.integers(1, V, N)
        rng.choice(np.arange(1, T - 1), N, replace=False)
        out.append(N)
    return out


def per_dispatch(d, ksub):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if ksub not in row["Kernel_Name"]:
                continue
            k = (row["Dispatch_Id"], row["Counter_Name"])
            acc[k] = acc.get(k, 0.0) + float(row["Counter_Value"])
    by = {}
    for (disp, name), v in acc.items():
        by.setdefault(name, []).append(v)
    return {n: float(np.mean(v)) for n, v in by.items()}, {n: len(v) for n, v in by.items()}


def main():
    rnd = sys.argv[1]
    base = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    summary = {}
    for leg, (S, T, lo, hi, seed, V) in LEGS.items():
        d = os.path.join(base, leg)
        stats = glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True)
        if not stats:
            continue
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{rnd}_{leg}_kernel_stats.csv"))
        ksub = "trellis_kernel" if leg == "trellis3000" else "align_dp"
        rows = [r for r in csv.DictReader(open(stats[0])) if ksub in r["Name"]]
        top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
        avg_ns = float(top["AverageNs"])
        n = Ns(S, T, lo, hi, seed, V)
        if leg == "trellis3000":
            alg = sum(4 * T * V + 4 * x + 4 * (T + 1) * (x + 1) for x in n)
        else:
            alg = sum(4 * T * V + 4 * x + (T * x) // 8 + 16 * x for x in n)
        pmc = {}
        for sub in ("fetch", "write", "sq", "lds"):
            v, cnt = per_dispatch(os.path.join(d, sub), ksub)
            pmc.update(v)
        fetch_b = 2 * pmc.get("FETCH_SIZE", float("nan")) * 1024  # gfx950: FETCH_SIZE counts half
        write_b = pmc.get("WRITE_SIZE", float("nan")) * 1024
        achieved = alg / (avg_ns * 1e-9) / 1e9
        summary[leg] = {
            "kernel": top["Name"], "launches": int(top["Calls"]), "rocprof_avg_us": avg_ns / 1e3,
            "segments": S, "T": T, "algorithmic_bytes_per_launch": alg,
            "achieved_GBps": achieved, "frac_of_8TBps": achieved / 8000.0,
            "cells_per_s": sum(T * x for x in n) / (avg_ns * 1e-9),
            "pmc_fetch_bytes_corrected": fetch_b, "pmc_write_bytes": write_b,
            "pmc_traffic_bytes_per_launch": fetch_b + write_b,
            "traffic_over_algorithmic": (fetch_b + write_b) / alg,
            "sq": {k: v for k, v in pmc.items() if k.startswith("SQ_")},
        }
        sq = summary[leg]["sq"]
        if sq.get("SQ_BUSY_CYCLES") and sq.get("SQ_ACTIVE_INST_VALU"):
            summary[leg]["valu_active_per_busy_cycle"] = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_BUSY_CYCLES"]
        if sq.get("SQ_BUSY_CYCLES") and sq.get("SQ_LDS_CMD_FIFO_FULL") is not None:
            summary[leg]["lds_cmd_fifo_full_per_busy_cycle"] = sq["SQ_LDS_CMD_FIFO_FULL"] / sq["SQ_BUSY_CYCLES"]
        if sq.get("SQ_INSTS_VALU"):  # VALU instructions per 64 cells of one step (a wave64 step of 64 cells)
            summary[leg]["valu_per_64_cell_step"] = sq["SQ_INSTS_VALU"] / (sum(T * x for x in n) / 64.0)
        if leg in TRAFFIC_FILES:
            with open(os.path.join(ROOT, "profiles", f"{rnd}_{TRAFFIC_FILES[leg]}"), "w") as fh:
                json.dump({"kernel": top["Name"], "command": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE "
                           f"(separate passes) -- python3 tools/legs.py {leg} --steps 5",
                           "algorithmic_bytes_per_launch": alg,
                           "traffic_over_algorithmic": (fetch_b + write_b) / alg,
                           "fetch_size_kb_raw": pmc.get("FETCH_SIZE"), "write_size_kb": pmc.get("WRITE_SIZE"),
                           "correction": "FETCH_SIZE doubled (MI355X_MICROARCH.md: gfx950 counts half of a "
                                         "16-B/lane streaming read)",
                           "traffic_bytes_per_launch": int(round(fetch_b + write_b))}, fh, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{rnd}_profile_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    for k, v in summary.items():
        print(k, {x: v[x] for x in ("kernel", "rocprof_avg_us", "frac_of_8TBps", "traffic_over_algorithmic")},
              v.get("valu_active_per_busy_cycle"))


if __name__ == "__main__":
    main()
