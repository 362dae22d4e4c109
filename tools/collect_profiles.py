#!/usr/bin/env python3
"""Copy the judged summaries of a tools/gpu.sh run from gpurun_out/ into profiles/<round>/:
rocprofv3 kernel stats per task, PMC traffic (also profiles/traffic_<task>.json, read by
bench.py), SQ issue/wait counters, phase-stamp breakdowns and the default bench line.

    python tools/collect_profiles.py r01
"""
import csv
import glob
import json
import os
import shutil
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def counters(d, kernel_sub="k_env_step"):
    """{counter: mean per dispatch} for kernels matching kernel_sub (CSV or rocpd db)."""
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub in row.get("Kernel_Name", ""):
                    acc.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        db = sqlite3.connect(f)
        for name, v in db.execute("select counter_name, value from counters_collection "
                                  "where kernel_name like ?", (f"%{kernel_sub}%",)):
            acc.setdefault(name, []).append(float(v))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    rnd = sys.argv[1]
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for task in ("Humanoid", "Ant", "Cartpole"):
        for f in glob.glob(os.path.join(OUT, f"prof_{task}", "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(dst, f"kernel_stats_{task.lower()}.csv"))
        if os.path.isdir(os.path.join(OUT, f"pmcf_{task}")):
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), task,
                            os.path.join(OUT, f"pmcf_{task}"), os.path.join(OUT, f"pmcw_{task}")],
                           check=True)
            shutil.copy(os.path.join(ROOT, "profiles", f"traffic_{task}.json"),
                        os.path.join(dst, f"traffic_{task.lower()}.json"))
    # obs/reward fuse (k_loco_post_tiled) at 1M Humanoid envs: stats, traffic, roofline sweep
    for f in glob.glob(os.path.join(OUT, "prof_fuse", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, "kernel_stats_fuse_humanoid.csv"))
    if os.path.isdir(os.path.join(OUT, "pmcf_fuse")):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), "Humanoid",
                        os.path.join(OUT, "pmcf_fuse"), os.path.join(OUT, "pmcw_fuse"), "--kernel",
                        "k_loco_post_tiled", "--out", os.path.join(dst, "traffic_fuse_humanoid.json")],
                       check=True)
    for t in ("humanoid", "ant"):
        p = os.path.join(OUT, f"fuse_roofline_{t}.json")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"fuse_roofline_{t}.json"))
    sq = {}
    for d in ("sq1", "sq2"):
        if os.path.isdir(os.path.join(OUT, d)):
            sq.update(counters(os.path.join(OUT, d)))
    if sq:
        w = sq.get("SQ_WAVES", 1.0)
        lines = ["SQ counters, Humanoid 4096 envs, fused env-step kernel; mean per dispatch "
                 "(SQ_*_CYCLES / WAIT / ACTIVE in quad-cycles, summed over waves)"]
        lines += [f"{k:24s} {v:.6g}" for k, v in sorted(sq.items())]
        if "SQ_WAVE_CYCLES" in sq:
            wc = sq["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if k in sq:
                    lines.append(f"{k:24s} {100 * sq[k] / wc:5.1f} % of wave cycles")
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if k in sq:
                    lines.append(f"{k:24s} {sq[k] / w:9.1f} per wave (per env-step)")
            if "GRBM_GUI_ACTIVE" in sq:
                # occupancy (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE sums the 8 XCDs; SQ cycle
                # counters are quad-cycles): mean resident waves per CU over the dispatch
                kcyc = sq["GRBM_GUI_ACTIVE"] / 8.0
                waves_cu = 4.0 * wc / (kcyc * 256.0)
                lines.append(f"{'kernel cycles / XCD':24s} {kcyc:.4g}")
                lines.append(f"{'mean wave lifetime':24s} {4.0 * wc / w:.4g} cycles")
                lines.append(f"{'resident waves / CU':24s} {waves_cu:5.2f} (mean over the dispatch)")
                lines.append(f"{'occupancy':24s} {100 * waves_cu / 8:5.1f} % of the kernel's 8 waves/CU "
                             f"(2/SIMD: VGPR + LDS), {100 * waves_cu / 32:5.1f} % of the CDNA4 32 waves/CU cap")
        with open(os.path.join(dst, "sq_counters_humanoid.txt"), "w") as f:
            f.write("\n".join(lines) + "\n")
    for name in ("stamps_humanoid", "stamps_ant", "bench_default"):
        p = os.path.join(OUT, f"{name}.log")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{name}.log"))
    print("collected into", dst, sorted(os.listdir(dst)))


if __name__ == "__main__":
    main()
