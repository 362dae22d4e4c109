#!/usr/bin/env python3
"""Copy the judged summaries of a tools/gpu.sh run from gpurun_out/ into profiles/<round>/:
rocprofv3 kernel stats of the default bench, PMC traffic split by source (also
profiles/traffic_<task>.json, read by bench.py), SQ issue / wait / occupancy counters, the
GPU test / smoke logs and the default bench line.

    python tools/collect_profiles.py r03 [tag of the sq runs, default = round]
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


def sq_summary(task, tag):
    """SQ issue / wait / occupancy summary of the fused env-step kernel from tools/gpu.sh sq."""
    sq = {}
    for d in ("sq1", "sq2", "sq3"):
        p = os.path.join(OUT, f"{d}_{task}_{tag}")
        if os.path.isdir(p):
            sq.update(counters(p))
    if not sq:
        return None
    kname = kernel_name(os.path.join(OUT, f"sq1_{task}_{tag}"))
    envs_per_wave = 2 if "pair" in kname else 1
    cap = 8 if ("pair" in kname or task == "Humanoid") else 16   # resident waves/CU the kernel allows
    w = sq.get("SQ_WAVES", 1.0)
    lines = [f"SQ counters, {task} 4096 envs, fused env-step kernel {kname}; mean per dispatch "
             "(SQ_*_CYCLES / WAIT / ACTIVE in quad-cycles, summed over waves)"]
    lines += [f"{k:24s} {v:.6g}" for k, v in sorted(sq.items())]
    if "SQ_WAVE_CYCLES" in sq:
        wc = sq["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS"):
            if k in sq:
                lines.append(f"{k:24s} {100 * sq[k] / wc:5.1f} % of wave cycles")
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR"):
            if k in sq:
                lines.append(f"{k:24s} {sq[k] / w:9.1f} per wave ({envs_per_wave} env(s) per wave, one env-step)")
        if "GRBM_GUI_ACTIVE" in sq:
            # occupancy (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE sums the 8 XCDs; SQ cycle counters
            # are quad-cycles): mean resident waves per CU over the dispatch
            kcyc = sq["GRBM_GUI_ACTIVE"] / 8.0
            waves_cu = 4.0 * wc / (kcyc * 256.0)
            lines.append(f"{'kernel cycles / XCD':24s} {kcyc:.4g}")
            lines.append(f"{'mean wave lifetime':24s} {4.0 * wc / w:.4g} cycles")
            lines.append(f"{'resident waves / CU':24s} {waves_cu:5.2f} (mean over the dispatch)")
            lines.append(f"{'resident envs / CU':24s} {waves_cu * envs_per_wave:5.2f} ({envs_per_wave} per wave)")
            lines.append(f"{'occupancy':24s} {100 * waves_cu / cap:5.1f} % of the kernel's {cap} waves/CU, "
                         f"{100 * waves_cu / 32:5.1f} % of the CDNA4 32 waves/CU cap")
    return "\n".join(lines) + "\n"


def kernel_name(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_env_step" in row.get("Kernel_Name", ""):
                    return row["Kernel_Name"].split("(")[0]
    return "?"


def main():
    """python tools/collect_profiles.py <round> [tag]: summaries of tools/gpu.sh sq / prof /
    traffic / tests / smoke / bench outputs into profiles/<round>/."""
    rnd = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else rnd
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for task in ("Humanoid", "Ant", "Cartpole"):
        txt = sq_summary(task, tag)
        if txt:
            with open(os.path.join(dst, f"sq_counters_{task.lower()}.txt"), "w") as f:
                f.write(txt)
        if glob.glob(os.path.join(OUT, f"tsf_{task}_*")):
            out = os.path.join(ROOT, "profiles", f"traffic_{task}.json")
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_split.py"), task, OUT,
                            "--out", out], check=True)
            shutil.copy(out, os.path.join(dst, f"traffic_{task.lower()}.json"))
    for f in glob.glob(os.path.join(OUT, "prof_bench", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, "kernel_stats_bench_default.csv"))
    for f in glob.glob(os.path.join(OUT, "prof_fuse", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, "kernel_stats_fuse_humanoid.csv"))
    for t in ("humanoid", "ant"):
        p = os.path.join(OUT, f"fuse_roofline_{t}.json")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"fuse_roofline_{t}.json"))
    for name in ("bench_default", "pytest_gpu", "smoke"):
        p = os.path.join(OUT, f"{name}.log")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{name}.log"))
    print("collected into", dst, sorted(os.listdir(dst)))


if __name__ == "__main__":
    main()
