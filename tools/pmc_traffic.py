#!/usr/bin/env python3
"""Per-launch HBM traffic of the fused env-step kernel from rocprofv3 PMC passes.

    python tools/pmc_traffic.py <Task> <fetch_dir> <write_dir> [--out profiles/traffic_<task>.json]

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB (TCC_EA0 memory-side requests;
Infinity-Cache hits are counted, not excluded). Per MI355X_MICROARCH.md (HBM section) gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads: we report the raw value and the
doubled one; `bytes_per_launch` (what bench.py quotes as roofline.traffic) uses the doubled
read bytes + write bytes, i.e. the upper estimate."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(d: str, counter: str, kernel_sub: str):
    """Per-dispatch counter values of kernels whose name contains kernel_sub, from the
    rocprofv3 output under d (CSV counter_collection files or the rocpd SQLite database)."""
    vals = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and kernel_sub in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)):
        import sqlite3
        db = sqlite3.connect(f)
        q = ("select value from counters_collection where counter_name = ? and kernel_name like ? "
             "order by dispatch_id")
        vals += [float(r[0]) for r in db.execute(q, (counter, f"%{kernel_sub}%"))]
    if not vals:
        raise SystemExit(f"no {counter} rows for *{kernel_sub}* under {d}")
    vals = vals[len(vals) // 4:]   # drop the warm-up quarter
    return sum(vals) / len(vals), len(vals)


def main():
    task, fdir, wdir = sys.argv[1:4]
    out = os.path.join(ROOT, "profiles", f"traffic_{task}.json")
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_env_step"
    n_envs = int(sys.argv[sys.argv.index("--num-envs") + 1]) if "--num-envs" in sys.argv else None
    fkb, nf = per_launch(fdir, "FETCH_SIZE", kern)
    wkb, nw = per_launch(wdir, "WRITE_SIZE", kern)
    rec = {
        "task": task, "kernel": kern + ("* (fused env step)" if kern == "k_env_step" else "*"),
        "num_envs": n_envs, "launches": {"fetch": nf, "write": nw},
        "fetch_kib_raw": round(fkb, 1), "write_kib_raw": round(wkb, 1),
        "read_bytes_corrected": round(2 * fkb * 1024), "write_bytes": round(wkb * 1024),
        "bytes_per_launch": round(2 * fkb * 1024 + wkb * 1024),
        # lower estimate: FETCH_SIZE as reported (the x2 correction is calibrated for 16-B-per-lane
        # streaming reads; narrower per-lane reads are uncalibrated, MI355X_MICROARCH.md HBM)
        "bytes_per_launch_uncorrected": round(fkb * 1024 + wkb * 1024),
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate runs, --kernel-trace; "
                  "FETCH doubled per the gfx950 correction; warm-up quarter dropped",
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
