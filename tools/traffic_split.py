#!/usr/bin/env python3
"""Per-launch HBM traffic of the fused env-step kernel, split into instruction fetch, per-env
reads and per-env writes, from the env-count sweep of tools/gpu.sh traffic.

    python tools/traffic_split.py <Task> <sweep_dir> [--n 4096] [--out profiles/traffic_<task>.json]

Calibration (tools/fetch_calib.hip, profiles/r02/fetch_calib.json): on gfx950 FETCH_SIZE
reports 1/2 of the bytes of the wave kernel's data reads (4 B/lane partial waves and
16 B/lane streaming alike: factor 2.0), but the instruction fetch of a launch at face value
(factor 1.0: a 196 684-B straight-line kernel on 2048 workgroups reads 8 x its code size, one
copy per XCD L2 per launch). WRITE_SIZE reads the bytes exactly (factor 1.0).

The sweep separates the two read sources: FETCH_SIZE(N) = fixed + slope * N, where the fixed
part is the launch's instruction fetch (8 XCDs x the code the launch touches; the L2s do not keep
it from one launch to the next) and the slope the per-env data reads. So
    reads  = fixed + 2 * slope * N        (code at face value, data doubled)
    writes = WRITE_SIZE(N)
at the bench's N, with the fixed / slope from a least-squares fit over the sweep."""
import glob
import json
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import per_launch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALGO = {"Humanoid": 920, "Ant": 552, "Cartpole": 80}   # SURVEY §8(d) bytes per env-step


def main():
    task, base = sys.argv[1], sys.argv[2]
    n_bench = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 4096
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else \
        os.path.join(ROOT, "profiles", f"traffic_{task}.json")
    kern = "k_env_step"
    ns, fr, wr = [], [], []
    for d in sorted(glob.glob(os.path.join(base, f"tsf_{task}_*"))):
        m = re.search(r"_(\d+)$", d)
        if not m or not os.path.isdir(d):
            continue
        n = int(m.group(1))
        wd = os.path.join(base, f"tsw_{task}_{n}")
        ns.append(n)
        fr.append(per_launch(d, "FETCH_SIZE", kern)[0] * 1024.0)
        wr.append(per_launch(wd, "WRITE_SIZE", kern)[0] * 1024.0)
    order = np.argsort(ns)
    ns, fr, wr = np.array(ns)[order], np.array(fr)[order], np.array(wr)[order]
    A = np.vstack([ns, np.ones(len(ns))]).T
    f_slope, f_fixed = np.linalg.lstsq(A, fr, rcond=None)[0]
    w_slope, w_fixed = np.linalg.lstsq(A, wr, rcond=None)[0]
    i = list(ns).index(n_bench)
    code = f_fixed
    data_raw = fr[i] - code
    reads = code + 2.0 * data_raw
    rec = {
        "task": task, "kernel": kern + "* (fused env step)", "num_envs": n_bench,
        "sweep_envs": [int(x) for x in ns],
        "fetch_bytes_raw": [round(x) for x in fr], "write_bytes": [round(x) for x in wr],
        "fit": {"fetch_raw_fixed_bytes": round(f_fixed), "fetch_raw_per_env": round(f_slope, 1),
                "write_fixed_bytes": round(w_fixed), "write_per_env": round(w_slope, 1)},
        "instruction_fetch_bytes": round(code),
        "data_read_bytes": round(2.0 * data_raw),
        "read_bytes": round(reads),
        "write_bytes_at_n": round(wr[i]),
        "bytes_per_launch": round(reads + wr[i]),
        "bytes_per_launch_uncorrected": round(fr[i] + wr[i]),
        "per_env": {"data_read": round(2.0 * f_slope, 1), "write": round(w_slope, 1),
                    "algorithmic": ALGO.get(task)},
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate runs over an env-count "
                  "sweep; fixed part of FETCH = instruction fetch (face value, calibrated), per-env "
                  "part doubled (gfx950 data-read factor 2.0, calibrated); warm-up quarter dropped",
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
