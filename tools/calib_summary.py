#!/usr/bin/env python3
"""Correction factors of FETCH_SIZE / WRITE_SIZE per access width, from the rocprofv3 passes of
tools/fetch_calib (tools/gpu.sh calib).

    python tools/calib_summary.py gpurun_out [--out profiles/r02/fetch_calib.json]

factor = known bytes per launch / counter bytes per launch (counter in KiB), i.e. what a counter
value of that access pattern must be multiplied by to give bytes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import per_launch  # noqa: E402

ES_BYTES = 96 * 4
CODE_BYTES = 196684   # k_code symbol size (llvm-readelf -s on the gfx950 code object)
READS = {"k_read16": ("record", "16 B/lane streaming read"),
         "k_read4": ("record", "4 B/lane, partial waves (the wave kernel's record loads)"),
         "k_read8s": ("scalar", "8 B, one lane per env (per-env scalars)"),
         "k_readsec": ("line", "16 B of one 128-B line per env (fetch granularity: factor 1 = "
                               "whole 128-B lines; 0.5 = 64-B sectors, each counted as a half)")}
WRITES = {"k_write4": ("record", "4 B/lane, partial waves (the wave kernel's record stores)"),
          "k_write8s": ("scalar", "8 B, one lane per env (per-env scalars)"),
          "k_write4p": ("partial", "lines 0-1 whole, 48 of 128 B of line 2 (factor vs 304 B/env)")}


def main():
    base = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    res = {}
    for n in (4096, 1048576):
        known = {"record": n * ES_BYTES, "scalar": n * 8, "line": n * 128, "partial": n * 304}
        rows = {}
        for counter, tag, kernels in (("FETCH_SIZE", "calf", READS), ("WRITE_SIZE", "calw", WRITES)):
            d = os.path.join(base, f"{tag}_{n}")
            if not os.path.isdir(d):
                continue
            for k, (what, desc) in kernels.items():
                kib, cnt = per_launch(d, counter, k)
                b = kib * 1024.0
                rows[k] = {"counter": counter, "pattern": desc, "known_bytes": known[what],
                           "counter_bytes": round(b), "factor": round(known[what] / b, 3) if b else None,
                           "launches": cnt}
        d = os.path.join(base, f"calf_{n}")
        if os.path.isdir(d):
            try:   # fill traffic of a partly written line (0 if the L2 does not fill it)
                kib, cnt = per_launch(d, "FETCH_SIZE", "k_write4p")
                rows["k_write4p_fetch"] = {"counter": "FETCH_SIZE", "pattern": "reads caused by "
                                           "the partial-line store kernel", "counter_bytes": round(kib * 1024),
                                           "lines_per_launch": n, "launches": cnt}
            except SystemExit:
                pass
            try:
                kib, cnt = per_launch(d, "FETCH_SIZE", "k_code")
                known = 8 * CODE_BYTES   # each of the 8 XCDs' L2 fetches the code once
                rows["k_code"] = {"counter": "FETCH_SIZE", "pattern": f"instruction fetch of a "
                                  f"{CODE_BYTES}-B kernel, 2048 workgroups", "known_bytes": known,
                                  "counter_bytes": round(kib * 1024), "launches": cnt,
                                  "factor": round(known / (kib * 1024), 3) if kib else None}
            except SystemExit:
                pass
        res[str(n)] = rows
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
