#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (results .db): per kernel name the dispatch count,
mean duration, grid / workgroup, resources, and the mean of every PMC counter per dispatch;
for the wave env-step kernel also the derived occupancy figures DESIGN.md quotes.

usage: rocpd_summary.py <dir-or-db> [kernel-substring]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_env_step_wave"
    db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, name, duration, grid_x, workgroup_x, lds_size, scratch_size, "
                     "vgpr_count, accum_vgpr_count, sgpr_count from kernels").fetchall()
    by = defaultdict(list)
    for r in rows:
        by[r[1]].append(r)
    pmc = defaultdict(lambda: defaultdict(list))
    for did, name, val in c.execute("select dispatch_id, counter_name, counter_value from pmc_events"):
        pmc[did][name].append(val)
    for name, rs in sorted(by.items(), key=lambda kv: -sum(r[2] for r in kv[1])):
        if sub not in name:
            continue
        n = len(rs)
        dur = sum(r[2] for r in rs) / n / 1e3
        r0 = rs[0]
        print(f"{name[:90]}\n  dispatches {n}  mean {dur:.2f} us  grid {r0[3]} wg {r0[4]}  lds {r0[5]} B  "
              f"scratch {r0[6]}  vgpr {r0[7]} agpr {r0[8]} sgpr {r0[9]}")
        tot = defaultdict(float)
        for r in rs:
            for k, v in pmc.get(r[0], {}).items():
                tot[k] += sum(v)
        mean = {k: v / n for k, v in tot.items()}
        for k in sorted(mean):
            print(f"  {k:24s} {mean[k]:.6g}")
        if "SQ_WAVE_CYCLES" in mean:
            wc = mean["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if k in mean:
                    print(f"  {k:24s} {100 * mean[k] / wc:5.1f} % of wave cycles")
            if "SQ_WAVES" in mean and "SQ_BUSY_CYCLES" in mean:
                waves = mean["SQ_WAVES"]
                # SQ_WAVE_CYCLES in quad-cycles summed over waves; kernel cycles from the duration at
                # 2.4 GHz (GRBM_GUI_ACTIVE in its own pass when collected)
                kcyc = dur * 1e-6 * 2.4e9
                print(f"  mean wave lifetime     {4 * wc / waves:.4g} cycles")
                print(f"  resident waves / CU    {4 * wc / kcyc / 256:.2f} (mean over the dispatch, 2.4 GHz)")


if __name__ == "__main__":
    main()
