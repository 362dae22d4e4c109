#!/usr/bin/env python3
"""Where the slowest waves of a fused env-step launch spend their time (diagnostic build only).

Loads libmi_sim_stamps.so (-DMI_STAMPS: every wave adds the s_memtime delta of each phase to its
own slot), runs fused Humanoid env steps and prints, over the waves of the measured launches, the
distribution of per-wave cycles and the per-phase means of the slowest 2 % of waves against the
median ones, with the per-wave row / contact statistics. MI_WAVE_PAIR=1 selects the paired
kernels (one slot per wave = two envs). Timers fence every phase: read shares, not absolutes.

usage: pair_tail.py [Task] [num_envs] [launches]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ["MI_SIM_LIB"] = os.environ.get("MI_STAMPS_LIB", os.path.join(ROOT, "omniisaacgymenvs_amd", "libmi_sim_stamps.so"))
from phase_stamps import PHASES  # noqa: E402

STATS = {15: "rows", 16: "batch>32", 17: "rows>64", 18: "batch>64", 19: "rows>lam", 20: "contacts",
         21: "rows>16", 22: "rows>24", 23: "rows>20"}


def main():
    import torch

    from omniisaacgymenvs_amd import native as N
    from omniisaacgymenvs_amd.utils.task_util import make_env

    task = sys.argv[1] if len(sys.argv) > 1 else "Humanoid"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    launches = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    solver = sys.argv[4] if len(sys.argv) > 4 else "config"
    ov = {"pgs": ["solver_type=0"], "tgs": ["solver_type=1"]}.get(solver, [])
    env = make_env(task, num_envs=n, device="cuda:0", seed=1, overrides=ov)
    lib = N.lib()
    lib.mi_debug_stamps_raw.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    pair = env.task.get_robot().sim_kernel_path()[0] == 2
    nw = n // 2 if pair else n
    g = torch.Generator(device="cuda:0").manual_seed(0)
    env.reset()
    buf = (C.c_ulonglong * (nw * 32))()
    rows = []
    for step in range(40 + launches):
        if step >= 40:
            torch.cuda.synchronize()
            assert lib.mi_debug_stamps_raw(buf, nw) == 0          # read-and-reset
            if step > 40:
                rows.append(np.ctypeslib.as_array(buf).reshape(nw, 32).copy())
        env.step(torch.rand((n, env.num_actions), device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    assert lib.mi_debug_stamps_raw(buf, nw) == 0
    rows.append(np.ctypeslib.as_array(buf).reshape(nw, 32).copy())
    env.close()
    a = np.concatenate(rows).astype(np.float64)          # [waves x launches, 32]
    phases = dict(PHASES)
    phases[5] = "P4a column loads + register LTDL"
    phases[4] = "P4b 1/D + factor publish"
    phases[11] = "P10 pgs: u update"
    phases[27] = "P10 set-up: wide Delassus rows / narrow row data"
    phases[28] = "P10 pgs: sweeps"
    phases[29] = "P10 wide: entry (P9 tail, syncs)"
    phases[30] = "P10 wide: J rows + v"
    phases[24] = "P10 narrow: J row + v"
    phases[25] = "P10 narrow: Delassus rows"
    ph = list(phases)
    tot = a[:, ph].sum(axis=1)
    order = np.argsort(tot)
    k = max(1, len(tot) // 50)
    slow, mid = order[-k:], order[len(order) // 2 - k // 2: len(order) // 2 + k // 2 + 1]
    out = {"task": task, "envs": n, "pair": pair, "waves": int(len(tot)),
           "wave_cycles": {q: float(np.quantile(tot, v)) for q, v in
                           (("p50", .5), ("p90", .9), ("p99", .99), ("max", 1.0))},
           "phases_slow2pct_vs_median": {phases[p]: [round(a[slow, p].mean()), round(a[mid, p].mean())] for p in ph},
           "stats_slow2pct_vs_median_per_substep": {STATS[s]: [round(a[slow, s].mean() / 2, 3), round(a[mid, s].mean() / 2, 3)]
                                                    for s in STATS}}
    out["w_rows_lds"] = float(a[0, 26]) / 2          # LDS W rows per env (the rest: the slab)
    top = order[-5:][::-1]
    out["slowest5"] = [{"cycles": round(tot[w]), "P10": [round(a[w, 29]), round(a[w, 30]), round(a[w, 27]), round(a[w, 28]),
                                                          round(a[w, 11])], "rows": a[w, 15] / 2,
                        "rows>lam": a[w, 19] / 2, "contacts": a[w, 20] / 2} for w in top]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
