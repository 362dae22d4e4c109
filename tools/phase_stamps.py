#!/usr/bin/env python3
"""Per-phase cycle breakdown of the wavefront-per-env substep (diagnostic build only).

Loads libmi_sim_stamps.so (built with -DMI_STAMPS: every workgroup adds the s_memtime delta of
each phase to a device counter), runs fused env steps and prints the mean cycles per env-substep
of each phase over ALL envs. Timers add a barrier-like fence at every phase boundary, so read
the SHARES, not the absolute time."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MI_SIM_LIB"] = os.environ.get("MI_STAMPS_LIB", os.path.join(ROOT, "omniisaacgymenvs_amd", "libmi_sim_stamps.so"))

PHASES = {0: "load", 1: "P1 fk+link dynamics", 2: "P2 composite", 3: "P3 crba", 4: "P4 ltdl+publish",
          5: "P5 1/D (runtime path)", 6: "P8 contacts", 7: "P9 J build", 8: "P9 solves",
          9: "P9 u* + limit rows", 10: "P9 row filing", 11: "P10 pgs", 12: "P11 sensors+integrate",
          13: "task pre-step (per env-step)", 14: "task post-step (per env-step)"}


def main():
    import torch

    from omniisaacgymenvs_amd import native as N
    from omniisaacgymenvs_amd.utils.task_util import make_env

    task = sys.argv[1] if len(sys.argv) > 1 else "Humanoid"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    env = make_env(task, num_envs=n, device="cuda:0", seed=1)
    lib = N.lib()
    lib.mi_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    g = torch.Generator(device="cuda:0").manual_seed(0)
    env.reset()
    buf = (C.c_ulonglong * 32)()
    for step in range(60):
        if step == 20:
            torch.cuda.synchronize()
            assert lib.mi_debug_stamps(buf, 32) == 0   # read-and-reset: drop the warm-up
        env.step(torch.rand((n, env.num_actions), device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    assert lib.mi_debug_stamps(buf, 32) == 0
    env.close()
    cnt = max(1, buf[31])
    # per env-substep; the task phases (once per env-step) are amortised over its substeps
    per = {PHASES[k]: buf[k] / cnt for k in PHASES}
    tot = sum(per.values())
    print(json.dumps({"task": task, "envs": n, "substeps_measured": cnt,
                      "cycles_per_env_substep": {k: round(v, 1) for k, v in per.items()}}))
    for k, v in per.items():
        print(f"{k:26s} {v:9.0f}  {100.0 * v / tot:5.1f}%")
    print(f"{'total (1 env-substep)':26s} {tot:9.0f}")
    stats = {"mean rows": buf[15] / cnt, "frac rows > LDS W rows": buf[16] / cnt,
             "frac rows > 64": buf[17] / cnt, "frac solve vectors > 64": buf[18] / cnt,
             "frac rows > LDS J rows": buf[19] / cnt, "mean contacts": buf[20] / cnt,
             "frac rows > 16": buf[21] / cnt, "frac rows > 24": buf[22] / cnt,
             "frac rows > 32": buf[23] / cnt, "frac rows > 40": buf[24] / cnt,
             "frac rows > 48": buf[25] / cnt, "LDS W rows": buf[26] / cnt, "LDS J rows": buf[27] / cnt}
    print(json.dumps({"row_stats_per_env_substep": {k: round(v, 4) for k, v in stats.items()}}))


if __name__ == "__main__":
    main()
