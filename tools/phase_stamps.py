#!/usr/bin/env python3
"""Per-phase cycle breakdown of the wavefront-per-env substep (diagnostic build only).

Loads libmi_sim_stamps.so (built with -DMI_STAMPS: s_memtime at each phase boundary of
workgroup 7's last substep), runs a few fused env steps and prints the share of each phase.
Stamps forbid overlaps the real kernel has: read the SHARES, never the absolute time."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MI_SIM_LIB"] = os.path.join(ROOT, "omniisaacgymenvs_amd", "libmi_sim_stamps.so")

PHASES = ["load", "P1 fk/levels", "P2 composite", "P3 crba", "P4 ltdl", "P5 L^-1", "P6 Minv",
          "P7 u*", "P8 contacts", "P9 rows J/W", "P10 pgs", "P11 sensors+integrate"]


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
    out = {}
    for step in range(40):
        env.step(torch.rand((n, env.num_actions), device="cuda:0", generator=g) * 2 - 1)
        if step >= 20 and step % 5 == 0:
            torch.cuda.synchronize()
            buf = (C.c_ulonglong * 32)()
            assert lib.mi_debug_stamps(buf, 32) == 0
            st = list(buf)[:13]
            d = [st[k + 1] - st[k] for k in range(12)]
            tot = st[12] - st[0]
            out[step] = {"total_cycles": tot, **{PHASES[k]: d[k] for k in range(12)}}
    env.close()
    print(json.dumps(out))
    last = out[max(out)]
    tot = last["total_cycles"]
    for k in PHASES:
        print(f"{k:24s} {last[k]:9d}  {100.0 * last[k] / tot:5.1f}%")
    print(f"{'total (1 substep)':24s} {tot:9d}")


if __name__ == "__main__":
    main()
