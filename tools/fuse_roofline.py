#!/usr/bin/env python3
"""HBM roofline of the obs/reward fuse (north_star: "achieved HBM GB/s on the obs/reward fuse"):
RLTask.post_physics_step as ONE kernel (mi_task_post_step -> k_loco_post_tiled) at env counts
where the working set streams from HBM. Algorithmic bytes per env:
reads 4(13 + 3D + 6S + 1) + 16, writes 4(O + 3) + 16 — Humanoid 748 B, Ant 532 B.

usage: fuse_roofline.py [Task] [N,N,...] [launches]  -> one JSON line per N, and
gpurun_out/fuse_roofline_<task>.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def fuse_bytes(task) -> int:
    D, S, O = task.model.num_dof, task.model.num_sensors, task.num_observations
    return 4 * (13 + 3 * D + 6 * S + 1) + 16 + 4 * (O + 3) + 16


def kernel_label(n: int) -> str:
    """The kernel mi_task_post_step launches for n envs (mi_sim.hip): the pipelined kernel from two
    32-env tiles per resident workgroup up (resident = 256 CUs x 8 workgroups for Humanoid and Ant:
    253 VGPRs -> 2 waves / SIMD), else the one-tile kernel; MI_POST_TILE overrides."""
    var = os.environ.get("MI_POST_TILE", "32p")
    tiles = (n + 31) // 32
    if var == "32p" and tiles >= int(os.environ.get("MI_POST_PIPE_MIN", "2")) * 256 * 8:
        return "k_loco_post_pipe"
    return "k_loco_post_tiled<" + ("32s" if var == "32p" else var) + ">"


def measure(task_name: str, n: int, launches: int = 30, env=None) -> dict:
    import torch

    from omniisaacgymenvs_amd import native as N
    from omniisaacgymenvs_amd.utils.task_util import make_env

    own = env is None
    if own:
        env = make_env(task_name, num_envs=n, device="cuda:0", seed=3)
    t = env.task
    env.reset()
    h, s = t.get_robot().handle, t.get_robot().stream()
    args = (h, t.actions.data_ptr(), t.obs_buf.data_ptr(), t.rew_buf.data_ptr(), t.reset_buf.data_ptr(),
            t.progress_buf.data_ptr(), t.potentials.data_ptr(), t.prev_potentials.data_ptr(), s)
    for _ in range(3):
        N.check(N.lib().mi_task_post_step(*args), "mi_task_post_step")
    # HIP start / stop events carried by each launch's own dispatch (mi_sim_time_launches): the
    # kernel alone, no marker packets queued between launches (torch events around each launch
    # added ~4.5 us per 190-us launch)
    import ctypes as C
    N.check(N.lib().mi_sim_time_launches(h, 1, launches), "mi_sim_time_launches")
    for _ in range(launches):
        N.check(N.lib().mi_task_post_step(*args), "mi_task_post_step")
    buf = (C.c_float * launches)()
    nrec = C.c_int32(0)
    N.check(N.lib().mi_sim_launch_times(h, buf, launches, C.byref(nrec)), "mi_sim_launch_times")
    N.check(N.lib().mi_sim_time_launches(h, 0, 0), "mi_sim_time_launches")
    k = min(nrec.value, launches)
    if k == 0:
        raise RuntimeError("no timed launch recorded")
    ms = sum(buf[:k]) / k
    B = fuse_bytes(t)
    gbs = B * n / (ms * 1e-3) / 1e9
    label = t.get_robot().post_kernel()[0] or kernel_label(n)   # what mi_task_post_step launched
    if own:
        env.close()
    rec = {"kernel": label, "task": task_name, "num_envs": n, "kernel_ms": round(ms, 4),
           "algo_bytes_per_env": B, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 4)}
    # measured HBM bytes per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this kernel at
    # this env count, gfx950 read correction: tools/pmc_traffic.py), when committed
    tf = os.path.join(ROOT, "profiles", f"traffic_fuse_{task_name}.json")
    if os.path.exists(tf):
        with open(tf) as f:
            d = json.load(f)
        if int(d.get("num_envs", -1)) == n:
            rec["traffic"] = d["bytes_per_launch"]
            rec["traffic_per_env"] = round(d["bytes_per_launch"] / n, 1)
            rec["traffic_over_algo"] = round(d["bytes_per_launch"] / (B * n), 3)
            rec["traffic_source"] = f"profiles/traffic_fuse_{task_name}.json"
    return rec


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "Humanoid"
    sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [4096, 65536, 262144, 1048576]
    launches = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    out = []
    for n in sizes:
        rec = measure(task, n, launches)
        print(json.dumps(rec), flush=True)
        out.append(rec)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"fuse_roofline_{task.lower()}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
