#!/usr/bin/env python3
"""Backend cost of INTEGRATION.md path (A) — the reference's task code unchanged on top of the
ArticulationView tensor API — against path (B), the fused env step, on the same sim.

Path (A) per env-step, the backend calls the reference makes:
  pre_physics_step: set_joint_efforts(forces, indices=int32 arange)          (locomotion.py:111-114)
                    reset_idx of the envs due: set_joint_positions / velocities,
                    set_world_poses, set_velocities with int64 env ids       (locomotion.py:130-134)
  controlFrequencyInv = 2 physics substeps: World.step()                     (vec_env_rlgames.py:64-66)
  get_observations: get_world_poses, get_velocities, get_joint_positions,
                    get_joint_velocities, get_force_sensor_forces            (locomotion.py:81-89)
The reference's own torch task math (jit obs / reward / done) runs on top of these and is not
counted: it is the reference's code, unchanged. Resets: 1 % of the envs per step (about the
Humanoid reset rate under a random policy at 4096 envs).

usage: path_a_timing.py [Task] [num_envs] [steps] -> one JSON line (+ gpurun_out/path_a_<task>.json)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def measure(task_name: str = "Humanoid", n: int = 4096, steps: int = 200) -> dict:
    import torch

    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env(task_name, num_envs=n, device="cuda:0", seed=5)
    t, view, world = env.task, env.task.get_robot(), env._world
    env.reset()
    dev = "cuda:0"
    D = view.num_dof
    g = torch.Generator(device=dev).manual_seed(0)
    efforts = torch.rand((n, D), device=dev, generator=g) * 2 - 1
    all_i32 = torch.arange(n, dtype=torch.int32, device=dev)
    n_reset = max(1, n // 100)
    q0 = view.get_joint_positions()[:n_reset].clone()
    qd0 = torch.zeros_like(q0)
    pos0, rot0 = view.get_world_poses()
    pos0, rot0 = pos0[:n_reset].clone(), rot0[:n_reset].clone()
    vel0 = torch.zeros((n_reset, 6), device=dev)
    subs = t.control_frequency_inv

    def path_a(k):
        ids = (torch.arange(n_reset, device=dev, dtype=torch.int64) * 97 + k * 13) % n
        view.set_joint_positions(q0, indices=ids)
        view.set_joint_velocities(qd0, indices=ids)
        view.set_world_poses(pos0, rot0, indices=ids)
        view.set_velocities(vel0, indices=ids)
        view.set_joint_efforts(efforts, indices=all_i32)
        for _ in range(subs):
            world.step()
        out = (view.get_world_poses(clone=False), view.get_velocities(clone=False),
               view.get_joint_positions(clone=False), view.get_joint_velocities(clone=False),
               view._physics_view.get_force_sensor_forces())
        return out

    def timed(fn, k0):
        for k in range(20):
            fn(k0 + k)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        for k in range(steps):
            fn(k0 + 20 + k)
        b.record()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3, a.elapsed_time(b) / steps

    ms_a_wall, ms_a_dev = timed(path_a, 0)
    acts = torch.rand((8, n, t.num_actions), device=dev, generator=g) * 2 - 1
    ms_b_wall, ms_b_dev = timed(lambda k: env.step(acts[k % 8]), 1000)
    rec = {"task": task_name, "num_envs": n, "steps": steps, "resets_per_step": n_reset,
           "path_a_backend_ms_per_step": round(ms_a_wall, 4), "path_a_device_ms_per_step": round(ms_a_dev, 4),
           "path_a_launches_per_step": 5 + subs + 5,
           "path_b_fused_ms_per_step": round(ms_b_wall, 4), "path_b_device_ms_per_step": round(ms_b_dev, 4),
           "note": "path A excludes the reference's torch task math (its own code, unchanged)"}
    env.close()
    return rec


def main():
    task_name = sys.argv[1] if len(sys.argv) > 1 else "Humanoid"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    rec = measure(task_name, n, steps)
    print(json.dumps(rec), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"path_a_{task_name.lower()}.json"), "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
