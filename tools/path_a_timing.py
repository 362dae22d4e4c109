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
Resets follow the envs' own terminations (root z below terminationHeight or the episode
length, locomotion.py:257-268) with the reference's reset_idx draws (:116-145) in torch, so
the state distribution matches the fused path's; the rest of the reference's torch task math
(jit observations / reward) runs on top of these and is not counted: it is the reference's
code, unchanged. Actions U(-1, 1) as in scripts/random_policy.py:57.

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
    all_i32 = torch.arange(n, dtype=torch.int32, device=dev)
    subs = t.control_frequency_inv
    # the reference's reset_idx inputs (locomotion.py:116-145): initial root pose, dof limits
    pos0, rot0 = view.get_world_poses()
    pos0 = t._env_pos + torch.tensor(t._spawn_translation, device=dev)
    rot0 = torch.tensor([1.0, 0.0, 0.0, 0.0], device=dev).repeat(n, 1)
    lim = view.get_dof_limits()[0]
    lo, hi = lim[:, 0], lim[:, 1]
    reset_buf = torch.zeros(n, dtype=torch.int64, device=dev)
    progress = torch.zeros(n, dtype=torch.int64, device=dev)
    term_h, max_len = float(t.termination_height), float(t._max_episode_length)

    ev = []   # (start, stop) HIP events around each backend call when timing the backend alone
    cache = {}  # the reference ops alone: every backend call replaced by its last result
    host = {}   # host seconds per backend call (name -> [total, calls]) when timing the host side
    timing_host = False

    def backend(fn, *a, **kw):
        if timing_host:
            t0 = time.perf_counter()
            r = fn(*a, **kw)
            h = host.setdefault(getattr(fn, "__name__", str(fn)), [0.0, 0])
            h[0] += time.perf_counter() - t0
            h[1] += 1
            return r
        if ref_only:
            key = getattr(fn, "__name__", str(fn))
            if key not in cache:
                cache[key] = fn(*a, **kw)
            return cache[key]
        if timing_backend:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **kw)
            e1.record()
            ev.append((e0, e1))
            return r
        return fn(*a, **kw)

    def path_a(k):
        # pre_physics_step (locomotion.py:103-114): nonzero() (host sync) -> reset_idx's four
        # indexed scatters, then the efforts
        ids = reset_buf.nonzero(as_tuple=False).squeeze(-1)
        if len(ids) > 0:
            m = len(ids)
            q = torch.clamp(torch.rand((m, D), device=dev, generator=g) * 0.4 - 0.2, lo, hi)
            qd = torch.rand((m, D), device=dev, generator=g) * 0.2 - 0.1
            pr, rr, z6 = pos0[ids], rot0[ids], torch.zeros((m, 6), device=dev)
            backend(view.set_joint_positions, q, indices=ids)
            backend(view.set_joint_velocities, qd, indices=ids)
            backend(view.set_world_poses, pr, rr, indices=ids)
            backend(view.set_velocities, z6, indices=ids)
            reset_buf[ids] = 0
            progress[ids] = 0
        forces = (torch.rand((n, D), device=dev, generator=g) * 2 - 1) * t.joint_gears * t.power_scale
        backend(view.set_joint_efforts, forces, indices=all_i32)
        for _ in range(subs):
            if not ref_only:
                world.step()
        out = (backend(view.get_world_poses, clone=False), backend(view.get_velocities, clone=False),
               backend(view.get_joint_positions, clone=False), backend(view.get_joint_velocities, clone=False),
               backend(view._physics_view.get_force_sensor_forces))
        # is_done's state-driving part (locomotion.py:257-268): fallen or timed out -> reset
        progress.add_(1)
        reset_buf.copy_(((out[0][0][:, 2] < term_h) | (progress >= max_len - 1)).to(torch.int64))
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

    timing_backend = ref_only = False
    ms_a_wall, ms_a_dev = timed(path_a, 0)
    # the same loop with no backend work at all (physics, getters and setters skipped; the getters
    # hand back their previous tensors): the reference's own torch ops + nonzero() sync
    ref_only = True
    ms_ref_wall, _ = timed(path_a, 3000)
    ref_only = False
    # the same loop with events around the backend calls: the backend's own device time per step
    # (the deferred physics launch is issued inside get_world_poses, so it is included)
    timing_backend = True
    ev.clear()
    timed(path_a, 5000)
    torch.cuda.synchronize()
    backend_ms = sum(a.elapsed_time(b) for a, b in ev[-(len(ev) * steps // (steps + 20)):]) / steps
    timing_backend = False
    # host cost of each backend call (ctypes, argument checks, launch enqueue): while the host
    # is inside these the GPU can sit idle (the event intervals above count that idle time)
    timing_host = True
    timed(path_a, 7000)
    timing_host = False
    host_us = {k: round(1e6 * v[0] / v[1], 2) for k, v in host.items()}
    host_us_step = round(1e6 * sum(v[0] for v in host.values()) / (steps + 20), 2)
    acts = torch.rand((8, n, t.num_actions), device=dev, generator=g) * 2 - 1
    ms_b_wall, ms_b_dev = timed(lambda k: env.step(acts[k % 8]), 1000)
    rec = {"task": task_name, "num_envs": n, "steps": steps,
           "path_a_ms_per_step": round(ms_a_wall, 4), "path_a_device_ms_per_step": round(ms_a_dev, 4),
           "path_a_backend_device_ms_per_step": round(backend_ms, 4),
           "backend_host_us_per_call": host_us, "backend_host_us_per_step": host_us_step,
           "reference_ops_only_ms_per_step": round(ms_ref_wall, 4),
           "path_a_launches_per_step": "1 physics (deferred substeps; the paired kernel writes the five getters' "
                                       "state mirrors itself) + efforts + 4 reset scatters when any env is due",
           "path_b_fused_ms_per_step": round(ms_b_wall, 4), "path_b_device_ms_per_step": round(ms_b_dev, 4),
           "note": "path A: the reference's call sequence incl. its reset / termination torch ops and "
                   "nonzero() host sync; jit observation / reward math excluded. backend_device: "
                   "the libmi_sim calls alone (HIP events around each: includes the GPU's idle time while "
                   "the host enqueues the call; the kernels alone: rocprofv3 kernel trace); backend_host: "
                   "host time inside each call; reference_ops_only: the same loop with "
                   "every backend call skipped (the reference's own torch ops and host sync)"}
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
