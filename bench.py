#!/usr/bin/env python3
"""Env-steps/s of the hot path (physics + obs + reward + done + reset) — BASELINE.json metric.

One "step" = VecEnvRLGames.step on a batch of U(-1,1) actions (scripts/random_policy.py:57),
i.e. one fused mi_env_step launch: mask-driven reset_idx, efforts, controlFrequencyInv=2
physics substeps, observations, reward, done, obs clamp. Action batches are pre-generated in
HBM (Philox) before the timed region.

N=1: `python bench.py` (Humanoid, 4096 envs). N>1: launched by torch.distributed.run, one
rank per GPU; each rank owns 4096 envs of a global grid (weak scaling) and every
--gather-every steps the rollout slab (obs, rew, done), which the fused launch writes in
place, is all-gathered over RCCL asynchronously while the next horizon steps.

Prints ONE JSON line (rank 0). `roofline` is for the dominant kernel (k_env_step), timed
with HIP events on the stream it is launched on; `cpu_baseline` times the CPU oracle (the
build's C restatement; the reference's PhysX CPU path is closed and absent) on host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic HBM bytes per env-step of a fully fused step (SURVEY §8d / BASELINE.md)
ALGO_BYTES = {"Humanoid": 920, "Ant": 552, "Cartpole": 80}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--task", default="Humanoid", choices=["Humanoid", "Ant", "Cartpole"])
    ap.add_argument("--num-envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--gather-every", type=int, default=32, help="rollout gather period (N>1)")
    ap.add_argument("--cpu-seconds", type=float, default=30.0,
                    help="CPU baseline sample budget (split over the 1 / 4 / all-thread legs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--modular", action="store_true", help="method-by-method path, not fused")
    ap.add_argument("--fuse-envs", type=int, default=1048576,
                    help="envs of the obs/reward-fuse HBM roofline side measurement (0: skip)")
    return ap.parse_args()


def cpu_baseline(task_name: str, env, seconds: float) -> dict:
    """Time the CPU oracle's fused env step on a bounded sample of the same workload."""
    import numpy as np
    from oracle.oracle import OracleSim, lib as orc_lib, make_buffers

    task = env.task
    n = min(task.num_envs, 256 if task_name != "Cartpole" else 4096)
    origins = task.env_pos_cpu[:n]
    view = task.get_robot()
    results = {}
    ncpu = os.cpu_count() or 1
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    # the GPU box exposes the whole machine's CPUs but grants this job a share
    # (OMP_NUM_THREADS=16 there); never oversubscribe that share
    ncpu = min(ncpu, int(os.environ.get("OMP_NUM_THREADS", ncpu)))
    sweep = sorted({1, min(4, ncpu), ncpu})
    rng = np.random.default_rng(0)
    for threads in sweep:
        orc_lib().orc_set_threads(threads)
        orc = OracleSim(task.model, view.sim_params, n, origins, seed=42)
        orc.configure(task.task_params(), keep=task)
        b = make_buffers(n, task.num_observations, task.num_actions)
        acts = rng.uniform(-1, 1, (8, n, task.num_actions)).astype(np.float32)
        for k in range(3):  # warm-up (first resets)
            orc.env_step(acts[k % 8], task.control_frequency_inv, b)
        steps, t0 = 0, time.perf_counter()
        budget = seconds / len(sweep)
        while True:
            orc.env_step(acts[steps % 8], task.control_frequency_inv, b)
            steps += 1
            el = time.perf_counter() - t0
            if el >= budget and steps >= 3:
                break
        results[threads] = (n * steps / el, steps, el)
        orc.close()
    v1, steps1, el1 = results[1]
    return {
        "value": round(v1, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
        "sample": f"{task_name} {n} envs x {steps1} env-steps ({el1:.1f}s), oracle/oracle.c fused "
                  f"step (2 substeps), 1 thread",
        "threads_sweep": {str(t): round(v[0], 1) for t, v in results.items()},
    }


def kernel_name(view, task) -> str:
    from omniisaacgymenvs_amd import native as N
    """Name of the fused env-step kernel this configuration launches."""
    path, topo, _ = view.sim_kernel_path()
    if path == 1 and task.task_params().task_kind != N.MI_TASK_CARTPOLE:   # wave path
        return "k_env_step_wave<" + {0: "TopoRuntime", 1: "TopoCT<RobotHumanoid>",
                                     2: "TopoCT<RobotAnt>"}.get(topo, str(topo)) + ">"
    return "k_env_step"


BASELINE_METRIC = "env-steps/s (physics+obs+reward) Humanoid 4096 envs @1/2/4/8 MI355X"


def read_traffic(task_name: str):
    """HBM bytes per launch from the committed PMC pass (profiles/traffic_<task>.json), if any."""
    p = os.path.join(ROOT, "profiles", f"traffic_{task_name}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f).get("bytes_per_launch")
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    device = f"cuda:{local}"

    from omniisaacgymenvs_amd import native as N
    from omniisaacgymenvs_amd.utils.task_util import make_env

    n_local = args.num_envs
    env = make_env(args.task, num_envs=n_local, device=device, seed=args.seed,
                   env_id_offset=rank * n_local, global_num_envs=world * n_local)
    if args.modular:
        env.use_fused(False)
    task = env.task
    view = task.get_robot()
    A, O = task.num_actions, task.num_observations
    pool = 16
    actions = torch.empty((pool, n_local, A), device=device)
    for k in range(pool):
        N.check(N.lib().mi_fill_uniform(view.handle, actions[k].data_ptr(), A, args.seed, k, -1.0, 1.0,
                                        view.stream()))
    env.reset()
    from omniisaacgymenvs_amd.utils.distributed import RolloutGather

    rollout = RolloutGather(args.gather_every, n_local, O, device, world) if world > 1 else None

    def one_step(k):
        if rollout is None:
            return env.step(actions[k % pool])[0]
        # the launch writes obs/rew/done straight into the rollout slab row (no copies); a full
        # horizon is all-gathered asynchronously over RCCL while the next one steps
        h = k % args.gather_every
        if env.fused:
            obs = env.step(actions[k % pool], out=rollout.slot(h))[0]
        else:
            obs, rew, done, _ = env.step(actions[k % pool])
            rollout.record(h, obs["obs"], rew, done)
        if h == args.gather_every - 1:
            rollout.gather(async_op=True)
        return obs

    for k in range(args.warmup):
        one_step(k)
    if rollout is not None:
        rollout.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # kernel events around every fused launch inside the timed region (same stream)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    env.kernel_events = (starts, ends)
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(args.warmup + k)
    if rollout is not None:
        rollout.wait()   # every collective issued inside the window completes inside it
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    env.kernel_events = None
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / args.steps if env.fused else None
    total_env_steps = world * n_local * args.steps
    value = total_env_steps / elapsed
    nan = view.nan_count()

    out = None
    if rank == 0:
        roof = None
        if kernel_ms:
            achieved = ALGO_BYTES[args.task] * n_local / (kernel_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                    "traffic": read_traffic(args.task), "kernel": kernel_name(view, task),
                    "kernel_ms": round(kernel_ms, 4),
                    "algo_bytes_per_launch": ALGO_BYTES[args.task] * n_local}
        out = {
            "metric": BASELINE_METRIC if args.task == "Humanoid" else
                      f"env-steps/s (physics+obs+reward) {args.task} {args.num_envs} envs (side run)",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: U(-1,1) Philox actions, random-init resets (no policy)",
            "config": {"workload": f"{args.task} {n_local} envs/GPU x {world} GPU(s), fused env step "
                                   f"(controlFrequencyInv=2 substeps @ dt=0.0083)",
                       "task": args.task, "num_envs_per_gpu": n_local, "global_envs": world * n_local,
                       "substeps": task.control_frequency_inv, "path": "fused" if env.fused else "modular",
                       "lds_bytes_per_env": view.sim_kernel_path()[2],
                       "parallelism": f"env-shard x{world}" + (f" + async RCCL all_gather of the rollout slab every {args.gather_every} steps" if world > 1 else "")},
            "roofline": roof,
            "nan_resets": nan,
        }
        if world == 1 and args.fuse_envs > 0 and args.task != "Cartpole":
            # north_star: achieved HBM GB/s of the obs/reward fuse (RLTask.post_physics_step as ONE
            # streaming kernel, the method-by-method path) where its working set streams from HBM
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from fuse_roofline import measure
            out["obs_reward_fuse"] = measure(args.task, args.fuse_envs, 30)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.task, env, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
