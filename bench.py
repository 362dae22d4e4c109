#!/usr/bin/env python3
"""Env-steps/s of the hot path (physics + obs + reward + done + reset) — BASELINE.json metric.

One "step" = VecEnvRLGames.step on a batch of U(-1,1) actions (scripts/random_policy.py:57),
i.e. one fused mi_env_step launch: mask-driven reset_idx, efforts, controlFrequencyInv=2
physics substeps, observations, reward, done, obs clamp. Action batches are pre-generated in
HBM (Philox) before the timed region.

N=1: `python bench.py` (Humanoid, 4096 envs). N>1: `python bench.py --gpus N` starts
torch.distributed.run itself (or the driver launches it that way): one rank per GPU, each rank
owns 4096 envs of a global grid (weak scaling). Every rank writes its rollout slab (done, rew,
obs) in place from the fused launch and gathers it to the learner rank (rank 0) over RCCL once
per horizon (HumanoidPPO.yaml:66, 32 steps), asynchronously while the next horizon steps. The
timed window starts a fresh horizon and ends by gathering any partial one, so every window
holds at least one complete gather whatever --steps is.

Prints ONE JSON line (rank 0). `roofline` is for the dominant kernel — the launch the fused
step runs, named in the line (Humanoid / Ant: k_env_step_pair<Tgs<TopoCT<Robot*>>> under the
reference's TGS solver, k_env_step_pair<TopoCT<Robot*>> under PGS, two envs per wavefront;
Cartpole: k_env_step) — timed with HIP events carried by its own dispatch on the
stream it is launched on; `cpu_baseline` times the CPU oracle (the build's C restatement; the
reference's PhysX CPU path is closed and absent) on host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic HBM bytes per env-step of a fully fused step (SURVEY §8d / BASELINE.md)
ALGO_BYTES = {"Humanoid": 920, "Ant": 552, "Cartpole": 80}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BASELINE_METRIC = "env-steps/s (physics+obs+reward) Humanoid 4096 envs @1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--task", default="Humanoid", choices=["Humanoid", "Ant", "Cartpole"])
    ap.add_argument("--num-envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--gather-every", type=int, default=32, help="rollout horizon (N>1)")
    ap.add_argument("--cpu-seconds", type=float, default=30.0,
                    help="CPU baseline sample budget (split over the 1 / 4 / all-thread legs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-side", action="store_true", help="skip the Cartpole / Ant side runs")
    ap.add_argument("--modular", action="store_true", help="method-by-method path, not fused")
    ap.add_argument("--solver", choices=["config", "tgs", "pgs"], default="config",
                    help="contact / limit solver: the task config's (cfg/config.yaml solver_type: 1 = "
                         "TGS, the reference's default) or an override (A/B)")
    ap.add_argument("--events-apart", action="store_true",
                    help="diagnostic: time the window without kernel events, events in a second window")
    ap.add_argument("--fuse-envs", type=int, default=1048576,
                    help="envs of the obs/reward-fuse HBM roofline side measurement (0: skip)")
    return ap.parse_args(argv)


def launch_ranks(args) -> int:
    """`bench.py --gpus N` outside torch.distributed.run: start it as a CHILD process with N ranks
    (nothing here has touched the GPU) and return its exit code."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
           *sys.argv[1:]]
    return subprocess.call(cmd)


class ShardLoop:
    """The timed loop of one rank: step the env shard, write each step's (obs, rew, done) into the
    rollout slab row, gather every full horizon to the learner asynchronously.

    ``env``: a VecEnvRLGames (or any object with ``fused`` and ``step(actions[, out])``);
    ``actions``: a pool of action batches indexed by global step; ``rollout``: a RolloutGather or
    None (single process, nothing to gather)."""

    def __init__(self, env, actions, rollout=None, horizon: int = 32):
        self.env, self.actions, self.rollout = env, actions, rollout
        self.H = horizon if rollout is None else min(horizon, rollout.H)
        self.h = 0          # next row of the current horizon
        self.gathering = True
        self.ev = None      # (starts, ends, every, k0): kernel events on steps k0, k0 + every, ...

    def step(self, k: int):
        a = self.actions[k % len(self.actions)]
        if self.ev is not None:
            self.env.kernel_events = self.ev[:2] if (k - self.ev[3]) % self.ev[2] == 0 else None
        r = self.rollout
        if r is None:
            return self.env.step(a)[0]
        if self.env.fused:
            obs = self.env.step(a, out=r.slot(self.h))[0]
        else:
            obs, rew, done, _ = self.env.step(a)
            r.record(self.h, obs["obs"], rew, done)
        self.h += 1
        if self.h == self.H:
            if self.gathering:
                r.gather(async_op=True)
            self.h = 0
        return obs

    def flush(self) -> None:
        """Gather the partial horizon in progress (its first h rows), so no step of a window is
        left un-gathered."""
        if self.rollout is not None and self.h > 0:
            if self.gathering:
                self.rollout.gather(async_op=True, rows=self.h)
            self.h = 0

    def window(self, start: int, steps: int, sync=lambda: None, barrier=lambda: None,
               gathering: bool = True) -> dict:
        """Time `steps` steps from a fresh horizon; the window closes after the last gather it
        issued has completed (barrier + device sync on both sides)."""
        r = self.rollout
        self.flush()
        if r is not None:
            r.wait()
        sync(); barrier(); sync()
        self.gathering = gathering
        g0 = r.gathers if r is not None else 0
        b0 = r.bytes_sent if r is not None else 0
        t0 = time.perf_counter()
        for k in range(steps):
            self.step(start + k)
        self.flush()
        if r is not None:
            r.wait()   # every collective issued inside the window completes inside it
        sync(); barrier(); sync()
        el = time.perf_counter() - t0
        self.gathering = True
        return {"elapsed": el, "gathers": (r.gathers - g0) if r is not None else 0,
                "bytes": (r.bytes_sent - b0) if r is not None else 0}


def _cpu_share() -> int:
    ncpu = os.cpu_count() or 1
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    # the GPU box exposes the whole machine's CPUs but grants this job a share
    # (OMP_NUM_THREADS=16 there); never oversubscribe that share
    return min(ncpu, int(os.environ.get("OMP_NUM_THREADS", ncpu)))


WARM, TIMED, RUNS = 200, 2000, 5   # BASELINE.md / SURVEY §8(d) protocol


def cpu_baseline(task_name: str, env, seconds: float) -> dict:
    """The CPU baselines, each on BASELINE.md's protocol (200 warm-up env-steps, then the median
    of 5 runs of 2000 timed env-steps), on a bounded sample so the whole leg stays within
    `seconds`:
      * the C oracle's fused step of the metric's task (oracle/oracle.c, the build's CPU
        restatement: the reference's PhysX-CPU path is closed and absent) at 1, 4 and all granted
        threads, with the env count scaled per thread count to the time budget;
      * config 1 (Cartpole, 16 envs): the product's CPU pipeline (make_env(device="cpu"): the
        reference's Cartpole task as torch ops on CPU tensors, as its pipeline=cpu runs it) and
        the C oracle, 1 thread each."""
    import numpy as np
    from oracle.oracle import OracleSim, lib as orc_lib, make_buffers

    task = env.task
    view = task.get_robot()
    ncpu = _cpu_share()
    sweep = sorted({1, min(4, ncpu), ncpu})
    rng = np.random.default_rng(0)
    per_leg = 0.8 * seconds / len(sweep)

    def protocol(step_fn, n):
        for k in range(WARM):
            step_fn(k)
        runs = []
        for _ in range(RUNS):
            t0 = time.perf_counter()
            for k in range(TIMED):
                step_fn(k)
            runs.append(n * TIMED / (time.perf_counter() - t0))
        return statistics.median(runs)

    results = {}
    for threads in sweep:
        orc_lib().orc_set_threads(threads)

        def make(n):
            orc = OracleSim(task.model, view.sim_params, n, task.env_pos_cpu[:n], seed=42)
            orc.configure(task.task_params(), keep=task)
            return orc, make_buffers(n, task.num_observations, task.num_actions)
        # calibrate: cost of one env-step per env at this thread count, then size the sample
        orc, b = make(threads)
        acts = rng.uniform(-1, 1, (8, threads, task.num_actions)).astype(np.float32)
        t0 = time.perf_counter()
        for k in range(20):
            orc.env_step(acts[k % 8], task.control_frequency_inv, b)
        per_env_step = (time.perf_counter() - t0) / (20 * threads)
        orc.close()
        total = WARM + RUNS * TIMED
        n = int(per_leg / (total * per_env_step)) // threads * threads
        n = max(threads, min(n, 256, task.num_envs))
        orc, b = make(n)
        acts = rng.uniform(-1, 1, (8, n, task.num_actions)).astype(np.float32)
        v = protocol(lambda k: orc.env_step(acts[k % 8], task.control_frequency_inv, b), n)
        orc.close()
        results[threads] = (v, n)
    v1, n1 = results[1]
    orc_lib().orc_set_threads(1)
    c1 = c1t = None
    try:
        import torch
        from omniisaacgymenvs_amd.robots.articulations import GridCloner
        from tests.helpers import sim_params, task_params_from_cfg
        tp1, m1, _ = task_params_from_cfg("Cartpole")
        sp1 = sim_params(rest_offset=0.001)
        orc = OracleSim(m1, sp1, 16, GridCloner(4.0).get_clone_positions(16), seed=42)
        orc.configure(tp1)
        b1 = make_buffers(16, tp1.num_obs, tp1.num_actions)
        a1 = rng.uniform(-1, 1, (8, 16, tp1.num_actions)).astype(np.float32)
        c1 = {"value": round(protocol(lambda k: orc.env_step(a1[k % 8], 2, b1), 16), 1),
              "unit": "env-steps/s", "cores": 1, "kind": "port",
              "sample": "Cartpole 16 envs, 200 warm-up + median of 5 x 2000 env-steps (BASELINE.md "
                        "protocol), C oracle fused step (2 substeps)"}
        orc.close()
        threads0 = torch.get_num_threads()
        torch.set_num_threads(1)
        try:
            from omniisaacgymenvs_amd.utils.task_util import make_env
            ce = make_env("Cartpole", num_envs=16, device="cpu", seed=42)
            ce.reset()
            at = [torch.from_numpy(a1[k]) for k in range(8)]
            c1t = {"value": round(protocol(lambda k: ce.step(at[k % 8]), 16), 1), "unit": "env-steps/s",
                   "cores": 1, "kind": "product",
                   "sample": "Cartpole 16 envs on the product's CPU pipeline (make_env(device='cpu'): "
                             "CartpoleTask's cartpole.py:80-162 torch ops over robots/cpu_cartpole.py, "
                             "VecEnvRLGames.step method by method, Philox resets), 200 warm-up + median "
                             "of 5 x 2000 env-steps, 1 torch thread"}
            ce.close()
        finally:
            torch.set_num_threads(threads0)
    except Exception as e:   # noqa: BLE001 - the side leg must not sink the bench line
        c1 = c1 or {"error": str(e)}
        c1t = c1t or {"error": str(e)}
    return {
        "value": round(v1, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
        "sample": f"{task_name} {n1} envs (sample sized to the time budget), {WARM} warm-up + median of "
                  f"{RUNS} x {TIMED} env-steps (BASELINE.md protocol), 1 thread; oracle/oracle.c fused step "
                  f"(2 substeps). Algorithm: the oracle's dense CRBA + Cholesky articulated step (device: "
                  f"tree LTDL), same contacts / limits / PGS and task math",
        "threads_sweep": {str(t): round(v[0], 1) for t, v in results.items()},
        "threads_sweep_envs": {str(t): v[1] for t, v in results.items()},
        "config1_cartpole16": c1,
        "config1_cpu_torch": c1t,
    }


def kernel_name(view, task) -> str:
    """Name of the fused env-step kernel this configuration launches."""
    from omniisaacgymenvs_amd import native as N
    path, topo, _ = view.sim_kernel_path()
    if path in (1, 2) and task.task_params().task_kind != N.MI_TASK_CARTPOLE:   # wave / paired path
        t = {0: "TopoRuntime", 1: "TopoCT<RobotHumanoid>", 2: "TopoCT<RobotAnt>"}.get(topo, str(topo))
        if view.sim_params.solver_type == N.MI_SOLVER_TGS:   # the Tgs<> instantiation (with_topo)
            t = f"Tgs<{t}>"
        return ("k_env_step_wave<" if path == 1 else "k_env_step_pair<") + t + ">"
    return "k_env_step"


TIME_EVERY = 4   # every 4th fused launch of a timed window carries the kernel-timing events


def launch_times_ms(view, cap: int):
    """Mean duration (ms) of the fused launches timed since mi_sim_time_launches (dispatch-carried
    HIP events), then timing off; None when no launch was timed."""
    import ctypes as C
    from omniisaacgymenvs_amd import native as NL
    buf = (C.c_float * cap)()
    n = C.c_int32(0)
    NL.check(NL.lib().mi_sim_launch_times(view.handle, buf, cap, C.byref(n)), "mi_sim_launch_times")
    NL.check(NL.lib().mi_sim_time_launches(view.handle, 0, 0), "mi_sim_time_launches")
    k = min(n.value, cap)
    return sum(buf[:k]) / k if k else None


def read_traffic(task_name: str):
    """HBM bytes per launch from the committed PMC passes (profiles/traffic_<task>.json), if any:
    (instruction fetch at face value + data reads x2 + WRITE_SIZE, per the calibration of
    tools/fetch_calib.hip and the env-count sweep of tools/traffic_split.py; FETCH_SIZE as
    reported + WRITE_SIZE; the split by source)."""
    p = os.path.join(ROOT, "profiles", f"traffic_{task_name}.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        split = {k: d[k] for k in ("instruction_fetch_bytes", "data_read_bytes", "write_bytes_at_n")
                 if k in d}
        split["source"] = (f"committed PMC profile profiles/traffic_{task_name}.json "
                           f"({d.get('profile', 'rocprofv3 FETCH_SIZE / WRITE_SIZE env-count sweep')}), "
                           "not measured in this run")
        return d.get("bytes_per_launch"), d.get("bytes_per_launch_uncorrected"), split
    return None, None, {}


def action_pool(view, n, A, seed, device, pool=16):
    import torch
    from omniisaacgymenvs_amd import native as N

    actions = torch.empty((pool, n, A), device=device)
    for k in range(pool):
        N.check(N.lib().mi_fill_uniform(view.handle, actions[k].data_ptr(), A, seed, k, -1.0, 1.0,
                                        view.stream()))
    return actions


def solver_overrides(solver: str) -> list:
    return {"config": [], "tgs": ["solver_type=1"], "pgs": ["solver_type=0"]}[solver]


def solver_label(view) -> str:
    p = view.sim_params
    return (f"TGS ({p.solver_iterations} position / {p.velocity_iterations} velocity iterations)"
            if p.solver_type == 1 else f"PGS ({p.solver_iterations} sweeps)")


def side_run(task_name: str, n: int, steps: int = 200, warmup: int = 30, solver: str = "config") -> dict:
    """BASELINE configs 2 and 3 (Cartpole / Ant at 4096 envs on 1 GPU): the same fused step,
    kernel time from HIP events on the launch stream, algorithmic HBM fraction."""
    import torch
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env(task_name, num_envs=n, device="cuda:0", seed=42, overrides=solver_overrides(solver))
    task = env.task
    view = task.get_robot()
    actions = action_pool(view, n, task.num_actions, 42, "cuda:0")
    env.reset()
    for k in range(warmup):
        env.step(actions[k % len(actions)])
    from omniisaacgymenvs_amd import native as NL
    NL.check(NL.lib().mi_sim_time_launches(view.handle, TIME_EVERY, steps), "mi_sim_time_launches")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(actions[k % len(actions)])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kms = launch_times_ms(view, steps)
    ach = ALGO_BYTES[task_name] * n / (kms * 1e-3) / 1e9
    # the same steps replayed from a captured HIP graph (as the PPO rollout runs them,
    # rlg/a2c_continuous.py graph_rollout): no per-step Python / launch overhead
    G = len(actions)
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(graph):
        for k in range(G):
            env.step(actions[k])
    for _ in range(2):
        graph.replay()
    reps = max(1, steps // G)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        graph.replay()
    torch.cuda.synchronize()
    el_g = time.perf_counter() - t0
    out = {"workload": f"{task_name} {n} envs, fused env step", "kernel": kernel_name(view, task),
           "solver": solver_label(view),
           "value": round(n * steps / el, 1), "unit": "env-steps/s", "ms_per_step": round(el / steps * 1e3, 4),
           "kernel_ms": round(kms, 4), "achieved": round(ach, 3), "unit_bw": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 6), "algo_bytes_per_env": ALGO_BYTES[task_name],
           "lds_bytes_per_env": view.sim_kernel_path()[2], "nan_resets": view.nan_count(),
           "graph_replay": {"value": round(n * reps * G / el_g, 1), "ms_per_step": round(el_g / (reps * G) * 1e3, 4),
                            "steps": reps * G, "steps_per_graph": G}}
    env.close()
    return out


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if env_world is not None and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torch.distributed.run (even one rank) the RCCL process group and the rollout gather run
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    device = f"cuda:{local}"

    from omniisaacgymenvs_amd.utils.distributed import RolloutGather
    from omniisaacgymenvs_amd.utils.task_util import make_env

    n_local = args.num_envs
    env = make_env(args.task, num_envs=n_local, device=device, seed=args.seed,
                   env_id_offset=rank * n_local, global_num_envs=world * n_local,
                   overrides=solver_overrides(args.solver))
    if args.modular:
        env.use_fused(False)
    task = env.task
    view = task.get_robot()
    A, O = task.num_actions, task.num_observations
    actions = action_pool(view, n_local, A, args.seed, device)
    env.reset()
    rollout = RolloutGather(args.gather_every, n_local, O, device, world, mode="gather", dst=0) \
        if distributed else None
    loop = ShardLoop(env, actions, rollout, args.gather_every)
    sync = torch.cuda.synchronize
    barrier = dist.barrier if distributed else (lambda: None)

    for k in range(args.warmup):
        loop.step(k)
    # kernel time, live, over the timed region: HIP start / stop events carried by the dispatch of
    # every TIME_EVERY-th fused launch (hipExtLaunchKernelGGL inside libmi_sim,
    # mi_sim_time_launches), on the launch stream. Torch event records around every launch slowed
    # the window by 2.5 % (Humanoid) / 6.9 % (Ant), dispatch events on every launch by 1.7 % /
    # 4.3 % (`--events-apart`); on every 4th launch the window is within noise.
    from omniisaacgymenvs_amd import native as NL
    if args.events_apart:
        # diagnostic: the same window plain, with torch events around every launch, and with
        # the dispatch-carried events
        win = loop.window(args.warmup, args.steps, sync, barrier)
        s_all = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
        e_all = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
        env._ev_i = 0
        loop.ev = (s_all, e_all, 1, args.warmup + args.steps)
        win_ev = loop.window(args.warmup + args.steps, args.steps, sync, barrier)
        loop.ev = None
        env.kernel_events = None
        torch_ms = sum(a.elapsed_time(b) for a, b in zip(s_all, e_all)) / args.steps
        k0 = args.warmup + 2 * args.steps
        NL.check(NL.lib().mi_sim_time_launches(view.handle, 1, args.steps), "mi_sim_time_launches")
        win_x = loop.window(k0, args.steps, sync, barrier)
        ext_ms = launch_times_ms(view, args.steps)
        NL.check(NL.lib().mi_sim_time_launches(view.handle, TIME_EVERY, args.steps), "mi_sim_time_launches")
        win_s = loop.window(k0 + args.steps, args.steps, sync, barrier)
        s_ms = launch_times_ms(view, args.steps)
        print(json.dumps({"events_apart": {
            f"ms_per_step_dispatch_events_every_{TIME_EVERY}": round(win_s["elapsed"] / args.steps * 1e3, 4),
            f"kernel_ms_dispatch_events_every_{TIME_EVERY}": round(s_ms, 4) if s_ms else None,
            "ms_per_step_plain": round(win["elapsed"] / args.steps * 1e3, 4),
            "ms_per_step_torch_events": round(win_ev["elapsed"] / args.steps * 1e3, 4),
            "kernel_ms_torch_events": round(torch_ms, 4),
            "ms_per_step_dispatch_events": round(win_x["elapsed"] / args.steps * 1e3, 4),
            "kernel_ms_dispatch_events": round(ext_ms, 4) if ext_ms else None}}))
    else:
        if env.fused:
            NL.check(NL.lib().mi_sim_time_launches(view.handle, TIME_EVERY, args.steps), "mi_sim_time_launches")
        win = loop.window(args.warmup, args.steps, sync, barrier)
    elapsed = win["elapsed"]
    kernel_ms = launch_times_ms(view, args.steps) if env.fused else None
    gather_info = None
    if distributed:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # the same window without gathers (exposed gather time = difference), and one
        # synchronous horizon gather on its own
        nog = loop.window(args.warmup + args.steps, args.steps, sync, barrier, gathering=False)
        t = torch.tensor([nog["elapsed"]], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        nog_el = float(t.item())
        sync(); barrier(); sync()
        t0 = time.perf_counter()
        rollout.gather(async_op=False)
        sync(); barrier(); sync()
        g_ms = (time.perf_counter() - t0) * 1e3
        gather_info = {"collective": "gather to rank 0 (learner), RCCL" if dist.get_backend() == "nccl"
                       else f"gather to rank 0, {dist.get_backend()}",
                       "horizon": loop.H, "gathers_in_window": win["gathers"],
                       "gather_bytes_per_rank": win["bytes"] // max(1, win["gathers"]),
                       "bytes_per_rank_in_window": win["bytes"],
                       "window_ms_no_gather": round(nog_el * 1e3, 3),
                       "exposed_gather_ms": round((elapsed - nog_el) * 1e3, 3),
                       "standalone_horizon_gather_ms": round(g_ms, 3)}
    total_env_steps = world * n_local * args.steps
    value = total_env_steps / elapsed
    nan = view.nan_count()

    out = None
    if rank == 0:
        roof = None
        if kernel_ms:
            algo = ALGO_BYTES[args.task] * n_local
            achieved = algo / (kernel_ms * 1e-3) / 1e9
            traffic, traffic_raw, split = read_traffic(args.task)
            roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                    "kernel": kernel_name(view, task), "kernel_ms": round(kernel_ms, 4),
                    "algo_bytes_per_launch": algo,
                    "limiter": "latency: dependent per-env chains at the resident-wave count "
                               "(DESIGN.md §2, §6); HBM is not the limiter at 4096 envs"}
            if traffic:
                roof["traffic_gbs"] = round(traffic / (kernel_ms * 1e-3) / 1e9, 3)
            if traffic_raw:
                roof["traffic_uncorrected_fetch"] = traffic_raw
            if split:
                roof["traffic_split"] = split
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
                       "solver": solver_label(view),
                       "lds_bytes_per_env": view.sim_kernel_path()[2],
                       "parallelism": f"env-shard x{world}" + (
                           f" + async RCCL gather of the rollout slab to the learner rank every "
                           f"{loop.H} steps" if distributed else "")},
            "roofline": roof,
            "nan_resets": nan,
        }
        if gather_info:
            out["rollout_gather"] = gather_info
    if not distributed and env.fused:
        # the same workload replayed from a captured HIP graph (16 steps per graph, as the PPO
        # rollout runs it): what the step costs without per-step Python / launch overhead
        G = len(actions)
        graph = torch.cuda.CUDAGraph()
        sync()
        with torch.cuda.graph(graph):
            for k in range(G):
                env.step(actions[k])
        graph.replay()
        reps = max(1, args.steps // G)
        sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            graph.replay()
        sync()
        el_g = time.perf_counter() - t0
        out["graph_replay"] = {"value": round(n_local * reps * G / el_g, 1),
                               "ms_per_step": round(el_g / (reps * G) * 1e3, 4), "steps": reps * G,
                               "note": "informational; `value` is the eager per-step loop"}
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if world == 1 and not args.no_side and args.task == "Humanoid":
            out["side_configs"] = [side_run("Cartpole", 4096, solver=args.solver),
                                   side_run("Ant", 4096, solver=args.solver)]
        if world == 1 and args.fuse_envs > 0 and args.task != "Cartpole":
            # north_star: achieved HBM GB/s of the obs/reward fuse (RLTask.post_physics_step as ONE
            # streaming kernel, the method-by-method path) where its working set streams from HBM
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from fuse_roofline import measure
            out["obs_reward_fuse"] = measure(args.task, args.fuse_envs, 30)
        if world == 1 and not args.no_side and args.task != "Cartpole":
            # INTEGRATION.md path (A): the reference's own task code over the ArticulationView
            # tensor API (indexed reset scatters, set_joint_efforts, controlFrequencyInv x
            # World.step, the five getters) on the same task and env count
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from path_a_timing import measure as path_a
            out["path_a"] = path_a(args.task, n_local, 100)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.task, env, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
