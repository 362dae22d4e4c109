#!/usr/bin/env python3
"""End-to-end PPO training throughput over the hot path: the reference
configuration cfg/train/<Task>PPO.yaml (Humanoid: 4096 envs, horizon 32, minibatch 32768,
5 mini-epochs, MLP 400-200-100, fp16 mixed precision), random init, synthetic episodes.

    python tools/bench_train.py [--task Humanoid] [--epochs 6] [--warmup 3] [--no-graph]

Prints one JSON line: frames/s of the whole epoch (rollout + update, rl_games' "fps total"),
of the rollout alone ("fps step and policy inference") and the per-epoch split."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Humanoid")
    ap.add_argument("--num-envs", type=int, default=None)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true", help="eager rollout and eager updates")
    ap.add_argument("--no-graph-update", action="store_true", help="eager (sync-free) updates only")
    ap.add_argument("--no-fused-policy", action="store_true",
                    help="rollout policy as torch modules + sampling kernel (A/B of mi_rl_policy_step)")
    args = ap.parse_args()
    import torch

    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env(args.task, num_envs=args.num_envs, device="cuda:0", seed=42)
    register_env("rlgpu", lambda **kw: env)
    params = env.task_cfg["train"]["params"]
    params["config"]["graph_rollout"] = not args.no_graph
    params["config"]["graph_update"] = not (args.no_graph or args.no_graph_update)
    params["config"]["fused_policy"] = not args.no_fused_policy
    n = env.num_envs
    agent = A2CAgent(RLGPUEnv("rlgpu", n), params, run_dir=os.path.join("/tmp", "bench_train"))
    agent.env_reset()
    for _ in range(args.warmup):
        agent.train_epoch()
    torch.cuda.synchronize()
    play = upd = 0.0
    t0 = time.perf_counter()
    for _ in range(args.epochs):
        st = agent.train_epoch()
        play += st["play_time"]
        upd += st["update_time"]
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    frames = agent.batch_size * args.epochs
    c = params["config"]
    print(json.dumps({
        "metric": f"PPO training frames/s ({args.task}, rl_games a2c_continuous semantics)",
        "task": args.task, "num_envs": n, "horizon": agent.horizon,
        "minibatch": agent.minibatch_size, "mini_epochs": agent.mini_epochs,
        "mixed_precision": agent.mixed_precision, "graph_rollout": agent.graph is not None,
        "graph_update": len(agent.upd_graphs) > 0, "fused_policy": agent.fused_policy is not None,
        "units": params["network"]["mlp"]["units"], "epochs": args.epochs,
        "fps_total": round(frames / wall, 1), "fps_step_inference": round(frames / play, 1),
        "ms_per_epoch": round(1e3 * wall / args.epochs, 3),
        "ms_rollout": round(1e3 * play / args.epochs, 3), "ms_update": round(1e3 * upd / args.epochs, 3),
        "mean_reward_last": round(st["mean_rewards"], 3), "lr": st["lr"],
        "lr_schedule": c.get("lr_schedule"),
    }))
    env.close()


if __name__ == "__main__":
    main()
