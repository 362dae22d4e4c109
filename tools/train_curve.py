#!/usr/bin/env python3
"""The reference's training schedule end to end (VERDICT r3 "next" #3): cfg/train/<Task>PPO.yaml
as shipped (HumanoidPPO.yaml:58-59 max_epochs 1000, AntPPO.yaml:59-60 max_epochs 500; 4096
envs, horizon 32, minibatch 32768, 5 mini-epochs, adaptive LR) through the same calls
scripts/rlgames_train.py:67-84 makes (make_env -> A2CAgent.train), on one GPU.

    python tools/train_curve.py --task Ant [--epochs 500] [--out gpurun_out/train_curve_ant.jsonl]

Writes one JSON object per epoch (mean episode reward / length over the last 100 finished
episodes, as rl_games' game meters report them, frames, lr, kl, fps) and a final summary line;
the committed curves live in profiles/r04/."""
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
    ap.add_argument("--epochs", type=int, default=None, help="default: the PPO yaml's max_epochs")
    ap.add_argument("--num-envs", type=int, default=None)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env(args.task, num_envs=args.num_envs, device="cuda:0", seed=args.seed)
    register_env("rlgpu", lambda **kw: env)
    params = env.task_cfg["train"]["params"]
    epochs = int(args.epochs or params["config"]["max_epochs"])
    out = args.out or os.path.join(ROOT, "gpurun_out", f"train_curve_{args.task.lower()}.jsonl")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    agent = A2CAgent(RLGPUEnv("rlgpu", env.num_envs), params,
                     run_dir=os.path.join("/tmp", f"train_curve_{args.task}"))
    agent.max_epochs = epochs
    t0 = time.perf_counter()
    rows = []

    def log(_msg):
        st = agent.stats
        row = {"epoch": st["epoch"], "frames": st["frames"], "mean_reward": round(st["mean_rewards"], 4),
               "mean_length": round(st["mean_lengths"], 2), "games": st["games"],
               "lr": st.get("lr"), "kl": st.get("kl"), "a_loss": st.get("a_loss"), "c_loss": st.get("c_loss"),
               "grad_scale": agent.scaler.get_scale() if agent.mixed_precision else None,
               "fps_total": round(st["fps_total"], 1),
               "wall_s": round(time.perf_counter() - t0, 3)}
        rows.append(row)
        f.write(json.dumps(row) + "\n")
        if st["epoch"] % 25 == 0 or st["epoch"] == 1:
            print(json.dumps(row), flush=True)

    with open(out, "w") as f:
        agent.train(max_epochs=epochs, log=log)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    first = next((r for r in rows if r["games"] > 0), rows[0])
    best = max(rows, key=lambda r: r["mean_reward"])
    print(json.dumps({
        "summary": f"{args.task} PPO, reference schedule", "epochs": len(rows),
        "num_envs": env.num_envs, "frames": rows[-1]["frames"], "wall_s": round(wall, 2),
        "frames_per_s": round(rows[-1]["frames"] / wall, 1),
        "first_reward": first["mean_reward"], "first_reward_epoch": first["epoch"],
        "final_reward": rows[-1]["mean_reward"], "final_length": rows[-1]["mean_length"],
        "best_reward": best["mean_reward"], "best_epoch": best["epoch"], "curve": out}), flush=True)
    env.close()


if __name__ == "__main__":
    main()
