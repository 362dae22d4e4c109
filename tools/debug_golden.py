#!/usr/bin/env python3
"""Diagnostic: device env vs a golden fixture, per step and per field (tests/test_golden.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from omniisaacgymenvs_amd.utils.task_util import make_env
    from tests.helpers import task_params_from_cfg

    for task in sys.argv[1:] or ["Cartpole", "Ant"]:
        with np.load(os.path.join(ROOT, "tests", "golden", f"{task.lower()}_steps.npz")) as z:
            g = {k: z[k] for k in z.files}
        env = make_env(task, num_envs=32, device="cuda:0", seed=42)
        t = env.task
        a, _, _ = task_params_from_cfg(task)
        b = t.task_params()
        for f, _ in a._fields_:
            va, vb = getattr(a, f), getattr(b, f)
            va = list(va) if hasattr(va, "__len__") else va
            vb = list(vb) if hasattr(vb, "__len__") else vb
            if va != vb:
                print(task, "task param differs:", f, va, vb)
        obs = env.reset()["obs"]
        view = t.get_robot()
        for k in range(g["obs"].shape[0]):
            if k:
                obs = env.step(torch.tensor(g["actions"][k], device="cuda:0"))[0]["obs"]
            torch.cuda.synchronize()
            q = view.get_joint_positions().cpu().numpy()
            d_obs = np.abs(obs.cpu().numpy() - g["obs"][k]).max(axis=0)
            print(task, k, "obs max diff per column", np.round(d_obs, 5).tolist()[:16],
                  "q", float(np.abs(q - g["q"][k]).max()),
                  "rew", float(np.abs(t.rew_buf.cpu().numpy() - g["rew"][k]).max()),
                  "reset eq", bool(np.array_equal(t.reset_buf.cpu().numpy(), g["reset"][k])))
        env.close()


if __name__ == "__main__":
    main()
