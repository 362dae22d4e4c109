#!/usr/bin/env python3
"""Dump a short fused rollout (obs, rew, reset per step) to gpurun_out/<tag>.npz, for bit-level
comparison of two builds of libmi_sim.so (MI_SIM_LIB=...) on identical inputs.

usage: dump_rollout.py <tag> [Task] [num_envs] [steps]
       dump_rollout.py --compare <tagA> <tagB>
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "gpurun_out")


def dump(tag, task="Humanoid", n=4096, steps=6):
    import numpy as np
    import torch

    from omniisaacgymenvs_amd import native as N
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env(task, num_envs=n, device="cuda:0", seed=3)
    view = env.task.get_robot()
    env.reset()
    obs, rew, rst = [], [], []
    for k in range(steps):
        a = torch.empty((n, env.num_actions), device="cuda:0")
        N.check(N.lib().mi_fill_uniform(view.handle, a.data_ptr(), env.num_actions, 42, k, -1.0, 1.0,
                                        view.stream()))
        o, r, d, _ = env.step(a)
        obs.append(o["obs"].cpu().numpy())
        rew.append(r.cpu().numpy())
        rst.append(d.cpu().numpy())
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"{tag}.npz"), obs=np.stack(obs), rew=np.stack(rew), reset=np.stack(rst))
    env.close()


def compare(a, b):
    import numpy as np

    A = np.load(os.path.join(OUT, f"{a}.npz"))
    B = np.load(os.path.join(OUT, f"{b}.npz"))
    for k in range(A["obs"].shape[0]):
        d = np.abs(A["obs"][k] - B["obs"][k]).max(axis=1)
        bad = np.nonzero(d > 0)[0]
        print(f"step {k}: {bad.size} envs differ; max {d.max():.3g}; first {bad[:12].tolist()} "
              f"worst {np.argsort(-d)[:5].tolist()} {np.sort(d)[::-1][:5].tolist()}")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        args = sys.argv[2:]
        dump(sys.argv[1], *(args[:1]), *[int(x) for x in args[1:]])
