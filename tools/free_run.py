#!/usr/bin/env python3
"""Free-running device vs oracle rollout statistics (test infrastructure: the oracle is the
checker). Both start from the identical post-reset state (same seeds, the oracle synced once)
and then run `steps` fused env steps with the same Philox actions and NO re-sync. Contact-rich
dynamics are chaotic, so individual envs diverge; what must agree is the distribution:
per-step reward samples, completed-episode lengths and the per-step reset rate
(locomotion.py:257-321, cartpole.py:143-162).

usage: free_run.py [Task] [num_envs] [steps]  -> one JSON line
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ks_stat(a, b):
    """Two-sample Kolmogorov-Smirnov statistic sup |F_a - F_b|."""
    import numpy as np

    a, b = np.sort(a), np.sort(b)
    x = np.concatenate([a, b])
    fa = np.searchsorted(a, x, side="right") / a.size
    fb = np.searchsorted(b, x, side="right") / b.size
    return float(np.abs(fa - fb).max())


def free_run(task_name: str, n: int, steps: int, seed: int = 13) -> dict:
    import numpy as np
    import torch

    from omniisaacgymenvs_amd import native as N
    from omniisaacgymenvs_amd.utils.task_util import make_env
    from oracle.oracle import lib as orc_lib
    from tests.helpers import oracle_twin, task_buffers

    env = make_env(task_name, num_envs=n, device="cuda:0", seed=seed)
    task = env.task
    view = task.get_robot()
    env.reset()
    torch.cuda.synchronize()
    orc_lib().orc_set_threads(min(16, os.cpu_count() or 1))
    orc = oracle_twin(env, seed=seed)
    b = task_buffers(env)
    rew_d, rew_o, rst_d, rst_o, len_d, len_o = [], [], [], [], [], []
    for k in range(steps):
        a = torch.empty((n, env.num_actions), device="cuda:0")
        N.check(N.lib().mi_fill_uniform(view.handle, a.data_ptr(), env.num_actions, seed, k, -1.0, 1.0,
                                        view.stream()))
        _, r, d, _ = env.step(a)
        orc.env_step(a.cpu().numpy(), task.control_frequency_inv, b)
        torch.cuda.synchronize()
        dd = d.cpu().numpy().astype(bool)
        od = b["reset"].astype(bool)
        rew_d.append(r.cpu().numpy())
        rew_o.append(b["rew"].copy())
        rst_d.append(dd.mean())
        rst_o.append(od.mean())
        len_d.append(task.progress_buf.cpu().numpy()[dd])
        len_o.append(b["progress"][od])
    orc.close()
    env.close()
    rd, ro = np.concatenate(rew_d), np.concatenate(rew_o)
    ld, lo = np.concatenate(len_d), np.concatenate(len_o)
    rsd, rso = np.array(rst_d), np.array(rst_o)
    w = max(1, steps // 10)   # reset rate over windows of steps
    win = lambda x: x[: steps // w * w].reshape(-1, w).mean(axis=1)
    return {
        "task": task_name, "envs": n, "steps": steps,
        "reward_ks": ks_stat(rd, ro), "reward_mean": [float(rd.mean()), float(ro.mean())],
        "reward_q": {f"q{p}": [float(np.quantile(rd, p / 100)), float(np.quantile(ro, p / 100))]
                     for p in (5, 50, 95)},
        "episodes": [int(ld.size), int(lo.size)],
        "episode_len_ks": ks_stat(ld, lo) if ld.size and lo.size else None,
        "episode_len_mean": [float(ld.mean()) if ld.size else None, float(lo.mean()) if lo.size else None],
        "reset_rate_window_maxdiff": float(np.abs(win(rsd) - win(rso)).max()),
        "reset_rate_mean": [float(rsd.mean()), float(rso.mean())],
        "per_env_identical_frac_last_step": float(np.mean(rew_d[-1] == rew_o[-1])),
    }


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "Humanoid"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    print(json.dumps(free_run(task, n, steps)), flush=True)


if __name__ == "__main__":
    main()
