#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ with the CPU oracle.

The reference has no tests and no vectors, and importing it is denied, so the
fixtures come from the build's own oracle. Each fixture records the model/config hashes and
the seed, so a change to the assets or the oracle is visible as a diff.

For each task: 256 envs of the composed task config, seed 42, GridCloner origins. Step 0 is
VecEnvRLGames.reset (reset_buf = 1, zero actions); steps 1..23 use U(-1, 1) actions drawn from
numpy's PCG64(seed) (Humanoids start to fall at step 17 under these actions, so the last steps
carry terminations and the re-initialisation of the reset envs). Task creation's post_reset (one reset_idx of every env) runs first.
Per step: the clamped obs, reward, reset / progress masks, potentials, the physics state, the
per-env reset counters (the Philox counter of the reset noise), the oracle's contact-decision
margins and, for a self-colliding model, the smallest self-pair surface gap (< contact_offset:
a self contact is active). Everything a device needs to restart from step k's state is stored,
so the GPU test can check every step from the fixture's own state (tests/test_golden.py).

    python tools/make_golden.py            # (re)write tests/golden/*.npz + manifest.json
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
TASKS = ("Cartpole", "Ant", "Humanoid")
N_ENVS, SEED, STEPS = 256, 42, 23
ASSETS = {"Cartpole": "cartpole.xml", "Ant": "ant.xml", "Humanoid": "humanoid.xml"}


def sha256(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def run(task: str):
    """Oracle rollout of the fixture; returns (arrays, meta)."""
    from oracle.oracle import OracleSim, make_buffers
    from omniisaacgymenvs_amd.robots.articulations import GridCloner
    from omniisaacgymenvs_amd.utils.config_utils.sim_config import SimConfig
    from omniisaacgymenvs_amd.utils.hydra_cfg.hydra_utils import compose
    from tests.helpers import task_params_from_cfg

    cfg = compose([f"task={task}", f"seed={SEED}", f"num_envs={N_ENVS}", "pipeline=cpu",
                   "sim_device=cpu", "rl_device=cpu"])
    sp = SimConfig(cfg).mi_sim_params(task)
    tp, model, keep = task_params_from_cfg(task)
    spacing = float(cfg["task"]["env"]["envSpacing"])
    origins = GridCloner(spacing).get_clone_positions(N_ENVS, 0, N_ENVS)
    orc = OracleSim(model, sp, N_ENVS, origins, seed=SEED)
    orc.configure(tp, keep=keep)
    b = make_buffers(N_ENVS, tp.num_obs, tp.num_actions)
    # task creation: post_reset() resets every env once (locomotion.py:147-171,
    # cartpole.py post_reset) before VecEnvRLGames.reset's reset step
    orc.reset_idx(np.arange(N_ENVS), b)
    b["reset"][:] = 1                                        # VecEnv.reset (rl_task.py:218-221)
    rng = np.random.Generator(np.random.PCG64(SEED))
    rec = {k: [] for k in ("actions", "obs", "rew", "reset", "progress", "pot", "prev", "root_pos",
                           "root_quat", "root_vel", "q", "qd", "reset_count", "margin", "self_gap")}
    for step in range(STEPS + 1):
        a = np.zeros((N_ENVS, tp.num_actions), np.float32) if step == 0 else \
            rng.uniform(-1.0, 1.0, (N_ENVS, tp.num_actions)).astype(np.float32)
        orc.env_step(a, 2, b)
        p, qt, v = orc.root_state()
        q, qd = orc.dof_state()
        gap = np.array([orc.self_min_gap(i) for i in range(N_ENVS)], np.float32) \
            if sp.enable_self_collisions else np.full(N_ENVS, np.inf, np.float32)
        for k, x in (("actions", a), ("obs", b["obs"]), ("rew", b["rew"]), ("reset", b["reset"]),
                     ("progress", b["progress"]), ("pot", b["pot"]), ("prev", b["prev"]),
                     ("root_pos", p), ("root_quat", qt), ("root_vel", v), ("q", q), ("qd", qd),
                     ("reset_count", orc.reset_count()), ("margin", orc.decision_margin()),
                     ("self_gap", gap)):
            rec[k].append(np.array(x, copy=True))
    arrays = {k: np.stack(v) for k, v in rec.items()}
    arrays["origins"] = origins
    meta = {"task": task, "num_envs": N_ENVS, "seed": SEED, "steps": STEPS + 1, "substeps": 2,
            "enable_self_collisions": int(sp.enable_self_collisions),
            "contact_offset": float(sp.contact_offset),
            # the contact / limit solver the fixture was stepped with (include/mi_sim.h)
            "solver_type": int(sp.solver_type), "solver": "TGS" if sp.solver_type == 1 else "PGS",
            "solver_iterations": int(sp.solver_iterations),
            "velocity_iterations": int(sp.velocity_iterations),
            "model_sha256": sha256(os.path.join(ROOT, "omniisaacgymenvs_amd", "robots", "assets",
                                                ASSETS[task])),
            "task_cfg_sha256": sha256(os.path.join(ROOT, "omniisaacgymenvs_amd", "cfg", "task",
                                                   f"{task}.yaml")),
            "generator": "tools/make_golden.py (oracle/oracle.c)"}
    return arrays, meta


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    manifest = {}
    for task in TASKS:
        arrays, meta = run(task)
        np.savez_compressed(os.path.join(GOLDEN, f"{task.lower()}_steps.npz"), **arrays)
        manifest[task] = meta
        print(task, {k: v.shape for k, v in arrays.items()})
    with open(os.path.join(GOLDEN, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
