#!/usr/bin/env python3
"""Diagnostic: wave path vs one-lane-per-env path for ONE physics substep from identical
state (efforts held); prints the max difference of every state quantity."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from omniisaacgymenvs_amd.utils.task_util import make_env

    task = sys.argv[1] if len(sys.argv) > 1 else "Ant"
    n = 64
    ea = make_env(task, num_envs=n, device="cuda:0", seed=3)
    os.environ["MI_SIM_PATH"] = "thread"
    eb = make_env(task, num_envs=n, device="cuda:0", seed=3)
    del os.environ["MI_SIM_PATH"]
    va, vb = ea.task.get_robot(), eb.task.get_robot()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    eff = (torch.rand((n, va.num_dof), device="cuda:0", generator=g) * 2 - 1) * 5
    for view in (va, vb):
        view.set_joint_efforts(eff)
    for sub in range(3):
        for view in (va, vb):
            view.sim_step(1)
        torch.cuda.synchronize()
        pa, ra = va.get_world_poses()
        pb, rb = vb.get_world_poses()
        qa, qb = va.get_joint_positions(), vb.get_joint_positions()
        wa, wb = va.get_joint_velocities(), vb.get_joint_velocities()
        la, lb = va.get_velocities(), vb.get_velocities()
        sa, sb = va._physics_view.get_force_sensor_forces(), vb._physics_view.get_force_sensor_forces()
        print(f"substep {sub}: pos {float((pa - pb).abs().max()):.3e} rot {float((ra - rb).abs().max()):.3e} "
              f"q {float((qa - qb).abs().max()):.3e} qd {float((wa - wb).abs().max()):.3e} "
              f"rootvel {float((la - lb).abs().max()):.3e} sens {float((sa - sb).abs().max()):.3e}")
        print("   rootvel env0 wave  ", la[0].cpu().numpy())
        print("   rootvel env0 thread", lb[0].cpu().numpy())
        print("   qd env0 wave  ", wa[0].cpu().numpy())
        print("   qd env0 thread", wb[0].cpu().numpy())
        # re-align
        vb.set_world_poses(pa, ra)
        vb.set_velocities(la)
        vb.set_joint_positions(qa)
        vb.set_joint_velocities(wa)


if __name__ == "__main__":
    main()
