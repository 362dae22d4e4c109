#!/usr/bin/env python3
"""Device-vs-oracle error distribution of the fused env step from identical state (the
full-size parity test's setting, without the pass/fail): per env the max |obs - obs_oracle|
and |rew - rew_oracle| over each step, summarised as quantiles, and the worst envs with their
oracle decision margins. Test infrastructure (imports the oracle as the checker).

usage: parity_stats.py [Task] [num_envs] [steps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _ratio_above(err, sens, far, base):
    import numpy as np

    if base is None:
        return None
    m = far & (err > base)
    return float((err[m] / np.maximum(sens[m], 1e-6)).max()) if m.any() else 0.0


def main():
    import numpy as np
    import torch

    from omniisaacgymenvs_amd import native as N
    from omniisaacgymenvs_amd.utils.task_util import make_env
    from oracle.oracle import lib as orc_lib
    from tests.helpers import oracle_sensitivity, oracle_twin, sync_oracle, task_buffers
    from tests import parity_bounds as PB

    task_name = sys.argv[1] if len(sys.argv) > 1 else "Humanoid"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    solver = sys.argv[4] if len(sys.argv) > 4 else "config"
    env = make_env(task_name, num_envs=n, device="cuda:0", seed=3,
                   overrides={"pgs": ["solver_type=0"], "tgs": ["solver_type=1"]}.get(solver, []))
    task = env.task
    view = task.get_robot()

    def acts(k):
        a = torch.empty((n, env.num_actions), device="cuda:0")
        N.check(N.lib().mi_fill_uniform(view.handle, a.data_ptr(), env.num_actions, 42, k, -1.0, 1.0,
                                        view.stream()))
        return a

    env.reset()
    for k in range(3):
        env.step(acts(k))
    torch.cuda.synchronize()
    orc_lib().orc_set_threads(min(16, os.cpu_count() or 1))
    orc = oracle_twin(env, seed=3)
    sync_oracle(env, orc)
    D, S = task.model.num_dof, task.model.num_sensors
    if task_name == "Cartpole":
        groups = {"obs": slice(0, 4)}
    else:
        groups = {"root": slice(0, 12), "dof_pos": slice(12, 12 + D), "dof_vel": slice(12 + D, 12 + 2 * D),
                  "sensors": slice(12 + 2 * D, 12 + 2 * D + 6 * S), "actions": slice(12 + 2 * D + 6 * S, None)}
    gerr = {g: [] for g in list(groups) + ["rew"]}
    gsens = {g: [] for g in list(groups) + ["rew"]}
    errs, margins, senss, pmargins = [], [], [], []
    grel = {g: [] for g in groups}
    gmag = {g: [] for g in groups}
    potmag = []
    rew_refs = []
    probe_sens = {}
    n_probes = int(os.environ.get("PARITY_PROBES", "0")) or PB.SENS_PROBES
    widen_steps = []
    for k in range(3, 3 + steps):
        b = task_buffers(env)
        a = acts(k)
        # oracle-side conditioning of this step (tests/helpers.py oracle_sensitivity)
        pp = []
        sg, sr, _ = oracle_sensitivity(env, 3, a.cpu().numpy(), task.control_frequency_inv, b, groups,
                                       probes=n_probes, per_probe=pp)
        for j, (og, rg) in enumerate(pp):
            for g in groups:
                probe_sens.setdefault(f"{g}_p{j}", []).append(og[g].astype(np.float32))
            probe_sens.setdefault(f"rew_p{j}", []).append(rg.astype(np.float32))
        for g in groups:
            gsens[g].append(sg[g])
        gsens["rew"].append(sr)
        senss.append(np.maximum(np.max(np.stack(list(sg.values())), axis=0), sr))
        o, r, d, _ = env.step(a)
        torch.cuda.synchronize()
        orc.env_step(a.cpu().numpy(), task.control_frequency_inv, b)
        od = np.abs(o["obs"].cpu().numpy() - b["obs"])
        rd = np.abs(r.cpu().numpy() - b["rew"])
        for g, sl in groups.items():
            gerr[g].append(od[:, sl].max(axis=1))
            # mixed abs / rel error per entry: |d| / max(1, |oracle value|)
            grel[g].append((od[:, sl] / np.maximum(1.0, np.abs(b["obs"][:, sl]))).max(axis=1))
            gmag[g].append(np.abs(b["obs"][:, sl]).max(axis=1))
        potmag.append(np.maximum(np.abs(b["pot"]), np.abs(b["prev"])))
        gerr["rew"].append(rd)
        rew_refs.append(np.asarray(b["rew"], np.float64).copy())
        e = np.maximum(od.max(axis=1), rd)
        errs.append(e)
        margins.append(orc.decision_margin().copy())
        pmargins.append(orc.projection_margin().copy())
        if task_name != "Cartpole":   # the bounded check of tests/parity_bounds.py, reported per step
            ev = PB.evaluate(PB.bounds_key(task_name, env.task.get_robot().sim_params.solver_type), groups, o["obs"].cpu().numpy(), r.cpu().numpy(), b["obs"], b["rew"],
                             margins[-1], sens=senss[-1],
                             pot=np.maximum(np.abs(b["pot"]), np.abs(b["prev"])))
            need_b = np.concatenate([ev["bound"][g][ev["needed_widening"][g]] for g in ev["err"]])
            widen_steps.append({
                "step": k, "envs_needing_allowance": int(ev["any_needed"].sum()),
                "frac": float(ev["any_needed"].mean()), "widest_bound_applied": ev["widest_applied"],
                "bounds_applied": sorted(float(x) for x in need_b)[-8:],
                "over_bound_far": int(sum(int(v.sum()) for v in ev["over"].values())),
                "beyond_cap": int(ev["any_beyond_cap"].sum()),
                "near_threshold": int(ev["near"].sum()), "near_differ": int(ev["near_differ"].sum()),
                "groups_needing": {g: int(v.sum()) for g, v in ev["needed_widening"].items() if v.any()}})
            print(json.dumps({"parity_step": widen_steps[-1]}), flush=True)
        sync_oracle(env, orc)
    e = np.concatenate(errs)
    m = np.concatenate(margins)
    sens = np.concatenate(senss)
    pm_all = np.concatenate(pmargins)
    q = {f"q{p}": float(np.quantile(e, p / 100)) for p in (50, 90, 99, 99.9)}
    far = m >= 1e-4
    worst = np.argsort(-np.where(far, e, 0))[:8]
    out = {"task": task_name, "envs": n, "steps": steps, "sens_probes": n_probes, **q, "max": float(e.max()),
           "max_far_from_threshold": float(e[far].max()) if far.any() else None,
           "frac_gt_2e-3_far": float((e[far] > 2e-3).mean()) if far.any() else None,
           # (env, step, error, decision margin, oracle 2-ulp sensitivity, projection margin:
           # min |unprojected lambda - bound| x A_rr over the env's row projections, m/s)
           "worst_far": [(int(i % n), int(i // n), float(e[i]), float(m[i]), float(sens[i]), float(pm_all[i]))
                         for i in worst],
           "projection_margin_quantiles_far": {f"q{p}": float(np.quantile(pm_all[far], p / 100))
                                               for p in (1, 10, 50)} if far.any() else None,
           # far envs: error vs the oracle's own rounding sensitivity (2-ulp input perturbation)
           "sens_quantiles": {f"q{p}": float(np.quantile(sens, p / 100)) for p in (50, 99, 99.9)},
           "ratio_err_over_sens_far": {f"q{p}": float(np.quantile(e[far] / np.maximum(sens[far], 1e-7), p / 100))
                                       for p in (50, 99, 99.9, 100)},
           "max_far_err_where_sens_lt_2e-4": float(e[far & (sens < 2e-4)].max()) if (far & (sens < 2e-4)).any() else None,
           "frac_far_sens_ge_2e-4": float((sens[far] >= 2e-4).mean()) if far.any() else None,
           "groups": {g: {f"q{p}": float(np.quantile(np.concatenate(v), p / 100)) for p in (50, 99)} |
                      {"max_far": float(np.concatenate(v)[far].max()) if far.any() else None,
                       "max_far_ratio_to_sens": float((np.concatenate(v)[far] / np.maximum(
                           np.concatenate(gsens[g])[far], 1e-6)).max()) if far.any() else None,
                       # the same over the far envs whose error exceeds the task's PGS base bound
                       # (the envs an allowance is for; below it no allowance is needed)
                       "max_ratio_to_sens_above_pgs_base": _ratio_above(
                           np.concatenate(v), np.concatenate(gsens[g]), far,
                           PB.FAR_TOL.get(task_name, {}).get(g))}
                      for g, v in gerr.items()}}
    # reward: float32 potentials are ~6e4 (ulp 3.9e-3); the step's reward carries pot - prev
    pm = np.concatenate(potmag) if potmag else None
    if pm is not None and task_name != "Cartpole":
        r_all = np.concatenate(gerr["rew"])
        ulp = np.spacing(pm.astype(np.float32)).astype(np.float64)
        out["rew_err_over_pot_ulp_far"] = float((r_all[far] / ulp[far]).max())
    if widen_steps:
        out["conditioning_allowance"] = {
            "sens_k": PB.SENS_K, "cap": PB.SENS_CAP, "max_frac_allowed": PB.WIDEN_MAX_FRAC,
            "max_frac_per_step": max(w["frac"] for w in widen_steps),
            "widest_bound_applied": max(w["widest_bound_applied"] for w in widen_steps),
            "over_bound_far_total": sum(w["over_bound_far"] for w in widen_steps),
            "far_tol": PB.FAR_TOL[PB.bounds_key(task_name, env.task.get_robot().sim_params.solver_type)]}
    for g in groups:
        rel = np.concatenate(grel[g])
        mag = np.concatenate(gmag[g])
        ab = np.concatenate(gerr[g])
        w = int(np.argmax(np.where(far, ab, -1)))
        out["groups"][g]["max_far_mixed_rel"] = float(rel[far].max()) if far.any() else None
        out["groups"][g]["worst_far_abs_with_mag"] = [float(ab[w]), float(mag[w])]
    print(json.dumps(out), flush=True)
    dump = os.environ.get("PARITY_DUMP")
    if dump:   # per env-step arrays for offline bound analysis (tools/parity_bounds_fit.py)
        arrs = {"margin": m, "pmargin": pm_all, "sens_env": sens}
        for g in gerr:
            arrs[f"err_{g}"] = np.concatenate(gerr[g]).astype(np.float32)
            arrs[f"sens_{g}"] = np.concatenate(gsens[g]).astype(np.float32)
        for g in groups:
            arrs[f"mag_{g}"] = np.concatenate(gmag[g]).astype(np.float32)
        arrs["mag_rew"] = np.concatenate([np.abs(x) for x in rew_refs]).astype(np.float32)
        arrs["pot"] = np.concatenate(potmag).astype(np.float32) if potmag else np.zeros(0, np.float32)
        for k, v in probe_sens.items():
            arrs[f"probe_{k}"] = np.concatenate(v)
        np.savez_compressed(dump, **arrs)
    orc.close()
    env.close()


if __name__ == "__main__":
    main()
