"""The one-step parity bounds themselves (tests/parity_bounds.py), on synthetic errors: the
conditioning allowance is capped, counted and limited to < 1 % of the envs, base bounds are per
task and field group, threshold envs may differ but stay rare. CPU only."""
import numpy as np
import pytest

from tests import parity_bounds as PB

G = PB.group_slices(21, 2)
O = 12 + 3 * 21 + 12


def _case(n=1000, name="Humanoid"):
    rng = np.random.default_rng(0)
    ref = rng.normal(size=(n, O)).astype(np.float32)
    rew_ref = rng.normal(size=n).astype(np.float32)
    obs = ref + rng.uniform(-1e-6, 1e-6, size=ref.shape).astype(np.float32)
    obs[:, G["actions"]] = ref[:, G["actions"]]
    return ref, rew_ref, obs, rew_ref.copy(), np.full(n, 1.0), np.zeros(n)


def test_clean_step_passes_without_widening():
    ref, rr, obs, rew, margin, sens = _case()
    r = PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)
    assert r["any_needed"].sum() == 0 and r["widest_applied"] == 0.0


def test_allowance_counted_and_widest_reported():
    ref, rr, obs, rew, margin, sens = _case()
    ref[5, 20] = 0.5
    obs[5, 20] = 0.5 + 5e-3             # dof_pos: above its base bound (6e-4)
    sens[5] = 2e-3                      # the oracle says this env's step is ill-conditioned
    logs = []
    r = PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=logs.append)
    assert r["any_needed"].sum() == 1 and r["widest_applied"] == pytest.approx(8e-3)
    assert "1 needed the conditioning allowance" in logs[0] and "0.008" in logs[0]


def test_allowance_is_capped():
    ref, rr, obs, rew, margin, sens = _case()
    ref[7, 0] = obs[7, 0] = 0.5
    obs[7, 0] += 0.05
    sens[7] = 5e-3                      # 4 x sens = 0.02 would allow it: the cap (1e-2) does not
    with pytest.raises(AssertionError, match="root"):
        PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)


def test_allowance_cap_scales_with_magnitude():
    ref, rr, obs, rew, margin, sens = _case()
    sl = G["sensors"]
    ref[4, sl] = 0.0
    ref[4, sl.start] = 5.0              # a 5-unit force reading: the cap is 1 % of it
    obs[4, sl] = ref[4, sl]
    obs[4, sl.start] += 0.04
    sens[4] = 0.04                      # below the cap (0.05): 4 x sens is capped
    r = PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)
    assert r["widest_applied"] == pytest.approx(0.05)
    obs[4, sl.start] += 0.02            # 0.06 > 1 % of 5
    with pytest.raises(AssertionError, match="sensors"):
        PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)


def test_cap_yields_to_the_oracles_own_resolution():
    """Where the oracle's own 2-ulp response reaches the cap, the entry is undetermined at that
    level in float32: the bound is SENS_K x the response, counted as beyond the cap, and only
    ILL_MAX_FRAC of the envs (at least one) may need it."""
    ref, rr, obs, rew, margin, sens = _case()
    sl = G["sensors"]
    ref[4, sl] = 0.0
    ref[4, sl.start] = 0.56             # round 6's worst TGS env: error 1.08e-2, response 1.0e-2
    obs[4, sl] = ref[4, sl]
    obs[4, sl.start] += 1.08e-2
    sens[4] = 1.0e-2
    logs = []
    r = PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=logs.append)
    assert int(r["any_beyond_cap"].sum()) == 1 and "1 beyond the cap" in logs[0]
    obs[4, sl.start] = 0.56 + 4.1e-2    # past 4 x its response
    with pytest.raises(AssertionError, match="sensors"):
        PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)
    obs[4, sl.start] = 0.56 + 1.08e-2   # two such envs in 1000: over ILL_MAX_FRAC
    ref[9, sl] = 0.0
    ref[9, sl.start] = 0.3
    obs[9, sl] = ref[9, sl]
    obs[9, sl.start] += 2e-2
    sens[9] = 1.2e-2
    with pytest.raises(AssertionError, match="beyond the cap"):
        PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)


def test_tgs_base_bounds_are_pgs_derived():
    """the TGS base bounds are the PGS ones x 1.5 (not fitted to the device)."""
    for task in ("Humanoid", "Ant"):
        for g, v in PB.FAR_TOL[task].items():
            assert PB.FAR_TOL[f"{task}/TGS"][g] == pytest.approx(1.5 * v)
    assert PB.SENS_PROBES >= 4


def test_too_many_envs_needing_the_allowance_fail():
    ref, rr, obs, rew, margin, sens = _case()
    idx = np.arange(0, 1000, 50)[:15]   # 1.5 % of the envs
    obs[idx, 20] += 2e-3
    sens[idx] = 1e-3
    with pytest.raises(AssertionError, match="needed the conditioning allowance"):
        PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)


def test_ant_bounds_are_tighter_than_humanoid():
    ref, rr, obs, rew, margin, sens = _case(name="Ant")
    obs[3, 20] += 1e-4                  # fine for Humanoid dof_pos, not for Ant (6e-6)
    PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)
    with pytest.raises(AssertionError, match="dof_pos"):
        PB.check("Ant", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)


def test_reward_potential_quantisation_allowance():
    ref, rr, obs, rew, margin, sens = _case()
    rr[9] = 0.5
    rew[9] = 0.5 + 5e-3                 # 2 ulp of a 6e4 potential is 7.8e-3
    pot = np.full(1000, 10.0)
    with pytest.raises(AssertionError, match="rew"):
        PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, pot=pot, quantiles=False, log=None)
    pot[9] = 6e4
    PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, pot=pot, quantiles=False, log=None)


def test_threshold_envs_may_differ_but_stay_rare():
    ref, rr, obs, rew, margin, sens = _case()
    obs[:10, 0] += 0.5
    margin[:10] = 1e-6                  # 1 %: allowed
    PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)
    obs[:30, 0] += 0.5
    margin[:30] = 1e-6                  # 3 %: not
    with pytest.raises(AssertionError, match="at a threshold"):
        PB.check("Humanoid", G, obs, rew, ref, rr, margin, sens=sens, quantiles=False, log=None)
