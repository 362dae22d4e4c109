"""GPU: free-running device vs oracle rollouts (no re-sync), BASELINE full size (4096 envs).

The per-step parity tests re-sync the oracle to the device state every step; chaotic contact
makes per-env comparison meaningless over long horizons, so this test compares the
distributions a policy would see after `STEPS` free-running steps from the identical
post-reset state with identical Philox actions (tools/free_run.py): per-step reward samples
(two-sample KS statistic and the mean), completed-episode lengths (KS, count, mean) and the
per-step reset rate (locomotion.py:257-321, cartpole.py:143-162). Bounds are ~5-10x the
measured values: Humanoid reward KS 2e-4, episode-length KS 6e-4; Ant reward KS
1.5e-3 (Ant rarely falls in 200 random steps, so its episode statistics are count-only);
Cartpole identical.
"""
import pytest

from tools.free_run import free_run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,steps", [("Humanoid", 200), ("Ant", 200), ("Cartpole", 300)])
def test_free_running_distributions_match_oracle(gpu, name, steps):
    r = free_run(name, 4096, steps)
    assert r["reward_ks"] <= 0.01, r
    dm, om = r["reward_mean"]
    assert abs(dm - om) <= 0.01 * max(abs(om), 0.1), r
    assert r["reset_rate_window_maxdiff"] <= 0.005, r
    nd, no = r["episodes"]
    assert abs(nd - no) <= max(8, 0.03 * no), r
    if no >= 1000:
        assert r["episode_len_ks"] <= 0.02, r
        ld, lo = r["episode_len_mean"]
        assert abs(ld - lo) <= 0.02 * lo, r
