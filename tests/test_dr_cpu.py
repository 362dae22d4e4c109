"""Observation / action noise DR on CPU (utils/domain_randomization/randomize.py:212-306).

The oracle (oracle.c + include/mi_dr.h) recomputes correlated noise from a per-env epoch
instead of storing the reference's [N, C] correlated-noise buffer. `RefRandomizer` below is a
direct restatement of the reference's buffer algorithm (counter buffer, stored correlated
buffer initialised to zeros, nonzero() id sets) drawing from the same Philox values; the oracle
must match it over random reset masks (same schedule; values to 1 ulp of the transcendentals). Distribution moments and the config
validation of the Python Randomizer are checked too."""
import math

import numpy as np
import pytest

from omniisaacgymenvs_amd import native as N
from omniisaacgymenvs_amd.utils.domain_randomization.randomize import _noise
from oracle.oracle import OracleSim, lib as orc_lib
from tests.helpers import sim_params, task_params_from_cfg

F32 = np.float32
STREAMS = {("obs", "reset"): 2, ("obs", "interval"): 3, ("act", "reset"): 4, ("act", "interval"): 5}


def _draw(seed, gid, key, k, stream, dist, p0, p1):
    """mi_dr_value on the oracle's Philox uniforms, restated in float32 numpy."""
    u = [orc_lib().orc_uniform(seed, gid, key, 4 * (k >> 1) + q, stream) for q in range(4)]
    ua, ub = F32(u[2 * (k & 1)]), F32(u[2 * (k & 1) + 1])
    if dist == N.MI_DR_DIST_GAUSSIAN:
        r = np.sqrt(F32(-2.0) * np.log(F32(1.0) - ua, dtype=F32), dtype=F32)
        return F32(p0) + F32(p1) * (r * np.cos(F32(6.283185307179586) * ub, dtype=F32))
    if dist == N.MI_DR_DIST_UNIFORM:
        return (F32(p1) - F32(p0)) * ua + F32(p0)
    l0, l1 = np.log(F32(p0), dtype=F32), np.log(F32(p1), dtype=F32)
    return np.exp((l1 - l0) * ua + l0, dtype=F32)


class RefRandomizer:
    """randomize.py:176-306 restated literally for one buffer kind, stored buffers and all."""

    def __init__(self, kind, n, C, seed, on_reset=None, on_interval=None):
        self.kind, self.n, self.C, self.seed = kind, n, C, seed
        self.on_reset, self.on_interval = on_reset, on_interval
        self.counter = np.zeros(n, np.int64)                 # randomize.py:191 / :208
        self.corr = np.zeros((n, C), F32)                    # randomize.py:192 / :209
        self.n_reset_draws = np.zeros(n, np.int64)           # only to name the Philox key
        self.n_interval_draws = np.zeros(n, np.int64)

    def _noise(self, cfg, which, i, key):
        op, dist, (p0, p1) = cfg["op"], cfg["dist"], cfg["params"]
        return np.array([_draw(self.seed, i, key, k, STREAMS[(self.kind, which)], dist, p0, p1)
                         for k in range(self.C)], F32)

    def apply(self, buf, reset_buf):
        env_ids = np.nonzero(reset_buf)[0]
        self.counter[env_ids] = 0
        self.counter += 1
        if self.on_reset is not None:                        # _apply_correlated_noise
            for i in env_ids:
                self.n_reset_draws[i] += 1
                self.corr[i] = self._noise(self.on_reset, "reset", i, self.n_reset_draws[i])
            buf = buf + self.corr if self.on_reset["op"] == 0 else buf * self.corr
        if self.on_interval is not None:                     # _apply_uncorrelated_noise
            ids = np.nonzero(self.counter >= self.on_interval["freq"])[0]
            self.counter[ids] = 0
            for i in ids:
                self.n_interval_draws[i] += 1
                nz = self._noise(self.on_interval, "interval", i, self.n_interval_draws[i])
                buf[i] = buf[i] + nz if self.on_interval["op"] == 0 else buf[i] * nz
        return buf.astype(F32)


def _mk(op, dist, p, freq=1):
    n = N.MiDrNoise()
    n.enabled, n.operation, n.distribution, n.frequency_interval = 1, op, dist, freq
    n.params[0], n.params[1] = p
    return n


def _oracle(task="Ant", n=24, seed=11):
    tp, m, keep = task_params_from_cfg(task)
    origins = np.zeros((n, 3), F32)
    orc = OracleSim(m, sim_params(rest_offset=0.0), n, origins, seed=seed)
    orc.configure(tp, keep=keep)
    return orc, tp


@pytest.mark.parametrize("kind", ["obs", "act"])
@pytest.mark.parametrize("case", [
    dict(r=(0, 0, (0.0, 0.05)), i=(0, 0, (0.0, 0.02), 3)),   # additive gaussian, both schedules
    dict(r=(1, 1, (0.8, 1.2)), i=None),                       # scaling uniform, reset only (epoch-0 zeros)
    dict(r=None, i=(1, 2, (0.5, 2.0), 2)),                    # scaling loguniform, interval only
    dict(r=(0, 1, (-0.1, 0.1)), i=(0, 0, (0.0, 0.3), 1)),     # frequency 1: fires every call
])
def test_oracle_matches_reference_buffer_algorithm(kind, case):
    orc, tp = _oracle()
    C = tp.num_obs if kind == "obs" else tp.num_actions
    dr = N.MiDrParams()
    ref_r = ref_i = None
    if case["r"]:
        op, dist, p = case["r"]
        setattr(dr, f"{kind}_on_reset", _mk(op, dist, p))
        ref_r = dict(op=op, dist=dist, params=p)
    if case["i"]:
        op, dist, p, f = case["i"]
        setattr(dr, f"{kind}_on_interval", _mk(op, dist, p, f))
        ref_i = dict(op=op, dist=dist, params=p, freq=f)
    orc.set_dr(dr)
    ref = RefRandomizer(kind, orc.N, C, 11, ref_r, ref_i)
    rng = np.random.default_rng(3)
    for step in range(9):
        buf = rng.normal(size=(orc.N, C)).astype(F32)
        reset = np.zeros(orc.N, np.int64) if step else np.ones(orc.N, np.int64)
        if step:
            reset[rng.random(orc.N) < 0.25] = 1
        want = ref.apply(buf.copy(), reset)
        got = buf.copy()
        (orc.dr_apply_observations if kind == "obs" else orc.dr_apply_actions)(got, reset)
        # exact schedule; values to 1 ulp (numpy's float32 log/cos vs libm's logf/cosf)
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=5e-7, err_msg=f"step {step}")
        st = orc.dr_state()[:, (0 if kind == "obs" else 3):][:, :3]
        np.testing.assert_array_equal(st[:, 0], ref.counter)
    orc.close()


def test_scaling_with_epoch_zero_zeroes_the_row():
    """randomize.py:192/209 start the correlated buffer at zeros: an env whose first apply call
    is not a reset multiplies by 0 under "scaling" (a reference quirk, kept)."""
    orc, tp = _oracle(n=4)
    dr = N.MiDrParams()
    dr.obs_on_reset = _mk(N.MI_DR_OP_SCALING, N.MI_DR_DIST_UNIFORM, (0.9, 1.1))
    orc.set_dr(dr)
    buf = np.ones((4, tp.num_obs), F32)
    orc.dr_apply_observations(buf, np.array([1, 0, 1, 0], np.int64))
    assert np.all(buf[[1, 3]] == 0.0)
    assert np.all((buf[[0, 2]] >= 0.9) & (buf[[0, 2]] < 1.1))
    orc.close()


@pytest.mark.parametrize("dist,p", [(N.MI_DR_DIST_GAUSSIAN, (0.3, 0.05)),
                                    (N.MI_DR_DIST_UNIFORM, (-0.2, 0.6)),
                                    (N.MI_DR_DIST_LOGUNIFORM, (0.5, 4.0))])
def test_noise_distribution_moments(dist, p):
    orc, tp = _oracle(task="Humanoid", n=512)
    dr = N.MiDrParams()
    dr.obs_on_interval = _mk(N.MI_DR_OP_ADDITIVE, dist, p, 1)
    orc.set_dr(dr)
    buf = np.zeros((orc.N, tp.num_obs), F32)
    orc.dr_apply_observations(buf, np.zeros(orc.N, np.int64))
    x = buf.ravel().astype(np.float64)
    if dist == N.MI_DR_DIST_GAUSSIAN:
        mean, std = p
        assert abs(x.mean() - mean) < 5 * std / math.sqrt(x.size)
        assert abs(x.std() - std) < 0.02 * std
    elif dist == N.MI_DR_DIST_UNIFORM:
        lo, hi = float(F32(p[0])), float(F32(p[1]))
        assert x.min() >= lo and x.max() < hi
        assert abs(x.mean() - (lo + hi) / 2) < 0.01 * (hi - lo)
    else:
        lo, hi = p
        lx = np.log(x)
        assert x.min() >= lo and x.max() < hi * (1 + 1e-6)
        assert abs(lx.mean() - (math.log(lo) + math.log(hi)) / 2) < 0.01
    orc.close()


def test_noise_config_validation():
    ok = _noise({"operation": "additive", "distribution": "normal",
                 "distribution_parameters": [0, 0.1]}, "observations", False)
    assert ok.enabled == 1 and ok.distribution == N.MI_DR_DIST_GAUSSIAN
    iv = _noise({"operation": "scaling", "distribution": "log_uniform", "frequency_interval": 4,
                 "distribution_parameters": [0.5, 2]}, "actions", True)
    assert iv.frequency_interval == 4 and iv.operation == N.MI_DR_OP_SCALING
    with pytest.raises(ValueError, match="frequency_interval"):
        _noise({"operation": "additive", "distribution": "uniform",
                "distribution_parameters": [0, 1]}, "actions", True)
    with pytest.raises(ValueError, match="not supported"):
        _noise({"operation": "multiply", "distribution": "uniform",
                "distribution_parameters": [0, 1]}, "actions", False)
    with pytest.raises(ValueError, match="not supported"):
        _noise({"operation": "additive", "distribution": "beta",
                "distribution_parameters": [0, 1]}, "actions", False)


def test_fused_oracle_step_with_dr_is_deterministic_and_differs():
    """A DR-on fused oracle step differs from DR-off exactly in obs (noise) and keeps rewards /
    resets computed from the un-noised observations (calculate_metrics runs before the noise)."""
    from oracle.oracle import make_buffers
    outs = []
    for with_dr in (False, True, True):
        orc, tp = _oracle(task="Ant", n=16)
        if with_dr:
            dr = N.MiDrParams()
            dr.obs_on_reset = _mk(N.MI_DR_OP_ADDITIVE, N.MI_DR_DIST_GAUSSIAN, (0.0, 0.01))
            dr.obs_on_interval = _mk(N.MI_DR_OP_ADDITIVE, N.MI_DR_DIST_GAUSSIAN, (0.0, 0.01), 2)
            orc.set_dr(dr)
        b = make_buffers(16, tp.num_obs, tp.num_actions)
        b["reset"][:] = 1
        # step 1 (the reset step): epoch-0 correlated noise is zero and the interval counter is
        # 1 < 2, so the obs are still clean (randomize.py semantics); step 2 fires the interval
        for _ in range(2):
            orc.env_step(np.zeros((16, tp.num_actions), F32), 2, b)
        outs.append({k: v.copy() for k, v in b.items() if v is not None})
        orc.close()
    off, on1, on2 = outs
    for k in on1:
        np.testing.assert_array_equal(on1[k], on2[k])
    assert not np.array_equal(off["obs"], on1["obs"])
    np.testing.assert_array_equal(off["rew"], on1["rew"])
    np.testing.assert_array_equal(off["reset"], on1["reset"])


def test_randomizer_reads_task_yaml_block():
    """The composed config (Hydra-style +key overrides) reaches Randomizer like
    cfg/task/ShadowHand.yaml's block reaches the reference's (randomize.py:39-55)."""
    from omniisaacgymenvs_amd.utils.config_utils.sim_config import SimConfig
    from omniisaacgymenvs_amd.utils.domain_randomization.randomize import Randomizer
    from omniisaacgymenvs_amd.utils.hydra_cfg.hydra_utils import compose
    from tests.test_gpu_dr import DR_OVERRIDES

    off = Randomizer(SimConfig(compose(["task=Ant", "pipeline=cpu", "sim_device=cpu"])))
    assert off.randomize is False
    on = Randomizer(SimConfig(compose(["task=Ant", "pipeline=cpu", "sim_device=cpu"] + DR_OVERRIDES)))
    assert on.randomize is True
    rp = on._cfg["domain_randomization"]["randomization_params"]
    assert rp["observations"]["on_interval"]["frequency_interval"] == 2
    assert rp["actions"]["on_interval"]["distribution_parameters"] == [0.0, 0.02]
    phys = Randomizer(SimConfig(compose(["task=Ant", "pipeline=cpu", "sim_device=cpu"] + DR_OVERRIDES +
                                        ["task.domain_randomization.randomization_params.simulation.gravity.on_interval.frequency_interval=720"])))
    with pytest.raises(NotImplementedError, match="simulation"):
        phys.set_up_domain_randomization(task=None)
