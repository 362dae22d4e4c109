"""Randomizer — observation / action noise domain randomization (reference:
utils/domain_randomization/randomize.py:38-306, applied from envs/vec_env_rlgames.py:59-60,70-71).

Same configuration surface — the task YAML's ``domain_randomization`` block::

    domain_randomization:
      randomize: True
      randomization_params:
        observations: {on_reset: {operation, distribution, distribution_parameters},
                       on_interval: {frequency_interval, operation, distribution, distribution_parameters}}
        actions: {...same...}

with the same validation errors, flags (``task.randomize_observations`` / ``randomize_actions``)
and apply methods. The noise itself runs in HIP (include/mi_dr.h): inside the fused env-step
launch when VecEnvRLGames takes the fused path, or as one kernel per apply call
(``mi_dr_apply_actions`` / ``mi_dr_apply_observations``) on the method-by-method path.

Physics-parameter randomization (``simulation``, ``rigid_prim_views``, ``articulation_views``:
randomize.py:59-118,137-162,308-578) drives omni.replicator over PhysX views; it is outside this
build's hot path and is refused loudly rather than silently ignored.
"""
from __future__ import annotations

import ctypes as C

from ... import native as N

_OPS = {"additive": N.MI_DR_OP_ADDITIVE, "scaling": N.MI_DR_OP_SCALING}
_DISTS = {"gaussian": N.MI_DR_DIST_GAUSSIAN, "normal": N.MI_DR_DIST_GAUSSIAN,
          "uniform": N.MI_DR_DIST_UNIFORM, "loguniform": N.MI_DR_DIST_LOGUNIFORM,
          "log_uniform": N.MI_DR_DIST_LOGUNIFORM}
_PHYSICS_GROUPS = ("simulation", "rigid_prim_views", "articulation_views")


def _noise(params: dict, what: str, interval: bool) -> N.MiDrNoise:
    """One schedule -> mi_dr_noise, with the reference's required-key checks
    (randomize.py:183-191 / 200-208)."""
    need = {"operation", "distribution", "distribution_parameters"}
    if interval:
        need = need | {"frequency_interval"}
    if not need.issubset(params.keys()):
        kind = "on_interval" if interval else "on_reset"
        raise ValueError(f"Please ensure the following {what} {kind} randomization parameters are "
                         f"provided: " + ", ".join(sorted(need)) + ".")
    op, dist = params["operation"], params["distribution"]
    if op not in _OPS:
        raise ValueError(f"The specified {op} operation type is not supported.")
    if dist not in _DISTS:
        raise ValueError(f"The specified {dist} distribution is not supported.")
    p = [float(v) for v in params["distribution_parameters"]]
    if len(p) != 2:
        raise ValueError(f"{what}: distribution_parameters must hold 2 scalars, got {p}")
    n = N.MiDrNoise()
    n.enabled = 1
    n.operation = _OPS[op]
    n.distribution = _DISTS[dist]
    n.frequency_interval = int(params.get("frequency_interval", 1))
    n.params[0], n.params[1] = p
    return n


class Randomizer:
    def __init__(self, sim_config) -> None:
        """randomize.py:39-55."""
        self._cfg = sim_config.task_config
        self._config = sim_config.config
        self.randomize = False
        self.distributions = dict()
        self.active_domain_randomizations = dict()
        self._observations_dr_params = None
        self._actions_dr_params = None
        self._task = None
        dr_config = self._cfg.get("domain_randomization", None)
        if dr_config is not None:
            randomize = dr_config.get("randomize", False)
            randomization_params = dr_config.get("randomization_params", None)
            if randomize and randomization_params is not None:
                self.randomize = True
                self.min_frequency = dr_config.get("min_frequency", 1)

    def _physics_groups(self) -> list:
        rp = self._cfg["domain_randomization"]["randomization_params"]
        return [g for g in _PHYSICS_GROUPS if rp.get(g) is not None]

    def apply_on_startup_domain_randomization(self, task) -> None:
        """randomize.py:57-124: on_startup scale / mass / density of prim views."""
        if self.randomize:
            groups = self._physics_groups()
            if groups:
                raise NotImplementedError(
                    f"physics-parameter domain randomization ({', '.join(groups)}) is not part of "
                    f"this build (observation / action noise only)")
        elif self._cfg.get("domain_randomization", None) is None:
            raise ValueError("No domain randomization parameters are specified in the task yaml config file")
        else:
            print("On Startup Domain randomization will not be applied.")

    def set_up_domain_randomization(self, task) -> None:
        """randomize.py:126-174: registers the observation / action schedules with the task's
        mi_sim handle (mi_task_set_dr) and sets task.randomize_observations / randomize_actions."""
        if not self.randomize:
            if self._cfg.get("domain_randomization", None) is None:
                raise ValueError("No domain randomization parameters are specified in the task yaml config file")
            print("Domain randomization will not be applied.")
            return
        groups = self._physics_groups()
        if groups:
            raise NotImplementedError(
                f"physics-parameter domain randomization ({', '.join(groups)}) is not part of this "
                f"build (observation / action noise only)")
        rp = self._cfg["domain_randomization"]["randomization_params"]
        dr = N.MiDrParams()
        for key, which in (("observations", "obs"), ("actions", "act")):
            if key not in rp:
                continue
            params = rp[key]
            if params is None:
                raise ValueError(f"{key.capitalize()} randomization parameters are not provided.")
            if key == "observations":
                task.randomize_observations = True
                self._observations_dr_params = params
            else:
                task.randomize_actions = True
                self._actions_dr_params = params
            if "on_reset" in params:
                setattr(dr, f"{which}_on_reset", _noise(params["on_reset"], key, False))
                self.active_domain_randomizations[(key, "on_reset")] = list(params["on_reset"]["distribution_parameters"])
            if "on_interval" in params:
                setattr(dr, f"{which}_on_interval", _noise(params["on_interval"], key, True))
                self.active_domain_randomizations[(key, "on_interval")] = list(params["on_interval"]["distribution_parameters"])
        self._dr = dr
        self._task = task
        view = task.get_robot()
        N.check(N.lib().mi_task_set_dr(view.handle, C.byref(dr)), "mi_task_set_dr")

    def params(self):
        """The mi_dr_params registered with the sim (None before set-up)."""
        return getattr(self, "_dr", None)

    # -- the two apply calls of VecEnvRLGames.step's method-by-method path ------------------
    def apply_actions_randomization(self, actions, reset_buf):
        """randomize.py:237-260: in place on the clamped [N, A] actions."""
        view = self._task.get_robot()
        a = actions.contiguous()
        N.check(N.lib().mi_dr_apply_actions(view.handle, a.data_ptr(), reset_buf.data_ptr(),
                                            view.stream()), "mi_dr_apply_actions")
        if a.data_ptr() != actions.data_ptr():
            actions.copy_(a)
        return actions

    def apply_observations_randomization(self, observations, reset_buf):
        """randomize.py:212-235: in place on task.obs_buf."""
        view = self._task.get_robot()
        if not observations.is_contiguous():
            raise ValueError("observations must be contiguous (task.obs_buf)")
        N.check(N.lib().mi_dr_apply_observations(view.handle, observations.data_ptr(),
                                                 reset_buf.data_ptr(), view.stream()),
                "mi_dr_apply_observations")
        return observations
