"""SimConfig — merges the task YAML ``sim``/``physx``/per-actor blocks over defaults and turns
them into the solver parameters of libmi_sim.so.

Mirrors utils/config_utils/sim_config.py:36-142 (``_parse_config``, ``_sanitize_device``,
``parse_actor_config``, ``get_physics_params``); the USD-attribute plumbing of
``apply_articulation_settings`` (:353-403) has no equivalent — the parameters go straight to
the native solver (``mi_sim_params``).
"""
from __future__ import annotations

import copy
import math
from typing import Any, Dict

from ... import native as N

# restated from utils/config_utils/default_scene_params.py:30-112 (the keys the build uses)
default_physx_params: Dict[str, Any] = {
    "use_gpu": False,
    "worker_thread_count": 4,
    "solver_type": 1,
    "solver_position_iteration_count": 4,
    "solver_velocity_iteration_count": 1,
    "enable_gyroscopic_forces": False,
    "max_depenetration_velocity": 100.0,
    "contact_offset": 0.02,
    "rest_offset": 0.001,
    # build-specific (no PhysX counterpart): Baumgarte factor of the velocity-level solve
    "mi_erp": 0.2,
    # PhysX rigid-body default max angular velocity 5729.58 deg/s
    # (docs/transfering_policies_from_isaac_gym.md:73-76)
    "max_angular_velocity": math.radians(5729.58),
    # PhysX articulation-link default angular damping 0.05
    # (docs/transfering_policies_from_isaac_gym.md:74); the task YAMLs do not set it
    "angular_damping": 0.05,
    # accepted and validated, not modelled by the native solver (PHYSX_UNMODELLED below)
    "bounce_threshold_velocity": 0.2,
    "friction_offset_threshold": 0.04,
    "friction_correlation_distance": 0.025,
    "enable_sleeping": True,
    "enable_stabilization": True,
    "sleep_threshold": 0.0,
    "stabilization_threshold": 0.0,
}
default_physics_material = {"static_friction": 1.0, "dynamic_friction": 1.0, "restitution": 0.0}
default_sim_params: Dict[str, Any] = {
    "gravity": [0.0, 0.0, -9.81],
    "dt": 1.0 / 60.0,
    "substeps": 1,
    "use_gpu_pipeline": True,
    "add_ground_plane": True,
    "default_physics_material": default_physics_material,
}
default_actor_options: Dict[str, Any] = {
    "enable_self_collisions": -1,
    "enable_gyroscopic_forces": -1,
    "solver_position_iteration_count": -1,
    "solver_velocity_iteration_count": -1,
    "sleep_threshold": -1,
    "stabilization_threshold": -1,
    "max_depenetration_velocity": -1,
    "contact_offset": -1,
    "rest_offset": -1,
}


# PhysX knobs of the task YAMLs (cfg/task/Humanoid.yaml:57-61,86-87; Ant.yaml:62-63,88-89;
# Cartpole.yaml:45-46,71-72; defaults utils/config_utils/default_scene_params.py:34-63) that the
# native solver accepts but does not model, with the reason (DESIGN §5 "PhysX knobs"):
PHYSX_UNMODELLED = {
    "enable_sleeping": "articulations are never put to sleep: the task loop writes actuation "
                       "forces every step, and PhysX's articulation cache write wakes the "
                       "articulation (applyCache autowake), so a driven env does not sleep there "
                       "either; sleep_threshold is validated and ignored",
    "enable_stabilization": "PhysX's experimental stabilization pass (extra damping of bodies "
                            "below stabilization_threshold, mass-normalised kinetic energy) is not "
                            "modelled; stabilization_threshold is validated and ignored",
    "bounce_threshold_velocity": "no effect: every task's restitution is 0, so no contact bounces",
    "friction_offset_threshold": "no effect while contact_offset <= friction_offset_threshold "
                                 "(0.02 <= 0.04 in every task): every speculative contact within "
                                 "contact_offset already carries friction rows",
    "friction_correlation_distance": "friction is per contact point (two pyramid rows each), not "
                                     "merged into patch anchors",
}
_warned = set()


def _warn_unmodelled(keys) -> None:
    new = [k for k in keys if k not in _warned]
    if new:
        import warnings
        _warned.update(new)
        warnings.warn("mi_sim: PhysX settings accepted but not modelled: " +
                      "; ".join(f"{k} ({PHYSX_UNMODELLED[k]})" for k in new), stacklevel=3)


class SimConfig:
    def __init__(self, config: Dict[str, Any] = None):
        self._config = dict(config or {})
        self._cfg = self._config.get("task", {})
        self._parse_config()
        self._sanitize_device()

    def _parse_config(self) -> None:
        self._sim_params = copy.deepcopy(default_sim_params)
        self._physx_params = copy.deepcopy(default_physx_params)
        sim = self._cfg.get("sim", {}) or {}
        for k, v in sim.items():
            if k == "physx":
                self._physx_params.update(v or {})
            elif k == "default_physics_material":
                self._sim_params[k] = {**default_physics_material, **(v or {})}
            elif not isinstance(v, dict):
                self._sim_params[k] = v
        self._sim_params["physx"] = self._physx_params

    def _sanitize_device(self) -> None:
        if self._sim_params["use_gpu_pipeline"]:
            self._physx_params["use_gpu"] = True
        if self._config.get("sim_device", "gpu") == "gpu" or self._sim_params["use_gpu_pipeline"]:
            self._config["sim_device"] = f"cuda:{self._config.get('device_id', 0)}"
        else:
            self._config["sim_device"] = "cpu"
        self._config.setdefault("rl_device", "cuda:0")

    @property
    def sim_params(self) -> Dict[str, Any]:
        return self._sim_params

    @property
    def config(self) -> Dict[str, Any]:
        return self._config

    @property
    def task_config(self) -> Dict[str, Any]:
        return self._cfg

    @property
    def physx_params(self) -> Dict[str, Any]:
        return self._physx_params

    def get_physics_params(self) -> Dict[str, Any]:
        return self._sim_params

    def parse_actor_config(self, actor_name: str) -> Dict[str, Any]:
        actor = copy.deepcopy(default_actor_options)
        actor.update((self._cfg.get("sim", {}) or {}).get(actor_name, {}) or {})
        for k, v in actor.items():
            if v == -1 and k in self._physx_params:
                actor[k] = self._physx_params[k]
        return actor

    def mi_sim_params(self, actor_name: str) -> N.MiSimParams:
        """The native solver parameters for one articulation (mi_sim_params)."""
        a = self.parse_actor_config(actor_name)
        sp, px = self._sim_params, self._physx_params
        p = N.MiSimParams()
        p.dt = float(sp["dt"])
        p.gravity[:] = [float(g) for g in sp["gravity"]]
        # physx.solver_type (cfg/config.yaml:31, default 1 = TGS): TGS takes the position and
        # velocity iteration counts separately (position iterations are its sub-steps); PGS runs
        # their sum as sweeps (include/mi_sim.h MI_SOLVER_*)
        st = int(px.get("solver_type", 1))
        if st not in (N.MI_SOLVER_PGS, N.MI_SOLVER_TGS):
            raise ValueError(f"physx.solver_type {st}: this build implements 0 (PGS) and 1 (TGS)")
        npos, nvel = int(a["solver_position_iteration_count"]), int(a["solver_velocity_iteration_count"])
        p.solver_type = st
        if st == N.MI_SOLVER_TGS:
            p.solver_iterations, p.velocity_iterations = npos, nvel
        else:
            p.solver_iterations, p.velocity_iterations = npos + nvel, 0
        p.contact_offset = float(a["contact_offset"])
        p.rest_offset = float(a["rest_offset"])
        p.friction = float(sp["default_physics_material"]["dynamic_friction"])
        p.max_depenetration_velocity = float(a["max_depenetration_velocity"])
        p.erp = float(px.get("mi_erp", 0.2))
        esc = a.get("enable_self_collisions", False)
        p.enable_self_collisions = 1 if esc is True or esc == 1 else 0
        p.max_angular_velocity = float(px.get("max_angular_velocity", math.radians(5729.58)))
        p.angular_damping = float(a.get("angular_damping", px.get("angular_damping", 0.05)))
        self.unmodelled(actor_name)
        return p

    def unmodelled(self, actor_name: str) -> Dict[str, Any]:
        """The PhysX settings of this actor that the native solver accepts but does not model
        (PHYSX_UNMODELLED), validated the way PhysX would (thresholds in [0, inf), booleans);
        warns once per key and process. Returns {key: value} of those in effect."""
        a = self.parse_actor_config(actor_name)
        px = self._physx_params
        out: Dict[str, Any] = {}
        for k in ("sleep_threshold", "stabilization_threshold"):
            v = float(a[k])
            if not (0.0 <= v < math.inf):
                raise ValueError(f"{actor_name}.{k} = {v}: allowed range [0, max_float)")
            out[k] = v
        for k in ("enable_sleeping", "enable_stabilization"):
            if not isinstance(px[k], bool) and px[k] not in (0, 1):
                raise ValueError(f"physx.{k} = {px[k]!r}: a boolean")
            out[k] = bool(px[k])
        for k in ("bounce_threshold_velocity", "friction_offset_threshold", "friction_correlation_distance"):
            out[k] = float(px[k])
        if float(self._sim_params["default_physics_material"].get("restitution", 0.0)) != 0.0:
            raise ValueError("default_physics_material.restitution != 0: restitution is not modelled")
        active = [k for k in ("enable_sleeping", "enable_stabilization") if out[k]]
        if out["friction_offset_threshold"] < float(a["contact_offset"]):
            active.append("friction_offset_threshold")
        active.append("friction_correlation_distance")
        _warn_unmodelled(active)
        return out
