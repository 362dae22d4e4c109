"""ctypes binding of libmi_sim.so (include/mi_sim.h).

This is the only door into the native hot path. Loading is strict: when the HIP library is
missing, cannot be loaded, or no GPU is visible, :func:`lib` raises — there is no CPU
fallback anywhere in the product (the CPU oracle under ``oracle/`` is test infrastructure).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MI_SIM_LIB", os.path.join(_HERE, "libmi_sim.so"))

MI_OK = 0
MI_TASK_CARTPOLE, MI_TASK_ANT, MI_TASK_HUMANOID = 0, 1, 2
MI_DYN_ARTICULATION, MI_DYN_CARTPOLE = 0, 1
MI_SOLVER_PGS, MI_SOLVER_TGS = 0, 1
MI_JOINT_HINGE, MI_JOINT_SLIDE = 0, 1
MI_GEOM_SPHERE, MI_GEOM_CAPSULE = 0, 1

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)


class MiModelDesc(C.Structure):
    _fields_ = [
        ("dyn_kind", C.c_int32), ("root_free", C.c_int32), ("num_links", C.c_int32),
        ("num_geoms", C.c_int32), ("num_sensors", C.c_int32), ("num_pairs", C.c_int32),
        ("parent", _i32p), ("jtype", _i32p), ("axis", _f32p), ("pos", _f32p), ("quat", _f32p),
        ("mass", _f32p), ("com", _f32p), ("inertia", _f32p), ("lower", _f32p), ("upper", _f32p),
        ("damping", _f32p), ("armature", _f32p), ("geom_link", _i32p), ("geom_type", _i32p),
        ("geom_p0", _f32p), ("geom_p1", _f32p), ("geom_radius", _f32p), ("sensor_link", _i32p),
        ("sensor_pos", _f32p), ("pairs", _i32p),
        ("cart_mass", C.c_float), ("pole_mass", C.c_float), ("pole_com", C.c_float),
        ("pole_inertia", C.c_float), ("cart_damping", C.c_float), ("pole_damping", C.c_float),
    ]


class MiSimParams(C.Structure):
    _fields_ = [
        ("dt", C.c_float), ("gravity", C.c_float * 3), ("solver_iterations", C.c_int32),
        ("contact_offset", C.c_float), ("rest_offset", C.c_float), ("friction", C.c_float),
        ("max_depenetration_velocity", C.c_float), ("erp", C.c_float),
        ("enable_self_collisions", C.c_int32), ("max_angular_velocity", C.c_float),
        ("angular_damping", C.c_float), ("solver_type", C.c_int32), ("velocity_iterations", C.c_int32),
    ]


class MiTaskParams(C.Structure):
    _fields_ = [
        ("task_kind", C.c_int32), ("num_obs", C.c_int32), ("num_actions", C.c_int32),
        ("clip_actions", C.c_float), ("clip_obs", C.c_float), ("max_episode_length", C.c_float),
        ("power_scale", C.c_float), ("heading_weight", C.c_float), ("up_weight", C.c_float),
        ("actions_cost", C.c_float), ("energy_cost", C.c_float), ("dof_vel_scale", C.c_float),
        ("angular_velocity_scale", C.c_float), ("contact_force_scale", C.c_float),
        ("joints_at_limit_cost", C.c_float), ("death_cost", C.c_float),
        ("termination_height", C.c_float), ("alive_reward_scale", C.c_float),
        ("task_dt", C.c_float), ("target", C.c_float * 3), ("init_root_pos", C.c_float * 3),
        ("init_root_quat", C.c_float * 4), ("dof_pos_noise", C.c_float),
        ("dof_vel_noise", C.c_float), ("joint_gears", _f32p), ("motor_effort_ratio", _f32p),
        ("init_dof_pos", _f32p), ("reset_dist", C.c_float), ("max_push_effort", C.c_float),
    ]


MI_DR_OP_ADDITIVE, MI_DR_OP_SCALING = 0, 1
MI_DR_DIST_GAUSSIAN, MI_DR_DIST_UNIFORM, MI_DR_DIST_LOGUNIFORM = 0, 1, 2


class MiDrNoise(C.Structure):
    _fields_ = [("enabled", C.c_int32), ("operation", C.c_int32), ("distribution", C.c_int32),
                ("frequency_interval", C.c_int32), ("params", C.c_float * 2)]


class MiDrParams(C.Structure):
    _fields_ = [("obs_on_reset", MiDrNoise), ("obs_on_interval", MiDrNoise),
                ("act_on_reset", MiDrNoise), ("act_on_interval", MiDrNoise)]


def fptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(_f32p)


def iptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(_i32p)


class NativeUnavailable(RuntimeError):
    """libmi_sim.so could not be used: not built, failed to load, or no GPU."""


_LIB = None

_SIGS = {
    "mi_sim_create": (C.c_int, [C.POINTER(MiModelDesc), C.POINTER(MiSimParams), C.c_int32,
                                C.c_int64, C.c_int32, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "mi_sim_destroy": (C.c_int, [C.c_void_p]),
    "mi_sim_info": (C.c_int, [C.c_void_p, _i32p, _i32p, _i32p, _i32p, C.c_void_p]),
    "mi_get_root_state": (C.c_int, [C.c_void_p] + [C.c_void_p] * 4),
    "mi_get_dof_state": (C.c_int, [C.c_void_p] + [C.c_void_p] * 3),
    "mi_get_sensor_wrench": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mi_set_dof_efforts": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "mi_set_dof_state": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                   C.c_void_p]),
    "mi_set_root_state": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_int32, C.c_void_p]),
    "mi_set_dof_state_i32": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                       C.c_void_p]),
    "mi_set_root_state_i32": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_int32, C.c_void_p]),
    "mi_sim_set_mirror": (C.c_int, [C.c_void_p] + [C.c_void_p] * 6),
    "mi_get_state_mirror": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mi_sim_step": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p]),
    "mi_sim_flush": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mi_task_configure": (C.c_int, [C.c_void_p, C.POINTER(MiTaskParams)]),
    "mi_task_pre_step": (C.c_int, [C.c_void_p] + [C.c_void_p] * 7),
    "mi_task_reset_idx": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32] + [C.c_void_p] * 5),
    "mi_task_post_step": (C.c_int, [C.c_void_p] + [C.c_void_p] * 8),
    "mi_task_post_kernel": (C.c_int, [C.c_void_p, _i32p, _i32p]),
    "mi_task_observations": (C.c_int, [C.c_void_p] + [C.c_void_p] * 5),
    "mi_task_metrics": (C.c_int, [C.c_void_p] + [C.c_void_p] * 6),
    "mi_task_is_done": (C.c_int, [C.c_void_p] + [C.c_void_p] * 4),
    "mi_env_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32] + [C.c_void_p] * 11),
    "mi_sim_time_launches": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "mi_sim_launch_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, _i32p]),
    "mi_task_set_dr": (C.c_int, [C.c_void_p, C.POINTER(MiDrParams)]),
    "mi_dr_apply_actions": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mi_dr_apply_observations": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mi_get_dr_state": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mi_fill_uniform": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_uint64, C.c_uint64,
                                  C.c_float, C.c_float, C.c_void_p]),
    "mi_get_reset_count": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mi_set_reset_count": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mi_sim_pair_load": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]),
    "mi_sim_nan_count": (C.c_int, [C.c_void_p, _i64p]),
    "mi_sim_kernel_path": (C.c_int, [C.c_void_p, _i32p, _i32p, _i32p]),
    "mi_abi_version": (C.c_int, []),
    "mi_build_id": (C.c_char_p, []),
    "mi_last_error": (C.c_char_p, []),
}

EXPORTED_SYMBOLS = tuple(_SIGS)


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libmi_sim.so and declare every prototype of include/mi_sim.h (no GPU needed)."""
    if not os.path.exists(path):
        raise NativeUnavailable(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        lib = C.CDLL(path)
    except OSError as e:  # pragma: no cover - depends on the box
        raise NativeUnavailable(f"failed to load {path}: {e}") from e
    # a library named by MI_SIM_LIB (an A/B build of other sources) may predate entry points
    # added since; the shipped library must export every one (tests/test_host.py)
    lenient = "MI_SIM_LIB" in os.environ and path == LIB_PATH
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if lenient and name == "mi_build_id":
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    return lib


def lib() -> C.CDLL:
    """The loaded HIP library; raises NativeUnavailable (no fallback) if unusable."""
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


def check(rc: int, what: str = "") -> None:
    if rc != MI_OK:
        msg = lib().mi_last_error()
        raise RuntimeError(f"{what or 'mi_sim'} failed ({rc}): {msg.decode() if msg else ''}")


def ptr(t) -> Optional[int]:
    """Device pointer of a torch tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()
