"""Scene pieces the reference takes from closed Isaac Sim packages, rebuilt over libmi_sim.so:

* :class:`GridCloner` — env-origin grid of omni.isaac.cloner (used at tasks/base/rl_task.py:92,
  124-126). Restated from its public behaviour; the closed source is absent, so the exact
  layout is unverified.
* :class:`ArticulationView` — the omni.isaac.core tensor API the tasks call
  (get_world_poses / get_velocities / get_joint_positions / get_joint_velocities /
  set_* with indices / get_dof_limits / get_dof_index / _physics_view.get_force_sensor_forces,
  call sites tasks/shared/locomotion.py:81-89,114,130-134, tasks/cartpole.py:81-82,112,
  129-130,137-138). Every getter and setter is one HIP gather / scatter kernel on torch's
  current stream; the physics state itself never leaves HBM.
* :func:`Humanoid` / :func:`Ant` / :func:`Cartpole` — robot constructors
  (robots/articulations/{humanoid,ant,cartpole}.py) returning compiled model descriptions.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import torch

from .. import native as N
from .model import CompiledModel, load_robot


class GridCloner:
    def __init__(self, spacing: float, num_per_row: int = -1):
        self._spacing = float(spacing)
        self._num_per_row = num_per_row

    def get_clone_positions(self, num_clones: int, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        """[count, 3] origins of envs first..first+count-1 of a num_clones grid."""
        count = num_clones - first if count is None else count
        per_row = self._num_per_row if self._num_per_row > 0 else int(np.sqrt(num_clones))
        num_rows = np.ceil(num_clones / per_row)
        num_cols = np.ceil(num_clones / num_rows)
        row_offset = 0.5 * self._spacing * (num_rows - 1)
        col_offset = 0.5 * self._spacing * (num_cols - 1)
        i = np.arange(first, first + count, dtype=np.float64)
        row = np.floor(i / num_cols)
        col = i - row * num_cols
        x = row_offset - row * self._spacing
        y = col * self._spacing - col_offset
        return np.stack([x, y, np.zeros_like(x)], axis=1).astype(np.float32)


def Humanoid() -> CompiledModel:
    return load_robot("Humanoid")


def Ant() -> CompiledModel:
    return load_robot("Ant")


def Cartpole() -> CompiledModel:
    return load_robot("Cartpole")


class _PhysicsView:
    """``ArticulationView._physics_view`` (omni.physics.tensors) — force sensors only."""

    def __init__(self, view: "ArticulationView"):
        self._view = view

    def get_force_sensor_forces(self) -> torch.Tensor:
        """[count, S, 6] sensor wrenches: the view's state mirror (omni.physics.tensors hands out
        its own buffer as well; locomotion.py:89 only reads it before the next step)."""
        v = self._view
        v._refresh_mirror()
        return v._mir_sens


class ArticulationView:
    """One articulation replicated over ``count`` envs, backed by one mi_sim handle."""

    def __init__(self, model: CompiledModel, name: str = "view", prim_paths_expr: str = "",
                 reset_xform_properties: bool = False):
        self.model = model
        self.name = name
        self.prim_paths_expr = prim_paths_expr
        self.handle = None
        self.count = 0
        self.device = None
        self._desc = None
        self._physics_view = _PhysicsView(self)

    # ---- lifecycle (called by Scene.add / World) ----
    def initialize(self, sim_params: "N.MiSimParams", num_envs: int, env_origins: np.ndarray,
                   device: str, seed: int, env_id_offset: int = 0) -> None:
        dev = torch.device(device)
        if dev.type != "cuda":
            raise N.NativeUnavailable(
                f"sim_device={device!r}: libmi_sim.so runs on the GPU only (no CPU fallback; the "
                f"CPU pipeline, robots/cpu_cartpole.py, serves the Cartpole task alone)")
        lib = N.lib()
        self.device = dev
        self.count = int(num_envs)
        self.sim_params = sim_params
        self._desc = self.model.to_desc()
        origins = np.ascontiguousarray(env_origins, dtype=np.float32).reshape(self.count, 3)
        h = C.c_void_p()
        dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
        N.check(lib.mi_sim_create(self._desc.ref(), C.byref(sim_params), self.count,
                                  int(env_id_offset), int(dev_index),
                                  origins.ctypes.data, int(seed), C.byref(h)), "mi_sim_create")
        self.handle = h.value
        self.env_origins = origins
        # hot-path bindings (resolved once: the ArticulationView calls are per env-step)
        self._lib = lib
        self._dev_index = int(dev_index)
        self._raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        # state mirrors (include/mi_sim.h mi_sim_set_mirror): the tensors the getters hand out
        n, D, S = self.count, self.num_dof, self.num_sensors
        f32 = dict(dtype=torch.float32, device=dev)
        self._mir_pos, self._mir_rot = torch.zeros((n, 3), **f32), torch.zeros((n, 4), **f32)
        self._mir_vel = torch.zeros((n, 6), **f32)
        self._mir_q, self._mir_qd = torch.zeros((n, D), **f32), torch.zeros((n, D), **f32)
        self._mir_sens = torch.zeros((n, S, 6), **f32)
        N.check(lib.mi_sim_set_mirror(self.handle, self._mir_pos.data_ptr(), self._mir_rot.data_ptr(),
                                      self._mir_vel.data_ptr(), self._mir_q.data_ptr(),
                                      self._mir_qd.data_ptr(),
                                      self._mir_sens.data_ptr() if S else None), "mi_sim_set_mirror")

    def close(self) -> None:
        if self.handle:
            N.lib().mi_sim_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self) -> int:
        if self._raw_stream is not None:
            return self._raw_stream(self._dev_index)
        return torch.cuda.current_stream(self.device).cuda_stream

    # ---- sizes ----
    @property
    def num_dof(self) -> int:
        return self.model.num_dof

    @property
    def num_sensors(self) -> int:
        return self.model.num_sensors

    @property
    def dof_names(self):
        return list(self.model.dof_names)

    def get_dof_index(self, name: str) -> int:
        return self.model.get_dof_index(name)

    def get_dof_limits(self) -> torch.Tensor:
        lim = torch.from_numpy(self.model.dof_limits())
        return lim.unsqueeze(0).repeat(self.count, 1, 1).to(self.device)

    # ---- getters ----
    # Getters hand out the view's state mirrors (row-major copies the library refreshes in ONE
    # launch after the state changed, include/mi_sim.h mi_get_state_mirror): with clone=False the
    # mirror itself, which the next physics step overwrites — Isaac's clone=False returns its
    # internal buffer the same way (locomotion.py:81-88 reads them before stepping again); with
    # clone=True (the default) a copy. Contract (include/mi_sim.h): a clone=False result, and
    # get_force_sensor_forces', is read-only — an in-place edit would persist into later getters
    # until the state changes (the reference only reads them, locomotion.py:81-89). A read on
    # another stream than the refresh's is ordered after it by the library (event wait).
    def _empty(self, *shape) -> torch.Tensor:
        return torch.empty(shape, dtype=torch.float32, device=self.device)

    def _refresh_mirror(self) -> None:
        rc = self._lib.mi_get_state_mirror(self.handle, self.stream())
        if rc:
            N.check(rc, "mi_get_state_mirror")

    @staticmethod
    def _out(t: torch.Tensor, indices, clone: bool) -> torch.Tensor:
        if indices is not None:
            return t[indices.long()]
        return t.clone() if clone else t

    def get_world_poses(self, indices=None, clone: bool = True):
        self._refresh_mirror()
        return self._out(self._mir_pos, indices, clone), self._out(self._mir_rot, indices, clone)

    def get_velocities(self, indices=None, clone: bool = True) -> torch.Tensor:
        self._refresh_mirror()
        return self._out(self._mir_vel, indices, clone)

    def get_joint_positions(self, indices=None, clone: bool = True) -> torch.Tensor:
        self._refresh_mirror()
        return self._out(self._mir_q, indices, clone)

    def get_joint_velocities(self, indices=None, clone: bool = True) -> torch.Tensor:
        self._refresh_mirror()
        return self._out(self._mir_qd, indices, clone)

    # ---- setters (indices: env ids, rows of the value tensors align with them) ----
    @staticmethod
    def _f32(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        if t is None:
            return None
        if t.dtype is torch.float32 and t.is_contiguous():
            return t
        return t.to(torch.float32).contiguous()

    def _idx(self, indices, dtype) -> (Optional[torch.Tensor], int):
        if indices is None:
            return None, self.count
        if (isinstance(indices, torch.Tensor) and indices.dtype is dtype and indices.is_cuda
                and indices.get_device() == self._dev_index and indices.is_contiguous()):
            return indices, indices.numel()
        idx = torch.as_tensor(indices, device=self.device).to(dtype).contiguous()
        return idx, int(idx.numel())

    def _state_idx(self, indices) -> (Optional[torch.Tensor], int, bool):
        """(ids, count, int32?) for the state setters: int64 device ids (locomotion.py:130-134)
        and int32 ones (cartpole.py:129-130) pass as they are (the library takes both:
        mi_set_*_state / mi_set_*_state_i32), anything else becomes int64 ids."""
        if indices is None:
            return None, self.count, False
        if (isinstance(indices, torch.Tensor) and indices.is_cuda and indices.get_device() == self._dev_index
                and indices.is_contiguous()):
            if indices.dtype is torch.int32:
                return indices, indices.numel(), True
            if indices.dtype is torch.int64:
                return indices, indices.numel(), False
        idx = torch.as_tensor(indices, device=self.device).to(torch.int64).contiguous()
        return idx, int(idx.numel()), False

    def set_joint_efforts(self, efforts: torch.Tensor, indices=None) -> None:
        e = self._f32(efforts)
        idx, n = self._idx(indices, torch.int32)
        if n == 0:              # empty index list: nothing to write
            return
        rc = self._lib.mi_set_dof_efforts(self.handle, e.data_ptr(), None if idx is None else idx.data_ptr(),
                                          n, self.stream())
        if rc:
            N.check(rc, "mi_set_dof_efforts")

    def _set_dof_state(self, q, qd, indices) -> None:
        idx, n, i32 = self._state_idx(indices)
        if n == 0:              # empty index list: nothing to write
            return
        fn = self._lib.mi_set_dof_state_i32 if i32 else self._lib.mi_set_dof_state
        rc = fn(self.handle, N.ptr(q), N.ptr(qd), None if idx is None else idx.data_ptr(), n, self.stream())
        if rc:
            N.check(rc, "mi_set_dof_state")

    def _set_root_state(self, pos, quat, vel, indices) -> None:
        idx, n, i32 = self._state_idx(indices)
        if n == 0:              # empty index list: nothing to write
            return
        fn = self._lib.mi_set_root_state_i32 if i32 else self._lib.mi_set_root_state
        rc = fn(self.handle, N.ptr(pos), N.ptr(quat), N.ptr(vel), None if idx is None else idx.data_ptr(), n,
                self.stream())
        if rc:
            N.check(rc, "mi_set_root_state")

    def set_joint_positions(self, positions: torch.Tensor, indices=None) -> None:
        self._set_dof_state(self._f32(positions), None, indices)

    def set_joint_velocities(self, velocities: torch.Tensor, indices=None) -> None:
        self._set_dof_state(None, self._f32(velocities), indices)

    def set_world_poses(self, positions=None, orientations=None, indices=None) -> None:
        self._set_root_state(self._f32(positions), self._f32(orientations), None, indices)

    def set_velocities(self, velocities: torch.Tensor, indices=None) -> None:
        self._set_root_state(None, None, self._f32(velocities), indices)

    # ---- physics ----
    def sim_step(self, substeps: int = 1) -> None:
        N.check(N.lib().mi_sim_step(self.handle, int(substeps), self.stream()), "mi_sim_step")

    def sim_kernel_path(self) -> tuple:
        """(path, topology, lds_bytes): path 1 = wavefront-per-env kernel, 0 = one lane per
        env; topology = compile-time topology id (0: runtime tables); LDS bytes per env."""
        p, t, b = C.c_int32(), C.c_int32(), C.c_int32()
        N.check(N.lib().mi_sim_kernel_path(self.handle, C.byref(p), C.byref(t), C.byref(b)),
                "mi_sim_kernel_path")
        return int(p.value), int(t.value), int(b.value)

    POST_KERNELS = {0: "k_loco_post_tiled<64s>", 1: "k_loco_post_tiled<64d>", 2: "k_loco_post_tiled<32s>",
                    3: "k_loco_post_tiled<32d>", 4: "k_loco_post_pipe", 5: "k_post_step",
                    6: "k_loco_post_pipe<16>"}

    def post_kernel(self) -> tuple:
        """(kernel name, grid) of the last mi_task_post_step launch (None before the first)."""
        k, g = C.c_int32(), C.c_int32()
        N.check(N.lib().mi_task_post_kernel(self.handle, C.byref(k), C.byref(g)), "mi_task_post_kernel")
        return self.POST_KERNELS.get(int(k.value)), int(g.value)

    def sim_topology(self) -> int:
        return self.sim_kernel_path()[1]

    def nan_count(self) -> int:
        c = C.c_int64()
        N.check(N.lib().mi_sim_nan_count(self.handle, C.byref(c)), "mi_sim_nan_count")
        return int(c.value)
