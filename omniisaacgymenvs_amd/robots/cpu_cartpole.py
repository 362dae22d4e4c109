"""The reference's CPU pipeline for Cartpole (BASELINE config 1: "Cartpole 16 envs, 1-DOF
analytic dynamics on CPU torch"): an :class:`ArticulationView` whose state lives in CPU torch
tensors and whose ``World.step`` is the analytic cart-pole as torch ops.

The reference selects it with ``pipeline: 'cpu'`` / ``sim_device: 'cpu'``
(cfg/config.yaml:20-23); PhysX then steps on the host and the task's torch ops run on CPU
tensors (tasks/cartpole.py:80-162). This build serves exactly that configuration: the Cartpole
task on CPU torch. It is selected only by an explicit ``sim_device=cpu`` / ``pipeline=cpu``,
never as a stand-in for a missing GPU or HIP library (a ``cuda`` device without
libmi_sim.so still raises :class:`NativeUnavailable`), and it serves only the cart-pole: the
articulated robots have no CPU pipeline here (:meth:`ArticulationView.initialize` refuses them).

Physics: the 2-DOF cart-pole of libmi_sim.so's ``k_env_step`` (mass matrix
[[m_c + m_p, m_p l cos th], [m_p l cos th, I_p + m_p l^2]], joint damping, gravity on the pole,
semi-implicit Euler with the sim dt, efforts held over the substeps), in the same float32
operation order as the device kernel, so both pipelines agree to the rounding of sin / cos.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import native as N
from .model import CompiledModel


class CpuCartpoleView:
    """ArticulationView tensor API (get/set joint state, efforts, dof limits / index) over CPU
    torch tensors for the analytic cart-pole model."""

    def __init__(self, model: CompiledModel, name: str = "view", prim_paths_expr: str = "",
                 reset_xform_properties: bool = False):
        if model.dyn_kind != N.MI_DYN_CARTPOLE:
            raise N.NativeUnavailable("the CPU pipeline serves the analytic cart-pole only; "
                                      "articulated robots need sim_device=cuda (libmi_sim.so)")
        self.model = model
        self.name = name
        self.prim_paths_expr = prim_paths_expr
        self.count = 0
        self.device = torch.device("cpu")

    # ---- lifecycle (called by Scene.add / World) ----
    def initialize(self, sim_params: "N.MiSimParams", num_envs: int, env_origins: np.ndarray,
                   device: str, seed: int, env_id_offset: int = 0) -> None:
        if torch.device(device).type != "cpu":
            raise ValueError(f"CpuCartpoleView on device {device!r}")
        cp = self.model.cartpole
        f = np.float32
        self.count = int(num_envs)
        self.sim_params = sim_params
        self.env_origins = np.ascontiguousarray(env_origins, dtype=np.float32).reshape(self.count, 3)
        self.seed = int(seed)
        self.env_ids = torch.arange(env_id_offset, env_id_offset + self.count, dtype=torch.int64)
        # float32 constants, combined in the kernel's order (mp*l, mp*l*l, mp*g*l)
        mc, mp, l = f(cp["cart_mass"]), f(cp["pole_mass"]), f(cp["pole_com"])
        g = f(-sim_params.gravity[2])
        m11, m22 = f(mc + mp), f(f(cp["pole_inertia"]) + f(mp * l) * l)
        self._m11, self._m22, self._m11m22 = float(m11), float(m22), float(f(m11 * m22))
        self._mpl = float(mp * l)
        self._mgl = float(f(mp * g) * l)
        self._cd, self._pd = float(f(cp["cart_damping"])), float(f(cp["pole_damping"]))
        self._dt = float(f(sim_params.dt))
        D = self.num_dof
        self._q = torch.zeros((self.count, D), dtype=torch.float32)
        self._qd = torch.zeros((self.count, D), dtype=torch.float32)
        self._eff = torch.zeros((self.count, D), dtype=torch.float32)
        self._nan = torch.zeros(self.count, dtype=torch.bool)
        self._nan_total = 0
        # per-env reset counter: the Philox counter of the reset draws (the device's DevState)
        self.reset_count = torch.zeros(self.count, dtype=torch.int64)

    def close(self) -> None:
        pass

    # ---- sizes ----
    @property
    def num_dof(self) -> int:
        return self.model.num_dof

    @property
    def num_sensors(self) -> int:
        return 0

    @property
    def dof_names(self):
        return list(self.model.dof_names)

    def get_dof_index(self, name: str) -> int:
        return self.model.get_dof_index(name)

    def get_dof_limits(self) -> torch.Tensor:
        lim = torch.from_numpy(self.model.dof_limits())
        return lim.unsqueeze(0).repeat(self.count, 1, 1)

    # ---- getters (clone=False hands out the view's own buffer, as Isaac's does) ----
    @staticmethod
    def _out(t: torch.Tensor, indices, clone: bool) -> torch.Tensor:
        if indices is not None:
            return t[torch.as_tensor(indices).long()]
        return t.clone() if clone else t

    def get_joint_positions(self, indices=None, clone: bool = True) -> torch.Tensor:
        return self._out(self._q, indices, clone)

    def get_joint_velocities(self, indices=None, clone: bool = True) -> torch.Tensor:
        return self._out(self._qd, indices, clone)

    def get_joint_efforts(self, indices=None, clone: bool = True) -> torch.Tensor:
        return self._out(self._eff, indices, clone)

    # ---- setters (indices: env ids; rows of the value tensor align with them) ----
    def _rows(self, dst: torch.Tensor, src: torch.Tensor, indices) -> None:
        src = torch.as_tensor(src).to(torch.float32)
        if indices is None:
            dst.copy_(src.reshape(dst.shape))
        else:
            idx = torch.as_tensor(indices).long()
            if idx.numel():
                dst[idx] = src.reshape(idx.numel(), dst.shape[1])

    def set_joint_efforts(self, efforts: torch.Tensor, indices=None) -> None:
        self._rows(self._eff, efforts, indices)

    def set_joint_positions(self, positions: torch.Tensor, indices=None) -> None:
        self._rows(self._q, positions, indices)

    def set_joint_velocities(self, velocities: torch.Tensor, indices=None) -> None:
        self._rows(self._qd, velocities, indices)

    # ---- physics: World.step ----
    def sim_step(self, substeps: int = 1) -> None:
        dt = self._dt
        for _ in range(int(substeps)):
            x, th = self._q[:, 0], self._q[:, 1]
            xd, thd = self._qd[:, 0], self._qd[:, 1]
            s, c = torch.sin(th), torch.cos(th)
            m12 = self._mpl * c
            r1 = self._eff[:, 0] + self._mpl * s * thd * thd - self._cd * xd
            r2 = self._eff[:, 1] + self._mgl * s - self._pd * thd
            det = self._m11m22 - m12 * m12
            xdd = (self._m22 * r1 - m12 * r2) / det
            thdd = (self._m11 * r2 - m12 * r1) / det
            xd = xd + dt * xdd
            thd = thd + dt * thdd
            # in place: clone=False getters hand out these buffers
            self._q.copy_(torch.stack([x + dt * xd, th + dt * thd], dim=1))
            self._qd.copy_(torch.stack([xd, thd], dim=1))
        # NaN guard (the device's per-env flag): a non-finite state forces a reset
        self._nan |= ~torch.isfinite(self._q).all(1) | ~torch.isfinite(self._qd).all(1)

    def take_nan_flags(self) -> torch.Tensor:
        """Envs whose state went non-finite since the last call (then cleared)."""
        f = self._nan
        self._nan = torch.zeros_like(f)
        self._nan_total += int(f.sum())
        return f

    def sim_kernel_path(self) -> tuple:
        return (-1, 0, 0)

    def nan_count(self) -> int:
        return self._nan_total
