"""Host-side logic without a GPU: config composition (the Hydra surface), SimConfig merge,
model compilation (BFS DOF order, gear table), GridCloner, the C-ABI library (loads, exports
every symbol include/mi_sim.h declares, rejects bad input, fails loudly without a GPU)."""
import ctypes as C
import os
import re

import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd import native as N
from omniisaacgymenvs_amd.robots.articulations import GridCloner
from omniisaacgymenvs_amd.robots.model import load_robot
from omniisaacgymenvs_amd.utils.config_utils.sim_config import SimConfig
from omniisaacgymenvs_amd.utils.hydra_cfg.hydra_utils import RESOLVERS, compose, resolve

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- config
def test_resolvers_match_reference_semantics():
    # utils/hydra_cfg/hydra_utils.py:36-41
    assert RESOLVERS["eq"]("GPU", "gpu") is True
    assert RESOLVERS["contains"]("cuda", "cuda:0") is True
    assert RESOLVERS["if"](True, 1, 2) == 1 and RESOLVERS["if"](False, 1, 2) == 2
    assert RESOLVERS["resolve_default"](4096, "") == 4096
    assert RESOLVERS["resolve_default"](4096, 64) == 64


def test_relative_interpolation():
    cfg = resolve({"a": 1, "b": {"c": "${..a}", "d": {"e": "${...a}", "f": "${.g}", "g": 7},
                                 "h": "${eq:${..s},'gpu'}"}, "s": "gpu"})
    assert cfg["b"]["c"] == 1 and cfg["b"]["d"]["e"] == 1 and cfg["b"]["d"]["f"] == 7
    assert cfg["b"]["h"] is True


def test_compose_defaults_and_overrides():
    c = compose(["task=Humanoid"])
    assert c["task_name"] == "Humanoid" and c["task"]["env"]["numEnvs"] == 4096
    assert c["task"]["sim"]["use_gpu_pipeline"] is True
    assert c["train"]["params"]["config"]["num_actors"] == 4096
    c = compose(["task=Ant", "num_envs=64", "task.env.episodeLength=100", "seed=9"])
    assert c["task"]["env"]["numEnvs"] == 64 and c["task"]["env"]["episodeLength"] == 100
    assert c["train"]["params"]["seed"] == 9
    c = compose([])
    assert c["task_name"] == "Cartpole" and c["task"]["env"]["numEnvs"] == 512
    assert c["task"]["env"]["clipObservations"] == 5.0


def test_sim_config_params():
    sc = SimConfig(compose(["task=Ant", "device_id=0"]))
    assert sc.config["sim_device"] == "cuda:0"
    p = sc.mi_sim_params("Ant")
    assert abs(p.dt - 0.0083) < 1e-7 and p.solver_iterations == 4
    assert p.rest_offset == 0.0 and abs(p.contact_offset - 0.02) < 1e-7
    assert p.enable_self_collisions == 0 and p.friction == 1.0
    ph = SimConfig(compose(["task=Humanoid"])).mi_sim_params("Humanoid")
    assert ph.enable_self_collisions == 1 and abs(ph.rest_offset - 0.001) < 1e-7   # default
    assert abs(ph.max_depenetration_velocity - 10.0) < 1e-6
    cpu = SimConfig(compose(["task=Cartpole", "pipeline=cpu", "sim_device=cpu"]))
    assert cpu.config["sim_device"] == "cpu"


def test_sleep_and_stabilization_are_validated_and_reported():
    """the task YAMLs enable sleeping / stabilization (Humanoid.yaml:60-61,86-87).
    The native solver does not model them (DESIGN §5 "PhysX knobs"): they are read with the
    actor overrides, range-checked as PhysX would, and reported once per process."""
    from omniisaacgymenvs_amd.utils.config_utils import sim_config as SC

    SC._warned.clear()
    sc = SimConfig(compose(["task=Humanoid"]))
    with pytest.warns(UserWarning, match="enable_sleeping"):
        sc.mi_sim_params("Humanoid")
    u = sc.unmodelled("Humanoid")
    assert u["enable_sleeping"] and u["enable_stabilization"]
    assert u["sleep_threshold"] == 0.005 and u["stabilization_threshold"] == 0.001   # :86-87
    assert u["friction_offset_threshold"] == 0.04 and u["bounce_threshold_velocity"] == 0.2
    bad = SimConfig(compose(["task=Humanoid", "task.sim.Humanoid.sleep_threshold=-0.5"]))
    with pytest.raises(ValueError, match="sleep_threshold"):
        bad.mi_sim_params("Humanoid")
    off = SimConfig(compose(["task=Ant", "task.sim.physx.enable_sleeping=False",
                             "task.sim.physx.enable_stabilization=False"])).unmodelled("Ant")
    assert not off["enable_sleeping"] and not off["enable_stabilization"]


# ---------------------------------------------------------------- models
def test_humanoid_bfs_order_matches_gear_table():
    m = load_robot("Humanoid")
    bodies = [m.body_of_link[l] for l in range(1, m.num_links)]
    # tasks/humanoid.py:82-107 comments, in order
    expect = (["lower_waist"] * 2 + ["right_upper_arm"] * 2 + ["left_upper_arm"] * 2 + ["pelvis"]
              + ["right_lower_arm", "left_lower_arm"] + ["right_thigh"] * 3 + ["left_thigh"] * 3
              + ["right_shin", "left_shin"] + ["right_foot"] * 2 + ["left_foot"] * 2)
    assert bodies == expect
    assert m.dof_names[9:12] == ["right_hip_x", "right_hip_y", "right_hip_z"]
    assert m.num_dof == 21 and m.num_sensors == 2 and m.root_free == 1
    assert np.all(m.parent[1:] < np.arange(1, m.num_links))
    assert 30.0 < m.total_mass() < 50.0


def test_ant_and_cartpole_models():
    a = load_robot("Ant")
    assert a.dof_names == ["hip_1", "hip_2", "hip_3", "hip_4", "ankle_1", "ankle_2", "ankle_3", "ankle_4"]
    assert a.num_sensors == 4 and 12 + 3 * 8 + 6 * 4 == 60
    lim = a.dof_limits()
    np.testing.assert_allclose(lim[4], np.radians([30, 100]), rtol=1e-6)
    c = load_robot("Cartpole")
    assert c.get_dof_index("cartJoint") == 0 and c.get_dof_index("poleJoint") == 1
    assert c.root_free == 0 and c.dyn_kind == N.MI_DYN_CARTPOLE


def test_grid_cloner_shards_consistently():
    g = GridCloner(5.0)
    full = g.get_clone_positions(4096)
    assert full.shape == (4096, 3) and np.all(full[:, 2] == 0)
    assert len({tuple(p) for p in full}) == 4096
    np.testing.assert_allclose(full.mean(0)[:2], 0.0, atol=2.5)
    for r in range(4):
        np.testing.assert_array_equal(g.get_clone_positions(4096, r * 1024, 1024), full[r * 1024:(r + 1) * 1024])


# ---------------------------------------------------------------- C ABI
def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "mi_sim.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(mi_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = N.load_library()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(N.EXPORTED_SYMBOLS)
    assert lib.mi_abi_version() == 4


def test_rl_library_exports_every_header_symbol():
    """libmi_rl.so exports every entry point include/mi_rl.h declares, and its MLP descriptor
    checks run on the host (no GPU)."""
    from omniisaacgymenvs_amd.rlg import ops
    txt = open(os.path.join(ROOT, "include", "mi_rl.h")).read()
    syms = sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char\*)\s+(mi_rl_\w+)\s*\(", txt, flags=re.M)))
    assert len(syms) >= 8
    lib = ops.load_library()
    for s in syms:
        assert hasattr(lib, s), s
    d = ops.MiRlMlp()
    d.num_obs, d.num_actions, d.num_hidden = 87, 21, 3
    d.units[0], d.units[1], d.units[2] = 400, 200, 100
    # padded [N16][K16] + bias per layer: 400x96, 208x400, 112x208, head 32x112
    want = 400 * 96 + 400 + 208 * 400 + 208 + 112 * 208 + 112 + 32 * 112 + 32
    assert lib.mi_rl_mlp_packed_size(C.byref(d)) == want
    d.num_hidden = 0
    assert lib.mi_rl_mlp_packed_size(C.byref(d)) == -1
    d.num_hidden, d.units[0] = 3, 600                       # wider than the kernel's 512
    assert lib.mi_rl_mlp_packed_size(C.byref(d)) == -1


def test_abi_rejects_bad_input_without_touching_a_gpu():
    lib = N.load_library()
    out = C.c_void_p()
    assert lib.mi_sim_create(None, None, 4, 0, 0, None, 0, C.byref(out)) == -1       # MI_E_NULL
    assert b"null" in lib.mi_last_error()
    m = load_robot("Ant")
    d = m.to_desc()
    p = N.MiSimParams()
    org = np.zeros((4, 3), np.float32)
    assert lib.mi_sim_create(d.ref(), C.byref(p), 0, 0, 0, org.ctypes.data, 0, C.byref(out)) == -2
    bad = m.to_desc()
    bad._keep["parent"][3] = 5
    assert lib.mi_sim_create(bad.ref(), C.byref(p), 4, 0, 0, org.ctypes.data, 0, C.byref(out)) == -4
    if not torch.cuda.is_available():
        assert lib.mi_sim_create(d.ref(), C.byref(p), 4, 0, 0, org.ctypes.data, 0, C.byref(out)) == -6
    for fn, args in [("mi_sim_step", (None, 1, None)), ("mi_env_step", (None, None, 2) + (None,) * 11),
                     ("mi_task_pre_step", (None,) * 8), ("mi_get_dof_state", (None,) * 4)]:
        assert getattr(lib, fn)(*args) == -1


def test_product_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from omniisaacgymenvs_amd.utils.task_util import make_env

    # sim_device=cpu is the reference's CPU pipeline: served for Cartpole only
    # (robots/cpu_cartpole.py), refused for the articulated robots
    with pytest.raises(N.NativeUnavailable):
        make_env("Humanoid", num_envs=8, device="cpu")
    for task in ("Cartpole", "Humanoid"):
        with pytest.raises(RuntimeError):
            make_env(task, num_envs=8, device="cuda:0")


def test_generated_topologies_up_to_date():
    """csrc/mi_topo_gen.hpp (compile-time topologies of the shipped robots) matches the assets."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "gen_topologies.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_libraries_are_built_from_this_tree():
    """The shipped .so files embed the SHA-256 of the sources they were compiled from
    (__graft_entry__.source_hash, mi_build_id / mi_rl_build_id): a stale or restored binary
    fails here (and in smoke()) instead of silently testing other code."""
    import __graft_entry__ as g
    from omniisaacgymenvs_amd.rlg import ops

    assert N.load_library().mi_build_id().decode() == g.source_hash()
    assert ops.load_library().mi_rl_build_id().decode() == g.source_hash("mi_rl.hip")
    assert g.built_id(g.LIB) == g.source_hash() and g.built_id(g.LIB_RL) == g.source_hash("mi_rl.hip")
