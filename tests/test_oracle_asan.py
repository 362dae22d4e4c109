"""The CPU oracle under AddressSanitizer + UBSan ("compile the CPU restatement with
-fsanitize=address,undefined"). `make -C oracle asan` links oracle.c into a standalone
executable (oracle/asan_driver.c); this test writes one scenario per task — model description,
sim / task parameters, origins, a reset step plus seeded U(-1.2, 1.2) actions (the ±1 clamp,
resets, contacts, Humanoid self-collision and the task math all run) — runs it with the
sanitizers set to abort on the first finding, and checks the outputs against liboracle.so bit
for bit (the same C built -O1 vs -O2, FP contraction off in both)."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from omniisaacgymenvs_amd.robots.articulations import GridCloner
from oracle.oracle import OracleSim, make_buffers
from tests.helpers import task_params_from_cfg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "oracle", "_asan", "asan_driver")
N_ENVS, STEPS, SEED = 16, 24, 42


def _sim_params(task):
    from omniisaacgymenvs_amd.utils.config_utils.sim_config import SimConfig
    from omniisaacgymenvs_amd.utils.hydra_cfg.hydra_utils import compose

    cfg = compose([f"task={task}", f"num_envs={N_ENVS}", "pipeline=cpu", "sim_device=cpu", "rl_device=cpu"])
    return SimConfig(cfg).mi_sim_params(task), float(cfg["task"]["env"]["envSpacing"])


def _scenario(path, task, actions):
    tp, m, keep = task_params_from_cfg(task)
    sp, spacing = _sim_params(task)
    origins = GridCloner(spacing).get_clone_positions(N_ENVS, 0, N_ENVS).astype(np.float32)
    A, D = tp.num_actions, m.num_dof
    if keep is None:   # cartpole: no locomotion arrays
        keep = (np.zeros(A, np.float32), np.zeros(A, np.float32), np.zeros(D, np.float32))
    f32 = lambda a: np.ascontiguousarray(a, np.float32).tobytes()
    i32 = lambda a: np.ascontiguousarray(a, np.int32).tobytes()
    cp = m.cartpole
    with open(path, "wb") as f:
        f.write(i32([m.dyn_kind, m.root_free, m.num_links, m.num_geoms, m.num_sensors, m.pairs.shape[0]]))
        f.write(i32(m.parent) + i32(m.jtype))
        for a in (m.axis, m.pos, m.quat, m.mass, m.com, m.inertia, m.lower, m.upper, m.damping, m.armature):
            f.write(f32(a))
        f.write(i32(m.geom_link) + i32(m.geom_type) + f32(m.geom_p0) + f32(m.geom_p1) + f32(m.geom_radius))
        f.write(i32(m.sensor_link) + f32(m.sensor_pos) + i32(m.pairs))
        f.write(f32([cp.get(k, 0.0) for k in ("cart_mass", "pole_mass", "pole_com", "pole_inertia",
                                                "cart_damping", "pole_damping")]))
        f.write(bytes(sp))
        f.write(bytes(tp))
        f.write(f32(keep[0]) + f32(keep[1]) + f32(keep[2]))
        f.write(i32([N_ENVS]) + np.uint64(SEED).tobytes() + f32(origins))
        f.write(i32([STEPS, 2, A, tp.num_obs]) + f32(actions))
    return tp, m, sp, origins


def _reference_run(tp, m, sp, origins, actions):
    orc = OracleSim(m, sp, N_ENVS, origins, seed=SEED)
    orc.configure(tp, keep=getattr(tp, "_keep", None))
    b = make_buffers(N_ENVS, tp.num_obs, tp.num_actions)
    b["reset"][:] = 1
    for k in range(STEPS):
        orc.env_step(actions[k], 2, b)
    orc.close()
    return b


@pytest.fixture(scope="module")
def driver():
    if shutil.which(os.environ.get("CC", "gcc")) is None:
        pytest.skip("no C compiler")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    return DRIVER


@pytest.mark.parametrize("task", ["Cartpole", "Ant", "Humanoid"])
def test_oracle_clean_under_asan_ubsan(driver, task, tmp_path):
    tp0, _, _ = task_params_from_cfg(task)
    rng = np.random.default_rng(7)
    actions = rng.uniform(-1.2, 1.2, (STEPS, N_ENVS, tp0.num_actions)).astype(np.float32)
    actions[0] = 0.0
    scen, out = str(tmp_path / "scenario.bin"), str(tmp_path / "out.bin")
    tp, m, sp, origins = _scenario(scen, task, actions)
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="1")
    r = subprocess.run([driver, scen, out], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"{task}: sanitizer / driver failure\n{r.stderr[-4000:]}"
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    O = tp.num_obs
    raw = open(out, "rb").read()
    obs = np.frombuffer(raw, np.float32, N_ENVS * O).reshape(N_ENVS, O)
    rew = np.frombuffer(raw, np.float32, N_ENVS, 4 * N_ENVS * O)
    reset = np.frombuffer(raw, np.int64, N_ENVS, 4 * N_ENVS * (O + 1))
    progress = np.frombuffer(raw, np.int64, N_ENVS, 4 * N_ENVS * (O + 1) + 8 * N_ENVS)
    b = _reference_run(tp, m, sp, origins, actions)
    np.testing.assert_array_equal(obs, b["obs"])
    np.testing.assert_array_equal(rew, b["rew"])
    np.testing.assert_array_equal(reset, b["reset"])
    np.testing.assert_array_equal(progress, b["progress"])
    assert np.isfinite(obs).all()
