"""Launch timing through the C ABI (mi_sim_time_launches / mi_sim_launch_times, include/mi_sim.h):
the measurement bench.py's roofline and tools/fuse_roofline.py use. A timed launch is the same
kernel with a HIP event pair on its own dispatch, so its outputs must be bit-identical to an
untimed launch; launches into a capturing stream are not timed."""
import ctypes as C

import pytest
import torch

from omniisaacgymenvs_amd import native as N
from omniisaacgymenvs_amd.utils.task_util import make_env

pytestmark = pytest.mark.gpu


def _times(view, cap):
    buf = (C.c_float * cap)()
    n = C.c_int32(0)
    N.check(N.lib().mi_sim_launch_times(view.handle, buf, cap, C.byref(n)), "mi_sim_launch_times")
    return n.value, list(buf[:min(n.value, cap)])


@pytest.mark.parametrize("name", ["Humanoid", "Cartpole"])
def test_timed_launches_match_untimed(gpu, name):
    envs = [make_env(name, num_envs=512, device="cuda:0", seed=21) for _ in range(2)]
    acts = torch.rand((6, 512, envs[0].task.num_actions), device="cuda:0") * 2 - 1
    for e in envs:
        e.reset()
    view = envs[1].task.get_robot()
    N.check(N.lib().mi_sim_time_launches(view.handle, 2, 8), "mi_sim_time_launches")
    for k in range(6):
        o0 = envs[0].step(acts[k])
        o1 = envs[1].step(acts[k])
        for a, b in zip((o0[0]["obs"], o0[1], o0[2]), (o1[0]["obs"], o1[1], o1[2])):
            assert torch.equal(a, b)
    n, ms = _times(view, 8)
    assert n == 3                                   # launches 0, 2, 4 of six, every = 2
    assert all(0.0 < x < 50.0 for x in ms), ms
    N.check(N.lib().mi_sim_time_launches(view.handle, 0, 0), "mi_sim_time_launches")
    envs[1].step(acts[0])
    assert _times(view, 8)[0] == 0                  # timing off: nothing recorded
    for e in envs:
        e.close()


def test_post_step_timed_and_capture_untimed(gpu):
    env = make_env("Humanoid", num_envs=4096, device="cuda:0", seed=4)
    t = env.task
    env.reset()
    view = t.get_robot()
    h, s = view.handle, view.stream()
    args = (h, t.actions.data_ptr(), t.obs_buf.data_ptr(), t.rew_buf.data_ptr(), t.reset_buf.data_ptr(),
            t.progress_buf.data_ptr(), t.potentials.data_ptr(), t.prev_potentials.data_ptr(), s)
    N.check(N.lib().mi_sim_time_launches(h, 1, 4), "mi_sim_time_launches")
    N.check(N.lib().mi_task_post_step(*args), "mi_task_post_step")
    n, ms = _times(view, 4)
    assert n == 1 and 0.0 < ms[0] < 50.0
    # a step captured into a HIP graph is not timed (its dispatch cannot carry the events)
    N.check(N.lib().mi_sim_time_launches(h, 0, 0), "mi_sim_time_launches")
    a = torch.zeros((4096, t.num_actions), device="cuda:0")
    env.step(a)
    torch.cuda.synchronize()
    N.check(N.lib().mi_sim_time_launches(h, 1, 4), "mi_sim_time_launches")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        env.step(a)
    assert _times(view, 4)[0] == 0
    g.replay()
    torch.cuda.synchronize()
    N.check(N.lib().mi_sim_time_launches(h, 0, 0), "mi_sim_time_launches")
    env.close()
