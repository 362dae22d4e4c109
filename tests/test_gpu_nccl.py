"""Config 5's code path on one GPU: an in-process world-size-1 NCCL (= RCCL on ROCm) process group
(FileStore rendezvous: no launcher, no re-exec), driving

  * bench.py's own ShardLoop + RolloutGather(mode="gather") over the fused Humanoid step for 40
    steps (one full 32-step horizon gathered asynchronously while the next one steps, then the
    partial horizon flushed at the window's end): the gathered slab rows must equal, bit for bit,
    what a twin env (same seed, same actions, no gather) returns from each step;
  * one A2CAgent epoch with ``multi_gpu: True`` (horizon gather + bootstrap-tail gather + episode
    all-reduce + weight broadcast over RCCL): the learner's dataset must equal its own rollout and
    the update must equal the same agent run without the process group.

Reference anchors: cfg/train/HumanoidPPO.yaml:43 (multi_gpu), :66 (horizon_length 32);
SURVEY §8(e). The 8-GPU run itself is the driver's (SCALE); this is the same code at world 1.
"""
import math
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

N_ENVS, STEPS, HORIZON = 4096, 40, 32


@pytest.fixture
def nccl_group(gpu, tmp_path):
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg_store", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        assert dist.get_backend() == "nccl"
        yield
    finally:
        dist.destroy_process_group()


def test_shard_loop_rccl_gather_equals_twin_env(nccl_group):
    import bench
    from omniisaacgymenvs_amd.utils.distributed import RolloutGather
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env("Humanoid", num_envs=N_ENVS, device="cuda:0", seed=42, env_id_offset=0,
                   global_num_envs=N_ENVS)
    twin = make_env("Humanoid", num_envs=N_ENVS, device="cuda:0", seed=42)
    view = env.task.get_robot()
    O = env.task.num_observations
    actions = bench.action_pool(view, N_ENVS, env.task.num_actions, 42, "cuda:0")
    env.reset()
    twin.reset()
    g = RolloutGather(HORIZON, N_ENVS, O, "cuda:0", 1, mode="gather", dst=0)
    loop = bench.ShardLoop(env, actions, g, HORIZON)
    assert env.fused
    win = loop.window(0, STEPS, torch.cuda.synchronize, dist.barrier)
    assert win["gathers"] == 2                                   # 32 rows, then the flushed 8
    assert win["bytes"] == STEPS * g.step_bytes
    ref = []
    for k in range(STEPS):
        o, r, d, _ = twin.step(actions[k % len(actions)])
        ref.append((o["obs"].clone(), r.clone(), d.clone()))
    torch.cuda.synchronize()
    full, part = g.outs[0], g.outs[1]
    for k in range(STEPS):
        out, h = (full, k) if k < HORIZON else (part, k - HORIZON)
        assert torch.equal(out.obs[0, h], ref[k][0]), f"obs row of step {k}"
        assert torch.equal(out.rew[0, h], ref[k][1]), f"rew row of step {k}"
        assert torch.equal(out.done[0, h], ref[k][2]), f"done row of step {k}"
    # the partial gather's global view is exactly its 8 rows
    gv = g.global_view()
    assert gv.shape == (STEPS - HORIZON, N_ENVS, O + 2)
    assert torch.equal(gv[-1, :, :O], ref[-1][0])
    # the env's own obs buffer is not the slab row it returned (caller buffers: no alias)
    assert env.task.obs_buf.data_ptr() != g.slabs[1].obs[STEPS - HORIZON - 1].data_ptr()
    assert torch.equal(env.task.obs_buf, ref[-1][0])
    env.close()
    twin.close()


def _agent(n, seed, multi_gpu, tag, mode="central", graph_update=False):
    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env("Humanoid", num_envs=n, device="cuda:0", seed=seed,
                   overrides=[f"train.params.config.minibatch_size={n * 8}"])
    name = f"rlgpu_nccl_{tag}"
    register_env(name, lambda **kw: env)
    params = env.task_cfg["train"]["params"]
    params["config"]["multi_gpu"] = multi_gpu
    params["config"]["multi_gpu_mode"] = mode
    params["config"]["graph_rollout"] = False
    params["config"]["graph_update"] = graph_update
    params["config"]["save_frequency"] = 0
    params["config"]["save_best_after"] = 10 ** 9
    params["seed"] = seed
    return env, A2CAgent(RLGPUEnv(name, n), params, run_dir=f"/tmp/nccl_{tag}")


def test_multi_gpu_learner_epoch_over_rccl(nccl_group):
    """HumanoidPPO with multi_gpu: True at world 1: the rollout crosses RCCL (gather), the update
    runs on the gathered horizon, the weights are broadcast back; same result as without."""
    from omniisaacgymenvs_amd.rlg.a2c_continuous import swap_and_flatten01

    n = 512
    env_m, ag_m = _agent(n, 3, True, "mg")
    assert ag_m.distributed and ag_m.world == 1 and ag_m.rollout is not None
    assert "done" not in ag_m.rollout.slabs[0].views          # the learner keeps its own f32 dones
    env_s, ag_s = _agent(n, 3, False, "sg")
    assert not ag_s.distributed
    ag_m.env_reset(); ag_s.env_reset()
    st_m = ag_m.train_epoch()
    st_s = ag_s.train_epoch()
    torch.cuda.synchronize()
    assert ag_m.rollout.gathers == 1
    assert torch.equal(ag_m._data["obs"], swap_and_flatten01(ag_m.buf["obses"]))
    assert torch.equal(ag_m._data["obs"], ag_s._data["obs"])
    assert torch.equal(ag_m._data["actions"], ag_s._data["actions"])
    assert st_m["frames"] == st_s["frames"] == 32 * n
    for k in ("a_loss", "c_loss", "kl"):
        assert abs(st_m[k] - st_s[k]) <= 1e-5 * max(1.0, abs(st_s[k])), (k, st_m[k], st_s[k])
    for (k, a), b in zip(ag_m.model.state_dict().items(), ag_s.model.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=k)
    env_m.close(); env_s.close()


@pytest.mark.parametrize("graphed", [False, True])
def test_data_parallel_learner_over_rccl(nccl_group, graphed):
    """multi_gpu_mode data_parallel (rl_games' multi_gpu) at world 1 over RCCL: per minibatch the
    gradients + KL go through one all-reduce between the two captured halves of the update (or
    eagerly), the obs / value statistics merge through all-reduces; the result equals the single
    learner's (cfg/train/HumanoidPPO.yaml:43)."""
    n = 512
    epochs = 2 if graphed else 1          # updates are captured from epoch 2 on (rollouts from epoch 3)
    env_m, ag_m = _agent(n, 5, True, f"dp{int(graphed)}", mode="data_parallel", graph_update=graphed)
    env_s, ag_s = _agent(n, 5, False, f"dps{int(graphed)}", graph_update=graphed)
    assert ag_m.dp and not ag_m.central and ag_m.rollout is None and ag_m.is_learner
    assert ag_m.batch_size == ag_s.batch_size == 32 * n
    ag_m.env_reset(); ag_s.env_reset()
    for _ in range(epochs):
        st_m = ag_m.train_epoch()
        st_s = ag_s.train_epoch()
    torch.cuda.synchronize()
    if graphed:
        assert all(isinstance(g, tuple) for g in ag_m.upd_graphs.values()) and ag_m.upd_graphs
    # eager: the same launches (all-reduce of one rank is the identity); graphed: the BLAS may
    # pick other kernels under stream capture (GEMM rounding, as test_graph_update_matches_eager)
    rel = 1e-3 if graphed else 1e-5
    for k in ("a_loss", "c_loss", "kl"):
        assert math.isclose(st_m[k], st_s[k], rel_tol=rel, abs_tol=1e-6), (k, st_m[k], st_s[k])
    assert st_m["lr"] == st_s["lr"]
    for (k, a), b in zip(ag_m.model.state_dict().items(), ag_s.model.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=k)
    env_m.close(); env_s.close()
