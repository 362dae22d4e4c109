"""Multi-GPU PPO on CPU (world_size-2 gloo), both learner modes of rlg.a2c_continuous with
multi_gpu: True (cfg/train/*PPO.yaml `multi_gpu`):
  * central: each rank steps its own env shard with a policy replica, the horizon is gathered to
    the learner (rank 0) in one collective, the learner trains on every rank's actors and
    broadcasts the weights back ("single RCCL gather ... for the rollout buffer");
  * data_parallel (rl_games' multi_gpu, the default): every rank updates on its own shard, the
    gradients and the KL are averaged by one all-reduce per minibatch, the normalisation
    statistics merge the ranks' moments — replicas stay identical, and the averaged gradient is
    the gradient of one learner on the union of the ranks' minibatches.
The env is the product's CPU-pipeline Cartpole, one shard per rank (global env ids)."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_cartpole_cpu_rollout import N_ENVS

EPOCHS = 2


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from tests.test_cartpole_cpu_rollout import cartpole_cpu_env
    from tests.test_rl_cpu import _cartpole_cpu_params

    register_env(f"rlgpu_mg{rank}", lambda **kw: cartpole_cpu_env(seed=100, rank=rank, world=world))
    params = _cartpole_cpu_params()
    params["config"]["multi_gpu"] = True
    params["config"]["multi_gpu_mode"] = "central"
    agent = A2CAgent(RLGPUEnv(f"rlgpu_mg{rank}", N_ENVS), params, run_dir=f"/tmp/mg_{port}_{rank}")
    res = {"world": agent.world, "batch": agent.batch_size, "minibatches": agent.num_minibatches}
    agent.env_reset()
    for _ in range(EPOCHS):
        st = agent.train_epoch()
        # this rank's local horizon as it sat in the gathered slab (learner: compared below)
        local = {k: agent.buf[k].clone() for k in ("obses", "actions", "neglogpacs", "rewards", "dones")}
        gathered = {k: [torch.empty_like(v) for _ in range(world)] for k, v in local.items()}
        for k, v in local.items():
            dist.all_gather(gathered[k], v)
        if rank == 0:
            data = agent._data
            H, N = agent.horizon, agent.num_actors
            want = {k: torch.cat(gathered[k], dim=1) for k in gathered}   # [H, world * N, ...]

            def flat(x):   # swap_and_flatten01: actor-major rows
                return x.transpose(0, 1).reshape((H * world * N,) + tuple(x.shape[2:]))
            assert torch.equal(data["obs"], flat(want["obses"]))
            assert torch.equal(data["actions"], flat(want["actions"]))
            assert torch.equal(data["old_logp_actions"], flat(want["neglogpacs"]))
    state = torch.cat([t.detach().float().reshape(-1) for t in agent.model.state_dict().values()])
    allst = [torch.empty_like(state) for _ in range(world)]
    dist.all_gather(allst, state)
    res["replicas_equal"] = all(torch.equal(allst[0], x) for x in allst[1:])
    res["games"] = st["games"]
    res["frames"] = st["frames"]
    # distinct exploration noise per rank: the two shards' action rows differ
    res["noise_differs"] = not torch.equal(gathered["actions"][0], gathered["actions"][1])
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_central_learner():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        res = out[r]
        assert res["world"] == 2
        assert res["batch"] == 16 * N_ENVS * world          # the learner's batch: both shards
        assert res["minibatches"] == 2 * 4                  # minibatch 64: twice the single-rank count
        assert res["replicas_equal"]                         # weights broadcast after every update
        assert res["frames"] == EPOCHS * res["batch"]
        assert res["noise_differs"]
    assert out[0]["games"] == out[1]["games"]               # episode statistics summed over ranks
    assert np.isfinite(out[0]["games"])


def _state(agent):
    return torch.cat([t.detach().double().reshape(-1) for t in agent.model.state_dict().values()])


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from tests.test_cartpole_cpu_rollout import cartpole_cpu_env
    from tests.test_rl_cpu import _cartpole_cpu_params

    register_env(f"rlgpu_dp{rank}", lambda **kw: cartpole_cpu_env(seed=200, rank=rank, world=world))
    params = _cartpole_cpu_params()
    params["config"]["multi_gpu"] = True          # multi_gpu_mode defaults to data_parallel
    agent = A2CAgent(RLGPUEnv(f"rlgpu_dp{rank}", N_ENVS), params, run_dir=f"/tmp/dp_{port}_{rank}")
    res = {"world": agent.world, "dp": agent.dp, "batch": agent.batch_size,
           "minibatches": agent.num_minibatches, "equal_after_epoch": [], "lrs": []}
    agent.env_reset()
    for _ in range(EPOCHS):
        st = agent.train_epoch()
        s = _state(agent)
        allst = [torch.empty_like(s) for _ in range(world)]
        dist.all_gather(allst, s)
        res["equal_after_epoch"].append(all(torch.equal(allst[0], x) for x in allst[1:]))
        res["lrs"].append(agent.last_lr)
    # one learner on the union batch: the average of the ranks' minibatch-0 gradients equals the
    # gradient of the union of their minibatch-0 rows (statistics frozen for the comparison)
    agent.model.train()
    agent.model.running_mean_std.eval()
    mb = {k: v[:agent.minibatch_size].clone() for k, v in agent._data.items()}
    agent.calc_gradients(mb, step=False)
    g_local = torch.cat([p.grad.reshape(-1) for p in agent._params])
    g_all = [torch.empty_like(g_local) for _ in range(world)]
    dist.all_gather(g_all, g_local)
    union = {}
    for k, v in mb.items():
        parts = [torch.empty_like(v) for _ in range(world)]
        dist.all_gather(parts, v.contiguous())
        union[k] = torch.cat(parts)
    agent.calc_gradients(union, step=False)
    g_union = torch.cat([p.grad.reshape(-1) for p in agent._params])
    res["grad_err"] = float((torch.stack(g_all).mean(0) - g_union).abs().max())
    res["grad_mag"] = float(g_union.abs().max())
    res["games"] = st["games"]
    res["frames"] = st["frames"]
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_data_parallel_learner():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        res = out[r]
        assert res["world"] == 2 and res["dp"]
        assert res["batch"] == 16 * N_ENVS                 # per-rank batch (rl_games multi_gpu)
        assert res["minibatches"] == 4                     # as a single rank
        assert all(res["equal_after_epoch"])                # identical replicas after every update
        assert res["frames"] == EPOCHS * res["batch"] * 2       # whole-job frames (both shards)
        assert res["grad_err"] <= 1e-5 * max(1.0, res["grad_mag"]), (res["grad_err"], res["grad_mag"])
    assert out[0]["lrs"] == out[1]["lrs"]                  # one adaptive LR (averaged KL)
    assert out[0]["games"] == out[1]["games"]              # episode statistics all-reduced
