"""The data-parallel learner (multi_gpu: True, multi_gpu_mode data_parallel — rl_games'
multi_gpu, cfg/train/HumanoidPPO.yaml:43) at world size 2 on ONE GPU: two processes, each with
its own Humanoid env shard on cuda:0, a gloo process group (gloo takes CUDA tensors), the
rollout AND the per-minibatch update captured as HIP graphs (graph_rollout / graph_update), the
gradient all-reduce issued between the two captured halves of every minibatch.

Run for 3 epochs, so epochs 2-3 replay the captured update graphs: after every epoch both
replicas' parameters, optimizer state and normalisation statistics must be bit-identical, both
ranks must follow one adaptive-LR sequence, and the shards must have stepped different envs.
(the graphed data-parallel path had never run above world size 1.)"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_ENVS, EPOCHS, WORLD = 256, 3, 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
        from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
        from omniisaacgymenvs_amd.utils.task_util import make_env

        env = make_env("Humanoid", num_envs=N_ENVS, device="cuda:0", seed=42,
                       env_id_offset=rank * N_ENVS, global_num_envs=world * N_ENVS,
                       overrides=[f"train.params.config.minibatch_size={N_ENVS * 8}"])
        register_env(f"rlgpu_dpw{rank}", lambda **kw: env)
        params = env.task_cfg["train"]["params"]
        cfg = params["config"]
        cfg.update(multi_gpu=True, multi_gpu_mode="data_parallel", graph_rollout=True,
                   graph_update=True, save_frequency=0, save_best_after=10 ** 9)
        agent = A2CAgent(RLGPUEnv(f"rlgpu_dpw{rank}", N_ENVS), params, run_dir=f"/tmp/dpw_{port}_{rank}")
        res = {"dp": agent.dp, "world": agent.world, "minibatches": agent.num_minibatches,
               "equal": [], "lrs": [], "graphs": 0, "obs_differ": None}
        agent.env_reset()

        def state():
            parts = [t.detach().double().reshape(-1) for t in agent.model.state_dict().values()]
            for st in agent.optimizer.state.values():
                parts += [v.detach().double().reshape(-1) for v in st.values() if torch.is_tensor(v)]
            return torch.cat(parts)

        for _ in range(EPOCHS):
            agent.train_epoch()
            s = state()
            allst = [torch.empty_like(s) for _ in range(world)]
            dist.all_gather(allst, s)
            res["equal"].append(all(torch.equal(allst[0], x) for x in allst[1:]))
            res["lrs"].append(agent.last_lr)
        res["graphs"] = len(agent.upd_graphs)
        o = agent.buf["obses"][-1].contiguous()
        allo = [torch.empty_like(o) for _ in range(world)]
        dist.all_gather(allo, o)
        res["obs_differ"] = not torch.equal(allo[0], allo[1])
        res["finite"] = bool(torch.isfinite(state()).all())
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()
        env.close()
        q.put((rank, res))
    except Exception as e:          # noqa: BLE001 - report, do not hang the parent
        import traceback
        q.put((rank, {"error": f"{e!r}\n{traceback.format_exc()}"}))


def test_data_parallel_graphed_world2_replicas_identical(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=240) for _ in range(WORLD))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(WORLD):
        assert "error" not in out[r], out[r].get("error")
    for r in range(WORLD):
        res = out[r]
        assert res["dp"] and res["world"] == WORLD and res["minibatches"] == 4
        assert res["graphs"] > 0                          # the update ran from captured graphs
        assert all(res["equal"]), res["equal"]            # bit-identical replicas every epoch
        assert res["finite"] and res["obs_differ"]        # distinct shards, sane training state
    assert out[0]["lrs"] == out[1]["lrs"]                  # one adaptive LR sequence


def _overflow_worker(rank, world, port, q):
    """an f16-range overflow of a Linear gradient on ONE rank must make BOTH
    replicas skip the step (the reference's f16 gradient is inf before the all-reduce)."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
        from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
        from omniisaacgymenvs_amd.utils.task_util import make_env

        env = make_env("Humanoid", num_envs=N_ENVS, device="cuda:0", seed=42,
                       env_id_offset=rank * N_ENVS, global_num_envs=world * N_ENVS,
                       overrides=[f"train.params.config.minibatch_size={N_ENVS * 8}"])
        register_env(f"rlgpu_dpo{rank}", lambda **kw: env)
        params = env.task_cfg["train"]["params"]
        params["config"].update(multi_gpu=True, multi_gpu_mode="data_parallel", graph_rollout=True,
                                graph_update=False, save_frequency=0, save_best_after=10 ** 9)
        agent = A2CAgent(RLGPUEnv(f"rlgpu_dpo{rank}", N_ENVS), params, run_dir=f"/tmp/dpo_{port}_{rank}")
        assert agent.dp and agent._f16_begin is not None and agent.fused_opt is not None
        agent.env_reset()
        idx = agent._f16_begin + 5
        inject_at = 2 * agent.num_minibatches * agent.mini_epochs - 3   # a late minibatch of epoch 2
        calls = {"n": 0}
        rec = []
        orig_mask, orig_apply = agent._f16_overflow_to_inf, agent._mb_apply

        def mask():
            if calls["n"] == inject_at:
                rec.append(("rank0_small_entry", float(agent._flat[idx].abs())))
                if rank == 1:
                    agent._flat[idx] = 1.0e5     # over f16 range here, under it once averaged
            orig_mask()

        def apply(i):
            before = int(agent.fused_opt.tickets[1])
            orig_apply(i)
            torch.cuda.synchronize()
            if calls["n"] == inject_at:
                rec.append(("delta", int(agent.fused_opt.tickets[1]) - before))
                rec.append(("index", int(agent.fused_opt.tickets[2])))
            calls["n"] += 1

        agent._f16_overflow_to_inf, agent._mb_apply = mask, apply
        for _ in range(2):
            agent.train_epoch()
        res = {"rec": rec, "idx": idx, "calls": calls["n"], "inject_at": inject_at}
        dist.barrier()
        dist.destroy_process_group()
        env.close()
        q.put((rank, res))
    except Exception as e:          # noqa: BLE001 - report, do not hang the parent
        import traceback
        q.put((rank, {"error": f"{e!r}\n{traceback.format_exc()}"}))


def test_data_parallel_f16_overflow_on_one_rank_skips_everywhere(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=240) for _ in range(WORLD))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(WORLD):
        assert "error" not in out[r], out[r].get("error")
    for r in range(WORLD):
        res = out[r]
        assert res["calls"] > res["inject_at"], res
        rec = dict(res["rec"])
        if r == 0:   # rank 0's own gradient is in range: the skip can only come from rank 1
            assert rec["rank0_small_entry"] < 65520.0, rec
        assert rec["delta"] == 1, (r, rec)              # the step was skipped on this replica
        assert rec["index"] == res["idx"], (r, rec)     # ... for the injected entry
