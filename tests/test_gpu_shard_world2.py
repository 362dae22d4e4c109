"""Config 5's data path at world size 2 on ONE GPU (VERDICT r5 "next" #6; SURVEY §8(e);
cfg/train/HumanoidPPO.yaml:43 multi_gpu, :66 horizon_length 32): two spawned processes, each
with its own HIP Humanoid env shard on cuda:0 (global env ids: env_id_offset = rank x n,
global_num_envs = 2n), a gloo process group over the CUDA tensors (RCCL needs one GPU per rank;
the 8-GPU RCCL run is the driver's), and bench.py's own ShardLoop + RolloutGather(mode="gather"):
the fused step writes each step into the rollout slab row, every full 32-step horizon is gathered
to rank 0 asynchronously while the next one steps, and the partial horizon is flushed at the end.

Rank 0's gathered global slab of every horizon (obs | rew | done in global env order) must equal,
bit for bit, a single-process run of one 2n-env sim with the same seed and the same global
Philox action stream: shards are independent and every per-env key is the global env id."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_PER_RANK, WORLD, HORIZON, STEPS = 1024, 2, 32, 70   # two full horizons + a flushed 6-step one


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        from omniisaacgymenvs_amd.utils.distributed import RolloutGather, shard_range
        from omniisaacgymenvs_amd.utils.task_util import make_env

        off, total = shard_range(rank, world, N_PER_RANK)
        env = make_env("Humanoid", num_envs=N_PER_RANK, device="cuda:0", seed=42, env_id_offset=off,
                       global_num_envs=total)
        view = env.task.get_robot()
        O = env.task.num_observations
        actions = bench.action_pool(view, N_PER_RANK, env.task.num_actions, 42, "cuda:0")
        env.reset()
        g = RolloutGather(HORIZON, N_PER_RANK, O, "cuda:0", world, mode="gather", dst=0)
        loop = bench.ShardLoop(env, actions, g, HORIZON)
        assert env.fused
        horizons = []
        for k in range(STEPS):
            loop.step(k)
            if loop.h == 0:                    # a full horizon was just gathered (async)
                g.wait()
                if rank == 0:
                    horizons.append(g.global_view().cpu().numpy())
        loop.flush()                           # the partial horizon
        g.wait()
        if rank == 0:
            horizons.append(g.global_view().cpu().numpy())
            np.save(os.path.join(out_dir, "gathered.npy"), np.concatenate(horizons, axis=0))
        res = {"gathers": g.gathers, "bytes": g.bytes_sent, "step_bytes": g.step_bytes, "off": off}
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()
        env.close()
        q.put((rank, res))
    except Exception as e:          # noqa: BLE001 - report, do not hang the parent
        import traceback
        q.put((rank, {"error": f"{e!r}\n{traceback.format_exc()}"}))


def test_two_hip_shards_rollout_gather_equals_single_process(gpu, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, str(tmp_path), q)) for r in range(WORLD)]
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
        assert out[r]["gathers"] == 3 and out[r]["bytes"] == STEPS * out[r]["step_bytes"]
    assert out[1]["off"] == N_PER_RANK
    got = np.load(tmp_path / "gathered.npy")
    # the single-process reference: one sim over all 2n envs, the same global action stream
    import bench
    from omniisaacgymenvs_amd.utils.task_util import make_env

    n = WORLD * N_PER_RANK
    env = make_env("Humanoid", num_envs=n, device="cuda:0", seed=42)
    view = env.task.get_robot()
    O = env.task.num_observations
    actions = bench.action_pool(view, n, env.task.num_actions, 42, "cuda:0")
    env.reset()
    ref = np.zeros((STEPS, n, O + 2), np.float32)
    for k in range(STEPS):
        o, r, d, _ = env.step(actions[k % len(actions)])
        ref[k, :, :O] = o["obs"].cpu().numpy()
        ref[k, :, O] = r.cpu().numpy()
        ref[k, :, O + 1] = d.cpu().numpy()
    env.close()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert int(ref[:, :, O + 1].sum()) > 0                     # episodes end inside the window
    for k in range(STEPS):
        assert np.array_equal(got[k], ref[k]), f"step {k}: {np.count_nonzero(got[k] != ref[k])} entries differ"
