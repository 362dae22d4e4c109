"""N>1 path on CPU: world_size-2 gloo job. Each rank steps its env shard (the CPU oracle stands
in for the GPU sim here — test infrastructure only) with actions from the global Philox action
stream, records its rollout slab and all-gathers it; the gathered global rollout must equal a
single-process run over all 2n envs bit for bit (shards are independent; ids are global)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from omniisaacgymenvs_amd.robots.articulations import GridCloner
from omniisaacgymenvs_amd.utils.distributed import RolloutGather, shard_range
from oracle.oracle import OracleSim, lib as orc_lib, make_buffers
from tests.helpers import sim_params, task_params_from_cfg

N_PER_RANK, H, TASK = 6, 4, "Ant"


def _actions(offset, n, A, step, seed=42):
    return np.array([[2.0 * orc_lib().orc_uniform(seed, offset + i, step, c, 1) - 1.0 for c in range(A)]
                     for i in range(n)], np.float32)


def _rollout(offset, n, total):
    tp, m, _ = task_params_from_cfg(TASK)
    origins = GridCloner(5.0).get_clone_positions(total, offset, n)
    orc = OracleSim(m, sim_params(rest_offset=0.0), n, origins, seed=42, env_id_offset=offset)
    orc.configure(tp)
    b = make_buffers(n, tp.num_obs, tp.num_actions)
    out = np.zeros((H, n, tp.num_obs + 2), np.float32)
    for h in range(H):
        orc.env_step(_actions(offset, n, tp.num_actions, h), 2, b)
        out[h, :, : tp.num_obs] = b["obs"]
        out[h, :, tp.num_obs] = b["rew"]
        out[h, :, tp.num_obs + 1] = b["reset"]
    orc.close()
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, total = shard_range(rank, world, N_PER_RANK)
    local = _rollout(off, N_PER_RANK, total)
    g = RolloutGather(H, N_PER_RANK, local.shape[2] - 2, "cpu", world)
    for h in range(H):
        g.record(h, torch.from_numpy(local[h, :, :-2]), torch.from_numpy(local[h, :, -2]),
                 torch.from_numpy(local[h, :, -1]))
    g.gather()
    if rank == 0:
        q.put(g.global_view().numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather_equals_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _rollout(0, world * N_PER_RANK, world * N_PER_RANK)
    assert got.shape == ref.shape
    np.testing.assert_array_equal(got, ref)


def _async_worker(rank, world, port, q):
    """Three horizons through the double-buffered slabs with async gathers: every gathered
    horizon must hold each rank's rows exactly, even while the next horizon is being written."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, O, Hh = 5, 3, 4
    g = RolloutGather(Hh, n, O, "cpu", world)
    got = []
    for hz in range(3):
        for h in range(Hh):
            obs, rew, done = g.slot(h)
            base = 1000 * hz + 100 * rank + 10 * h
            obs.copy_(torch.arange(n * O, dtype=torch.float32).view(n, O) + base)
            rew.fill_(base + 0.5)
            done.fill_(hz + rank)
        out = g.gather(async_op=True)
        if hz > 0:
            got.append(prev_view())
        prev = out

        def prev_view(o=prev):
            g.wait()
            return (o.obs.clone(), o.rew.clone(), o.done.clone())
    got.append(prev_view())
    if rank == 0:
        q.put([tuple(t.numpy() for t in x) for x in got])
    dist.barrier()
    dist.destroy_process_group()


def test_async_double_buffered_gather_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, O, Hh = 5, 3, 4
    assert len(got) == 3
    for hz, (obs, rew, done) in enumerate(got):
        assert obs.shape == (world, Hh, n, O)
        for r in range(world):
            for h in range(Hh):
                base = 1000 * hz + 100 * r + 10 * h
                np.testing.assert_array_equal(obs[r, h], np.arange(n * O, dtype=np.float32).reshape(n, O) + base)
                np.testing.assert_array_equal(rew[r, h], np.full(n, base + 0.5, np.float32))
                np.testing.assert_array_equal(done[r, h], np.full(n, hz + r, np.int64))
