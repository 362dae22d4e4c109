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


def _async_worker(rank, world, port, q, mode):
    """Three horizons through the double-buffered slabs with async gathers: every gathered
    horizon must hold each rank's rows exactly, even while the next horizon is being written."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, O, Hh = 5, 3, 4
    g = RolloutGather(Hh, n, O, "cpu", world, mode=mode)
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
            if o is None:                  # gather mode, not the learner rank
                assert mode == "gather" and rank != 0
                return None
            return (o.obs.clone(), o.rew.clone(), o.done.clone())
    got.append(prev_view())
    if rank == 0:
        q.put([tuple(t.numpy() for t in x) for x in got])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["gather", "all_gather"])
def test_async_double_buffered_gather_two_ranks(mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000 + (7 if mode == "gather" else 0)
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, q, mode)) for r in range(world)]
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


class _OracleShardEnv:
    """CPU stand-in for one rank's fused VecEnvRLGames (test infrastructure: the oracle steps the
    shard): step(actions, out=(obs, rew, done)) writes the returned tensors into `out`."""
    fused = True

    def __init__(self, offset, n, total):
        tp, m, _ = task_params_from_cfg(TASK)
        origins = GridCloner(5.0).get_clone_positions(total, offset, n)
        self.orc = OracleSim(m, sim_params(rest_offset=0.0), n, origins, seed=42, env_id_offset=offset)
        self.orc.configure(tp)
        self.b = make_buffers(n, tp.num_obs, tp.num_actions)

    def step(self, actions, out=None):
        self.orc.env_step(actions.numpy(), 2, self.b)
        obs, rew, done = out
        obs.copy_(torch.from_numpy(self.b["obs"]))
        rew.copy_(torch.from_numpy(self.b["rew"]))
        done.copy_(torch.from_numpy(self.b["reset"]))
        return {"obs": obs}, rew, done, {}


STEPS_IN_WINDOW = 5


def _bench_loop_worker(rank, world, port, q):
    """bench.py's own ShardLoop with --steps 5 < horizon 32: the window must hold one complete
    gather (the partial horizon flushed at its end) whose rows are the global rollout."""
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, total = shard_range(rank, world, N_PER_RANK)
    env = _OracleShardEnv(off, N_PER_RANK, total)
    tp, _, _ = task_params_from_cfg(TASK)
    acts = [torch.from_numpy(_actions(off, N_PER_RANK, tp.num_actions, h)) for h in range(H)]
    g = RolloutGather(32, N_PER_RANK, tp.num_obs, "cpu", world, mode="gather", dst=0)
    loop = bench.ShardLoop(env, acts, g, 32)
    win = loop.window(0, STEPS_IN_WINDOW, barrier=dist.barrier)
    res = {"gathers": win["gathers"], "bytes": win["bytes"], "step_bytes": g.step_bytes}
    if rank == 0:
        res["rows"] = g.global_view().numpy().copy()
    else:
        assert g.out is None          # gather mode: only the learner holds the horizon
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_window_gathers_partial_horizon_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_bench_loop_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r]["gathers"] == 1
        assert got[r]["bytes"] == STEPS_IN_WINDOW * got[r]["step_bytes"]
    ref = _rollout(0, world * N_PER_RANK, world * N_PER_RANK)   # H = 4 steps of actions, cycled
    ref5 = np.concatenate([ref, _rollout_tail(world)], axis=0)[:STEPS_IN_WINDOW]
    np.testing.assert_array_equal(got[0]["rows"], ref5)


def _rollout_tail(world):
    """Step 5 of the single-process run (the action pool of H batches cycles: step 4 uses batch 0)."""
    tp, m, _ = task_params_from_cfg(TASK)
    n = world * N_PER_RANK
    origins = GridCloner(5.0).get_clone_positions(n, 0, n)
    orc = OracleSim(m, sim_params(rest_offset=0.0), n, origins, seed=42)
    orc.configure(tp)
    b = make_buffers(n, tp.num_obs, tp.num_actions)
    for h in range(H + 1):
        orc.env_step(_actions(0, n, tp.num_actions, h % H), 2, b)
    orc.close()
    out = np.zeros((1, n, tp.num_obs + 2), np.float32)
    out[0, :, : tp.num_obs] = b["obs"]
    out[0, :, tp.num_obs] = b["rew"]
    out[0, :, tp.num_obs + 1] = b["reset"]
    return out


def test_slab_without_done_field():
    """RolloutGather(with_done=False) (the learner's slab: its dones are f32 learner fields):
    slot() has no done, record() stores obs / rew and refuses a done it cannot hold."""
    import pytest

    from omniisaacgymenvs_amd.utils.distributed import RolloutGather

    g = RolloutGather(4, 8, 3, "cpu", 1, buffers=1, with_done=False)
    o, r, d = g.slot(1)
    assert d is None and "done" not in g.slabs[0].views
    obs = torch.arange(24, dtype=torch.float32).view(8, 3)
    rew = torch.arange(8, dtype=torch.float32)
    g.record(1, obs, rew)
    assert torch.equal(g.slabs[0].obs[1], obs) and torch.equal(g.slabs[0].rew[1], rew)
    with pytest.raises(ValueError, match="no done field"):
        g.record(2, obs, rew, torch.zeros(8, dtype=torch.int64))
    out = g.gather()
    assert torch.equal(out.obs[0, 1], obs)
