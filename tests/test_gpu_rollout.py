"""GPU: the zero-copy rollout path. VecEnvRLGames.step(actions, out=RolloutGather.slot(h)) — the
fused launch writing obs / rew / done straight into the slab row the RCCL gather sends — must
equal the default step (fresh tensors) bit for bit, and the world-size-1 gather must hand the
slab back unchanged."""
import pytest
import torch

from omniisaacgymenvs_amd.utils.distributed import RolloutGather
from omniisaacgymenvs_amd.utils.task_util import make_env
from tests.helpers import rand_actions

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["Cartpole", "Ant", "Humanoid"])
def test_step_into_rollout_slab_equals_default_step(gpu, name):
    n, H = 96, 4
    ea = make_env(name, num_envs=n, device="cuda:0", seed=5)
    eb = make_env(name, num_envs=n, device="cuda:0", seed=5)
    g = RolloutGather(H, n, ea.num_observations, "cuda:0", 1)
    ref = []
    for hz in range(2):
        for h in range(H):
            acts = rand_actions(n, ea.num_actions, 10 * hz + h).to("cuda:0")
            ea.step(acts, out=g.slot(h))
            ob, rb, db, _ = eb.step(acts)
            ref.append((ob["obs"].clone(), rb.clone(), db.clone()))
        out = g.gather(async_op=True)
        g.wait()
        torch.cuda.synchronize()
        for h in range(H):
            o, r, d = ref[hz * H + h]
            assert torch.equal(out.obs[0, h], o)
            assert torch.equal(out.rew[0, h], r)
            assert torch.equal(out.done[0, h], d)
    with pytest.raises(ValueError):
        ea.step(acts, out=(g.slot(0)[0][:, :-1], g.slot(0)[1], g.slot(0)[2]))
    ea.close()
    eb.close()
