#!/usr/bin/env python3
"""Rollout policy step timing (the learner's half of a rollout step):
mi_rl_policy_step (rlg/ops.py FusedPolicy) against the torch statement (the modules + the
sampling kernel), both captured in HIP graphs of 32 steps (a rollout horizon), replayed.
Prints one JSON line. MI_RL_LIB selects another build of libmi_rl.so for A/B.

usage: python tools/policy_bench.py [--task Humanoid] [--rows 4096] [--reps 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omniisaacgymenvs_amd.rlg import ops  # noqa: E402
from omniisaacgymenvs_amd.rlg.models import ModelA2CContinuousLogStd  # noqa: E402

NETS = {"Humanoid": (87, 21, [400, 200, 100]), "Ant": (60, 8, [256, 128, 64]), "Cartpole": (4, 1, [32, 32])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Humanoid")
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    O, A, units = NETS[a.task]
    cfg = {"mlp": {"units": units, "activation": "elu"},
           "space": {"continuous": {"fixed_sigma": True, "sigma_init": {"val": 0.0}}}}
    torch.manual_seed(0)
    m = ModelA2CContinuousLogStd(O, A, cfg, True, True).cuda().eval()
    fp = ops.FusedPolicy(m)
    R, H = a.rows, 32
    obs = torch.randn((R, O), device="cuda")
    cnt = torch.zeros((1,), dtype=torch.int64, device="cuda")
    outs = [torch.empty((H, R, w), device="cuda") for w in (O, A, 1, 1, A, A)]

    def fused():
        fp.pack()
        for n in range(H):
            fp.step(obs, 3, cnt, n, *(o[n] for o in outs))

    def torch_path():
        with torch.no_grad():
            for n in range(H):
                mu, logstd, v = m.policy(obs)
                act, nlp = ops.sample_gauss(mu, m.a2c_network.sigma.detach(), 3, cnt, n)
                outs[0][n].copy_(obs)
                outs[1][n].copy_(act)
                outs[2][n].copy_(nlp.unsqueeze(-1))
                outs[3][n].copy_(m.unnorm_value(v))
                outs[4][n].copy_(mu)
                outs[5][n].copy_(torch.exp(logstd))

    res = {"task": a.task, "rows": R, "horizon": H}
    for name, fn in (("fused", fused), ("torch", torch_path)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        res[f"{name}_us_per_step"] = round(s.elapsed_time(e) * 1e3 / (a.reps * H), 2)
    # MFMA work per step: 2 * rows * sum(in * out) over the layers and heads
    dims = [O] + units
    flops = 2 * R * (sum(dims[i] * dims[i + 1] for i in range(len(units))) + units[-1] * (A + 1))
    res["gflop_per_step"] = round(flops / 1e9, 4)
    res["fused_tflops"] = round(flops / (res["fused_us_per_step"] * 1e-6) / 1e12, 2)
    res["peak_tflops_f32_mfma"] = 157.3
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
