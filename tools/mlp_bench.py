#!/usr/bin/env python3
"""Kernel time of the fused training MLP (mi_rl_mlp_train_fwd / _bwd) at a minibatch of 32768
rows, Humanoid layout: median of HIP-event-timed launches. usage: mlp_bench.py [rows]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from omniisaacgymenvs_amd.rlg import ops
    from omniisaacgymenvs_amd.rlg.models import ModelA2CContinuousLogStd

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    torch.manual_seed(0)
    cfg = {"mlp": {"units": [400, 200, 100], "activation": "elu"},
           "space": {"continuous": {"fixed_sigma": True, "sigma_init": {"val": 0.0}}}}
    m = ModelA2CContinuousLogStd(87, 21, cfg, True, True).cuda()
    net = m.a2c_network
    flat = ops.flatten_parameters(net.parameters())
    net.shadow_weights(torch.float16, flat)
    f = net._train_mlp
    x = torch.randn((rows, 87), device="cuda")
    gmu = (torch.randn((rows, 21), device="cuda") * 1e-2).half()
    gv = (torch.randn((rows, 1), device="cuda") * 1e-2).half()
    f.pack()
    out = {}
    for what in ("pack", "fwd", "bwd"):
        ts = []
        for k in range(60):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if what == "bwd":
                mu, v, acts = f.forward(x)
            e0.record()
            if what == "pack":
                f.pack()
            elif what == "fwd":
                f.forward(x)
            else:
                f.backward(acts, gmu, gv)
            e1.record()
            torch.cuda.synchronize()
            if k >= 10:
                ts.append(e0.elapsed_time(e1) * 1e3)
        out[what + "_us"] = round(statistics.median(ts), 1)
    flops_f = 2 * rows * (87 * 400 + 400 * 200 + 200 * 100 + 100 * 22)
    flops_b = 2 * rows * (22 * 100 + 100 * 200 + 200 * 400)
    out["fwd_tflops"] = round(flops_f / out["fwd_us"] / 1e6, 1)
    out["bwd_tflops"] = round(flops_b / out["bwd_us"] / 1e6, 1)
    print(json.dumps({"rows": rows, **out}), flush=True)


if __name__ == "__main__":
    main()
