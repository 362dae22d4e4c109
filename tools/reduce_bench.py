#!/usr/bin/env python3
"""Per-minibatch reductions of the learner's backward (rlg/models.py _LinearSplitK): the bias
gradient gy.sum(0) over the 32768 minibatch rows and the split-K weight-gradient sum over the
32 row blocks, fp16 as under autocast, timed in graphs of 20 calls for each way of forming them.
Prints JSON lines (us per call). Informs the choice in _LinearSplitK.backward."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (5 * reps)


def main():
    K, S = 32768, 32
    dt = torch.float16
    for out in (1, 21, 100):
        gy = torch.randn((K, out), device="cuda", dtype=dt)
        ones_s = torch.ones((S, 1, K // S), device="cuda", dtype=dt)
        print(json.dumps({"out": out, "bias_sum0_f32acc": round(timed(lambda: gy.sum(0, dtype=torch.float32)), 2),
                          "bias_splitk_bmm_f32": round(timed(lambda: torch.bmm(ones_s, gy.reshape(S, K // S, out)).sum(0, dtype=torch.float32)), 2)}),
              flush=True)
    for out, inn in ((400, 87), (200, 400), (100, 200), (22, 100)):
        gy = torch.randn((K, out), device="cuda", dtype=dt)
        x = torch.randn((K, inn), device="cuda", dtype=dt)
        ones = torch.ones((1, K), device="cuda", dtype=dt)
        ones_s = torch.ones((S, 1, K // S), device="cuda", dtype=dt)
        part = torch.randn((S, out, inn), device="cuda", dtype=dt)
        res = {"out": out, "in": inn}
        res["bias_sum0"] = timed(lambda: gy.sum(0))
        res["bias_sum0_f32acc"] = timed(lambda: gy.sum(0, dtype=torch.float32))
        res["bias_ones_mm"] = timed(lambda: ones @ gy)
        res["bias_splitk_bmm"] = timed(lambda: torch.bmm(ones_s, gy.reshape(S, K // S, out)).sum(0))
        res["w_bmm"] = timed(lambda: torch.bmm(gy.reshape(S, K // S, out).transpose(1, 2), x.reshape(S, K // S, inn)))
        res["w_sum0"] = timed(lambda: part.sum(0))
        res["w_sum0_f32acc"] = timed(lambda: part.sum(0, dtype=torch.float32))
        res["w_single_gemm"] = timed(lambda: gy.t() @ x)
        f32 = torch.float32
        res["w_splitk_bmm_sum_f32"] = timed(lambda: torch.bmm(gy.reshape(S, K // S, out).transpose(1, 2),
                                                              x.reshape(S, K // S, inn)).sum(0, dtype=f32))
        res["b_splitk_bmm_sum_f32"] = timed(lambda: torch.bmm(ones_s, gy.reshape(S, K // S, out)).sum(0, dtype=f32))
        try:   # one GEMM with f32 output (aten::mm.dtype): no split-K partials, no reduction launch
            res["w_mm_out_f32"] = timed(lambda: torch.mm(gy.t(), x, out_dtype=f32))
            res["b_mm_out_f32"] = timed(lambda: torch.mm(ones, gy, out_dtype=f32))
        except Exception as e:   # noqa: BLE001 - report the op's absence
            res["mm_out_f32_error"] = f"{type(e).__name__}: {str(e)[:120]}"
        xa = torch.cat([x, torch.ones((K, 1), device="cuda", dtype=dt)], 1)
        res["w_bias_fused_bmm"] = timed(lambda: torch.bmm(gy.reshape(S, K // S, out).transpose(1, 2),
                                                          xa.reshape(S, K // S, inn + 1)).sum(0))
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
