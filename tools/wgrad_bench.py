#!/usr/bin/env python3
"""Weight-gradient GEMMs of the learner's MLP (dW = dYᵀ X over K = 32768 minibatch rows, fp16):
one GEMM vs split-K as a batched GEMM + a sum over the splits. Prints one JSON line per shape."""
import json

import torch


def t_ms(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    K = 32768
    dev = "cuda:0"
    for O, I in ((400, 87), (200, 400), (100, 200), (21, 100), (1, 100)):
        dy = torch.randn((K, O), device=dev, dtype=torch.float16)
        x = torch.randn((K, I), device=dev, dtype=torch.float16)
        ref = (dy.float().t() @ x.float())
        rec = {"O": O, "I": I, "K": K, "mm_ms": round(t_ms(lambda: dy.t() @ x), 4)}
        for S in (4, 8, 16, 32):
            def split():
                return torch.bmm(dy.view(S, K // S, O).transpose(1, 2), x.view(S, K // S, I)).sum(0)
            rec[f"split{S}_ms"] = round(t_ms(split), 4)
            err = (split().float() - ref).abs().max().item() / ref.abs().max().item()
            rec[f"split{S}_relerr"] = float(f"{err:.2e}")
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
