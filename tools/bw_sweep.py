#!/usr/bin/env python3
"""SURVEY §8(d) bandwidth sweep: the fused env step at N = 2^12 .. 2^20 envs on one GPU, each
N in its own bench.py process (bounded steps). Prints one JSON line per N and writes
gpurun_out/bw_sweep.json: env-steps/s, kernel ms, algorithmic GB/s and its HBM fraction."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "Humanoid"
    sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        [4096, 16384, 65536, 262144, 1048576]
    out = []
    for n in sizes:
        steps = max(10, min(200, (200 * 4096) // n))
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--task", task, "--num-envs", str(n),
               "--steps", str(steps), "--warmup", "5", "--no-cpu-baseline", "--no-side", "--fuse-envs", "0"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not line:
            print(json.dumps({"num_envs": n, "error": r.stderr[-400:]}), flush=True)
            break
        d = json.loads(line[-1])
        rec = {"task": task, "num_envs": n, "steps": steps, "env_steps_per_s": d["value"],
               "kernel_ms": d["roofline"]["kernel_ms"], "achieved_GBps": d["roofline"]["achieved"],
               "hbm_frac": d["roofline"]["frac"]}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"bw_sweep_{task.lower()}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
