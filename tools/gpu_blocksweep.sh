#!/bin/bash
# Block-size sweep of the round-1 one-lane-per-env kernel.
source "$(dirname "$0")/gpu_lib.sh"
for T in Humanoid Ant; do
  for B in 64 32 16 8 4; do
    MI_SIM_BLOCK=$B run bench_${T}_b$B 120 python -u bench.py --task $T --steps 100 --warmup 10 --no-cpu-baseline
  done
done
echo ALL_DONE
