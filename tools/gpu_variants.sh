#!/bin/bash
# A/B of library variants: bench Humanoid + Ant per variant (MI_SIM_LIB)
source "$(dirname "$0")/gpu_lib.sh"
for V in "" _B _C _D; do
  L=$PWD/omniisaacgymenvs_amd/libmi_sim$V.so
  for T in Humanoid Ant; do
    MI_SIM_LIB=$L run bench_${T}$V 150 python -u bench.py --task $T --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0
  done
done
echo ALL_DONE
