#!/bin/bash
# kernel ms of several libmi_sim builds (LIBS="a.so b.so ..."), Humanoid and Ant fused step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in $LIBS; do
  for T in ${TASKS:-Humanoid Ant}; do
    MI_SIM_LIB=$PWD/omniisaacgymenvs_amd/$L timeout -k 10 100 python -u bench.py --task $T --no-side --no-cpu-baseline --fuse-envs 0 --steps 300 --warmup 30 > gpurun_out/var_${L}_$T.log 2>&1 || exit 1
    echo "$L $T $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/var_${L}_$T.log)"
  done
done
echo ALL_DONE
