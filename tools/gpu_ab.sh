#!/bin/bash
# A/B of two libmi_sim builds: bit-level rollout comparison and kernel time (Humanoid, Ant).
# OLD=path to the baseline library (default omniisaacgymenvs_amd/libmi_sim_old.so)
source "$(dirname "$0")/gpu_lib.sh"
OLD=${OLD:-omniisaacgymenvs_amd/libmi_sim_old.so}
for T in Humanoid Ant; do
  run d_old_$T 120 env MI_SIM_LIB=$OLD python -u tools/dump_rollout.py old_$T $T
  run d_new_$T 120 python -u tools/dump_rollout.py new_$T $T
  python tools/dump_rollout.py --compare old_$T new_$T
done
for T in Humanoid Ant; do
  for L in old new; do
    if [ $L = old ]; then export MI_SIM_LIB=$OLD; else unset MI_SIM_LIB; fi
    timeout -k 10 100 python -u bench.py --task $T --no-side --no-cpu-baseline --fuse-envs 0 --steps 300 --warmup 30 > gpurun_out/ab_${L}_$T.log 2>&1 || exit 1
    echo "$L $T $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_${L}_$T.log)"
  done
done
unset MI_SIM_LIB
echo ALL_DONE
