#!/bin/bash
# kernel time of library variants (Humanoid fused step)
source "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline --fuse-envs 0 --no-side"
for v in libmi_sim libmi_sim_old libmi_sim_v5 libmi_sim_v6; do
  [ -f omniisaacgymenvs_amd/$v.so ] || continue
  run $v 120 env MI_SIM_LIB=omniisaacgymenvs_amd/$v.so $B
  echo "$v $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/$v.log)"
done
run w34 120 env MI_WAVE_WROWS=34 $B
echo "w34 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/w34.log)"
run e4 120 env MI_WAVE_ENVS=4 $B
echo "e4 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/e4.log)"
echo ALL_DONE
