#!/bin/bash
# one-resident-round experiment: Ant with LDS capped to 16 envs/CU, at 2 and 4 waves/SIMD
source "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline --fuse-envs 0 --no-side"
run ant_base 120 $B --task Ant
run ant_caps 120 env MI_WAVE_JROWS=16 MI_WAVE_WROWS=29 $B --task Ant
run ant_w4caps 120 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_w4.so MI_WAVE_JROWS=16 MI_WAVE_WROWS=29 $B --task Ant
run ant_w4 120 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_w4.so $B --task Ant
run hum_w4 120 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_w4.so $B
for f in ant_base ant_caps ant_w4caps ant_w4 hum_w4; do echo $f; grep -o '"lds_bytes_per_env": [0-9]*\|"kernel_ms": [0-9.]*' gpurun_out/$f.log; done
echo ALL_DONE
