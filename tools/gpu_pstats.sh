#!/bin/bash
# device-vs-oracle error distributions, old and new library
source "$(dirname "$0")/gpu_lib.sh"
run ps_old 200 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_old.so python -u tools/parity_stats.py Humanoid 4096 4
run ps_new 200 python -u tools/parity_stats.py Humanoid 4096 4
run ps_new1 200 env MI_WAVE_ENVS=1 python -u tools/parity_stats.py Humanoid 4096 4
grep -h '"task"' gpurun_out/ps_old.log gpurun_out/ps_new.log gpurun_out/ps_new1.log
echo ALL_DONE
