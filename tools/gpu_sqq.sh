#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/sq1 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side
run sq1o 300 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_old.so rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/sq1o -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side
echo ALL_DONE
