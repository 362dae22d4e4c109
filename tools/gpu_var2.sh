#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline --fuse-envs 0 --no-side"
run cur37 120 env MI_WAVE_WROWS=37 $B
echo "cur37 $(grep -o '"kernel_ms": [0-9.]*\|"lds_bytes_per_env": [0-9]*' gpurun_out/cur37.log | tr '\n' ' ')"
run dense37 120 env MI_WAVE_WROWS=37 MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_v5.so $B
echo "dense37 $(grep -o '"kernel_ms": [0-9.]*\|"lds_bytes_per_env": [0-9]*' gpurun_out/dense37.log | tr '\n' ' ')"
run cur 120 $B
echo "cur $(grep -o '"kernel_ms": [0-9.]*\|"lds_bytes_per_env": [0-9]*' gpurun_out/cur.log | tr '\n' ' ')"
echo ALL_DONE
