#!/bin/bash
# instruction-cache counters: current vs old library
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side"
for v in libmi_sim libmi_sim_old libmi_sim_v6; do
  run ${v}_ic 300 env MI_SIM_LIB=omniisaacgymenvs_amd/$v.so rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/${v}_ic -o run -- $B
done
echo ALL_DONE
