#!/bin/bash
# GPU tests + Humanoid / Ant bench lines (default library and the occupancy-4 build)
source "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline --fuse-envs 0 --no-side"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run hum 120 $B
run ant 120 $B --task Ant
if [ -f omniisaacgymenvs_amd/libmi_sim_w4.so ]; then
run hum_w4 120 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_w4.so $B
run ant_w4 120 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_w4.so $B --task Ant
fi
for f in hum ant hum_w4 ant_w4; do echo $f; grep -o '"lds_bytes_per_env": [0-9]*\|"kernel_ms": [0-9.]*' gpurun_out/$f.log 2>/dev/null; done
echo ALL_DONE
