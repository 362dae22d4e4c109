#!/bin/bash
# occupancy probe: kernel time vs envs per workgroup, kernel-trace resources, SQ wave counters
source "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --steps 100 --warmup 20 --no-cpu-baseline --fuse-envs 0 --no-side"
run e1 120 env MI_WAVE_ENVS=1 $B
run e2 120 env MI_WAVE_ENVS=2 $B
run e4 120 env MI_WAVE_ENVS=4 $B
run sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/sq1 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side
run sq3 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/sq3 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side
for f in e1 e2 e4; do echo $f; grep -o '"lds_bytes_per_env": [0-9]*\|"kernel_ms": [0-9.]*' gpurun_out/$f.log; done
echo ALL_DONE
