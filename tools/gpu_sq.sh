#!/bin/bash
# SQ counters of the fused env-step kernel (issue vs wait breakdown), one PMC pass each
source "$(dirname "$0")/gpu_lib.sh"
run sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/sq1 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0
run sq2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace -d gpurun_out/sq2 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0
run sq3 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/sq3 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0
echo ALL_DONE
