#!/bin/bash
# SQ counters of the obs/reward fuse kernel (k_loco_post_tiled, Humanoid 1 M envs), one PMC pass each
source "$(dirname "$0")/gpu_lib.sh"
RP="rocprofv3 --output-format csv"
CMD="python3 tools/fuse_roofline.py Humanoid 1048576 10"
run fsq1 120 $RP --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/fsq1 -o run -- $CMD
run fsq2 120 $RP --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace -d gpurun_out/fsq2 -o run -- $CMD
run fsq3 120 $RP --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/fsq3 -o run -- $CMD
run fpf 120 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/fpf -o run -- $CMD
run fpw 120 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/fpw -o run -- $CMD
echo ALL_DONE
