#!/bin/bash
# SQ / PMC counters of the obs/reward fuse at 1 M Humanoid envs, one PMC pass each, for the
# pipelined kernel (default) and the one-tile kernel (MI_POST_TILE=32s)
source "$(dirname "$0")/gpu_lib.sh"
RP="rocprofv3 --output-format csv"
CMD="python3 tools/fuse_roofline.py Humanoid 1048576 10"
for V in ${VARS:-32p 32s}; do
  export MI_POST_TILE=$V
  run fsq1_$V 120 $RP --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/fsq1_$V -o run -- $CMD
  run fsq2_$V 120 $RP --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace -d gpurun_out/fsq2_$V -o run -- $CMD
  run fsq3_$V 120 $RP --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/fsq3_$V -o run -- $CMD
  run fpf_$V 120 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/fpf_$V -o run -- $CMD
  run fpw_$V 120 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/fpw_$V -o run -- $CMD
done
echo ALL_DONE
