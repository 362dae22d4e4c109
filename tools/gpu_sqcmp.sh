#!/bin/bash
# PMC comparison of two libraries on the default Humanoid bench
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side"
for v in libmi_sim libmi_sim_old; do
  run ${v}_lds 300 env MI_SIM_LIB=omniisaacgymenvs_amd/$v.so rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/${v}_lds -o run -- $B
  run ${v}_ins 300 env MI_SIM_LIB=omniisaacgymenvs_amd/$v.so rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/${v}_ins -o run -- $B
done
echo ALL_DONE
