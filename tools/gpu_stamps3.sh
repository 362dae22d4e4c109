#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run st_new 150 python -u tools/phase_stamps.py Humanoid 4096
run st_old 150 env MI_STAMPS_LIB=omniisaacgymenvs_amd/libmi_sim_stamps_old.so python -u tools/phase_stamps.py Humanoid 4096
run sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/sq1 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side
run sq2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace -d gpurun_out/sq2 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side
for f in st_new st_old; do echo "== $f"; grep -v "^\[\|Task Dev\|RL dev\|amdgpu.ids" gpurun_out/$f.log | tail -17; done
echo ALL_DONE
