#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run st_w4 150 env MI_STAMPS_LIB=omniisaacgymenvs_amd/libmi_sim_stamps_w4.so python -u tools/phase_stamps.py Humanoid 4096
run st_def 150 python -u tools/phase_stamps.py Humanoid 4096
run st_w4a 150 env MI_STAMPS_LIB=omniisaacgymenvs_amd/libmi_sim_stamps_w4.so python -u tools/phase_stamps.py Ant 4096
for f in st_w4 st_def st_w4a; do echo "== $f"; grep -v "^\[\|Task Dev\|RL dev\|amdgpu.ids" gpurun_out/$f.log | tail -17; done
echo ALL_DONE
