#!/bin/bash
# phase stamps: new vs old library (Humanoid, Ant)
source "$(dirname "$0")/gpu_lib.sh"
run st_new 150 python -u tools/phase_stamps.py Humanoid 4096
run st_old 150 env MI_STAMPS_LIB=omniisaacgymenvs_amd/libmi_sim_stamps_old.so python -u tools/phase_stamps.py Humanoid 4096
run st_new_ant 150 python -u tools/phase_stamps.py Ant 4096
run st_old_ant 150 env MI_STAMPS_LIB=omniisaacgymenvs_amd/libmi_sim_stamps_old.so python -u tools/phase_stamps.py Ant 4096
for f in st_new st_old st_new_ant st_old_ant; do echo "== $f"; grep -v "^{" gpurun_out/$f.log | tail -17; done
echo ALL_DONE
