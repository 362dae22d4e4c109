#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run st_w4 150 env MI_STAMPS_LIB=omniisaacgymenvs_amd/libmi_sim_stamps_w4.so python -u tools/phase_stamps.py Humanoid 4096
run st_w4a 150 env MI_STAMPS_LIB=omniisaacgymenvs_amd/libmi_sim_stamps_w4.so python -u tools/phase_stamps.py Ant 4096
run pytest_view 300 python -u -m pytest tests/test_gpu_view.py -x -q --timeout 120 --timeout-method thread
run ps_hum 200 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_w4.so python -u tools/parity_stats.py Humanoid 4096 4
run ps_ant 200 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_w4.so python -u tools/parity_stats.py Ant 4096 4
for f in st_w4 st_w4a; do echo "== $f"; grep -v "^\[\|Task Dev\|RL dev\|amdgpu.ids" gpurun_out/$f.log | tail -17; done
grep -h '"task"' gpurun_out/ps_hum.log gpurun_out/ps_ant.log
echo ALL_DONE
