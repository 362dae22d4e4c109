#!/bin/bash
# bit-level comparison of two libmi_sim builds on one seeded rollout
source "$(dirname "$0")/gpu_lib.sh"
run d_old 120 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_old.so python -u tools/dump_rollout.py old
run d_new 120 python -u tools/dump_rollout.py new
run d_new1 120 env MI_WAVE_ENVS=1 python -u tools/dump_rollout.py new1
run d_ant_old 120 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_old.so python -u tools/dump_rollout.py ant_old Ant
run d_ant_new 120 python -u tools/dump_rollout.py ant_new Ant
python tools/dump_rollout.py --compare old new
python tools/dump_rollout.py --compare old new1
python tools/dump_rollout.py --compare ant_old ant_new
echo ALL_DONE
