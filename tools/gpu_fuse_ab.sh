#!/bin/bash
# obs/reward fuse A/B of two libraries (MI_SIM_LIB), Humanoid 1 M / 2 M envs, alternating passes
source "$(dirname "$0")/gpu_lib.sh"
for k in 1 2 3; do
for L in nt ntl; do
run ab_${L}_$k 200 env MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_$L.so python -u tools/fuse_roofline.py Humanoid 1048576,2097152
done
done
for f in gpurun_out/ab_*.log; do echo "$f $(grep -h '^{' $f | grep -o '"num_envs": [0-9]*\|"achieved": [0-9.]*' | tr '\n' ' ')"; done
echo ALL_DONE
