#!/bin/bash
# register / scratch / occupancy of the wave kernels as compiled (VGPR + AGPR, spills):
# tools/regs.sh [extra hipcc flags...]
D=$(mktemp -d)
cd "$D" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -fno-slp-vectorize -Wno-unused-function \
  -Wno-unused-variable "$@" -save-temps "/root/repo/omniisaacgymenvs_amd/csrc/mi_sim.hip" -o t.so 2>&1 | grep -i " error"
awk '/^_Z1[0-9]k_(env|sim)_step_(wave|pair)IN2mi/{f=1;n=$1} f&&/; (NumVgprs|NumAgprs|ScratchSize|Occupancy|NumSgprs):/{s=s" "$2$3} f&&/; Occupancy:/{print substr(n,1,64), s; s=""; f=0}' mi_sim-hip-amdgcn-amd-amdhsa-gfx950.s
rm -rf "$D"
