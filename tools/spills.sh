#!/bin/bash
# where a build spills: scratch stores / loads of one env-step kernel per source line (line
# tables on): KERNEL=RobotAnt|RobotHumanoid [KNAME=k_env_step_pair] tools/spills.sh [extra hipcc flags...]
D=$(mktemp -d)
K=${KERNEL:-RobotHumanoid}
cd "$D" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -fno-slp-vectorize -Wno-unused-function \
  -Wno-unused-variable ${SPILL_FLAGS:-} -gline-tables-only "$@" -save-temps /root/repo/omniisaacgymenvs_amd/csrc/mi_sim.hip -o t.so 2>&1 | grep -i " error"
S=mi_sim-hip-amdgcn-amd-amdhsa-gfx950.s
start=$(grep -n "^_Z[0-9]*${KNAME:-k_env_step_wave}IN2mi6TopoCTINS0_[0-9]*${K}.*:" $S | cut -d: -f1)
len=$(tail -n +$start $S | grep -n "^\s*\.end_amdhsa_kernel\|^\.Lfunc_end" | head -1 | cut -d: -f1)
sed -n "${start},$((start+len))p" $S | awk '/^\t\.loc\t/{i=index($0,"; "); if(i){x=substr($0,i+2); split(x,a," "); n=split(a[1],p,"/"); split(p[n],q,":"); line=q[1]":"q[2]}} /scratch_store/{st[line]++} /scratch_load/{ld[line]++} END{for(k in st) print "store", k, st[k]; for(k in ld) print "load", k, ld[k]}' | sort -k3 -n -r | head -${TOP:-25}
rm -rf "$D"
