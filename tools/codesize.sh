#!/bin/bash
# instruction count of the Humanoid env-step kernel per source phase (line tables):
# tools/codesize.sh [extra hipcc flags...]
D=$(mktemp -d)
cd "$D" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -fno-slp-vectorize -Wno-unused-function \
  -Wno-unused-variable -gline-tables-only "$@" -save-temps /root/repo/omniisaacgymenvs_amd/csrc/mi_sim.hip -o t.so 2>&1 | grep -i " error"
S=mi_sim-hip-amdgcn-amd-amdhsa-gfx950.s
start=$(grep -n "^_Z15k_env_step_waveIN2mi6TopoCTINS0_13RobotHumanoid.*:" $S | cut -d: -f1)
end=$(grep -n "^_Z15k_env_step_waveIN2mi6TopoCTINS0_8RobotAnt.*:" $S | cut -d: -f1)
sed -n "${start},${end}p" $S | awk '/^\t\.loc\t/{i=index($0,"; "); if(i){x=substr($0,i+2); split(x,a," "); n=split(a[1],p,"/"); split(p[n],q,":"); line=q[1]":"q[2]}; next} /^\t[a-z_]+[0-9a-z_]* /{c[line]++} END{for(k in c) print c[k], k}' > /tmp/codesize_lines.txt
rm -rf "$D"
python3 - <<'PY'
import re, collections
src = open('/root/repo/omniisaacgymenvs_amd/csrc/mi_wave.hpp').read().split('\n')
marks = [(i + 1, l.strip()[:58]) for i, l in enumerate(src) if re.search(r'// ---- P|^MI_D |^template|^__device__', l)]
def region(line):
    cur = 'top'
    for i, l in marks:
        if i <= line: cur = f"{i}: {l}"
    return cur
agg = collections.Counter()
tot = 0
for ln in open('/tmp/codesize_lines.txt'):
    n, loc = ln.split()
    n = int(n); tot += n
    f, l = loc.split(':') if ':' in loc else (loc, '0')
    agg[region(int(l)) if f == 'mi_wave.hpp' else f] += n
for k, v in agg.most_common(30): print(f"{v:6d} {100*v/tot:5.1f}%  {k}")
print("total instructions", tot)
PY
