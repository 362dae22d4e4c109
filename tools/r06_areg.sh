#!/bin/bash
# round 6: wide-PGS register rows 32 (default, 16 B of VGPR spills) vs 28 / 24 (spill-free):
# alternating bench passes, then WRITE_SIZE per variant
export TMPDIR=/tmp
L28=omniisaacgymenvs_amd/libmi_sim_areg28.so; L24=omniisaacgymenvs_amd/libmi_sim_areg24.so
TAG=areg LIBS="$L28 $L24" bash tools/gpu.sh abn || exit $?
mkdir -p gpurun_out/r06/wsize
B="python3 bench.py --task Humanoid --num-envs 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-side --fuse-envs 0"
for v in 28 24; do
  MI_SIM_LIB=omniisaacgymenvs_amd/libmi_sim_areg$v.so timeout -s KILL 90 rocprofv3 --output-format csv --pmc WRITE_SIZE --kernel-trace \
    -d gpurun_out/r06/wsize/w_areg$v -o run -- $B > gpurun_out/r06/wsize/w_areg$v.log 2>&1 || exit $?
done
