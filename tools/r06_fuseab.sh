#!/bin/bash
# round 6: the GPU suite on the default library, then obs/reward-fuse and env-step A/B of the
# default library against LIB_BASE (alternating passes; fuse at 1 M / 2 M Humanoid envs)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06/${ABN_TAG:-fuseab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
for k in 1 2 3; do
  for e in new:omniisaacgymenvs_amd/libmi_sim.so base:$LIB_BASE; do
    n=${e%%:*}; l=${e#*:}
    MI_SIM_LIB=$l timeout -k 10 120 python3 -u tools/fuse_roofline.py Humanoid 1048576,2097152 30 > $O/fuse_${n}_$k.log 2>&1 || exit $?
    MI_SIM_LIB=$l timeout -k 10 120 python3 -u tools/fuse_roofline.py Ant 1048576 30 > $O/fuseant_${n}_$k.log 2>&1 || exit $?
  done
done
for n in new base; do echo "fuse $n"; grep -h '"num_envs"' $O/fuse_${n}_*.log $O/fuseant_${n}_*.log | cut -c1-160; done
ABN_TAG=${ABN_TAG:-fuseab} LIBS="new:omniisaacgymenvs_amd/libmi_sim.so base:$LIB_BASE" bash tools/r06_abn.sh
